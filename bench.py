"""Benchmark of the hot path (BASELINE.json metric: query embeddings/sec + cosine-pairs/sec,
100k x 768 gallery).

python bench.py --gpus N --steps K --warmup W [--mode full|knn] [--preset cfg2|cfg3|cfg4|cfg5]
  full (default): one step = Swin-T tower on B synthetic 224x224 images + ClinicalBERT-geometry
        tower on B synthetic 128-token reports (bf16) -> joint-embedding head (default: the
        reference's default model_type "multimodal", 5 fusion layers x 8 heads) -> exact cosine
        top-K of the query embeddings over the gallery (config 2: B=256, 100k x 768 f32, K=10).
        --model-type text: text tower + text head only (config 3's text-only ClinicalBERT queries);
        image: image tower + image head only; both: both single-modality heads (2B embeddings).
  knn:  one step = exact cosine top-K of B resident queries over the gallery (kNN leg only).
Presets (BASELINE.json configs): cfg2 = the defaults; cfg3 = --model-type text --batch 1024
  --gallery 1000000 --k 50; cfg4 = cfg2 with 1M gallery rows per GPU (8M at --gpus 8); cfg5 =
  --tower-dtype fp8 --batch 2048 --dim 1024 --gallery 1000000 --rerank: MX-fp8 linears in all BERT
  layers and Swin stages 3-4, joint_dim 1024, top-10 per query over 1M x 1024 rows per GPU, then the
  KG / label rerank (reranker.py:240-333) of those 10 candidates (batch 2048 is per GPU: weak scaling
  like the other presets).  World 1: one fused kernel (mmr_index_rerank).  World > 1: each shard
  computes its candidates' raw components (mmr_index_rerank_components), they ride with the score /
  index lists through the all-gather and the merge (mmr_merge_topk_payload), and the min-max / mix /
  rank runs on the merged list (mmr_rerank_mix) — the same result as one index.
N>1: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run, one process per GPU,
RCCL) unless it already runs under a launcher (WORLD_SIZE set, which must equal --gpus).  The
gallery is row-sharded (--gallery rows per rank: weak scaling), every rank runs its own query batch
through the towers and searches its shard for ALL ranks' queries (all-gather of query embeddings),
then the per-shard top-K lists are all-gathered over RCCL and merged.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PRESETS = {
    "cfg2": {},
    "cfg3": {"model_type": "text", "batch": 1024, "gallery": 1_000_000, "k": 50},
    "cfg4": {"gallery": 1_000_000},
    "cfg5": {"batch": 2048, "gallery": 1_000_000, "dim": 1024, "k": 10, "tower_dtype": "fp8", "rerank": True,
             "gallery_dtype": "fp16"},
}
RERANK_DK = 128  # synthetic KG embedding width of the rerank tables


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", choices=["full", "knn"], default="full")
    p.add_argument("--preset", choices=sorted(PRESETS), default="cfg2",
                   help="BASELINE.json config: cfg2 (default), cfg3 (text-only B=1024, 1M x 768, top-50), "
                        "cfg4 (1M rows per GPU), cfg5 (fp8 towers, B=2048, 1M x 1024, rerank); explicit flags "
                        "override the preset")
    p.add_argument("--tower-dtype", choices=["bf16", "fp8", "x3"], default=None,
                   help="tower linears: bf16 (configs 2-4), MX-fp8 (config 5) or x3 (fp32-faithful parity mode: f32 "
                        "activations, every contraction on bf16x3 MFMA)")
    p.add_argument("--sequential-towers", action="store_true",
                   help="run the towers and the fusion layers on one stream (for rocprof per-kernel stats; the "
                        "default overlaps the Swin tower and the patch-side fusion work on side streams)")
    p.add_argument("--no-x3-line", action="store_true",
                   help="skip the x3 (fp32-faithful) throughput + parity block reported beside a bf16 / fp8 run")
    p.add_argument("--rerank", action="store_true", default=None,
                   help="fused KG / label rerank of each query's top-K candidates inside the step")
    p.add_argument("--batch", type=int, default=None)
    p.add_argument("--knn-mode", choices=["x3", "f16"], default="f16",
                   help="gallery scan: f16 (fp16 unit-row copy, default) or x3 (bf16 split GEMM; skinny f32 "
                        "stream for Q <= 32); both exact (f64 re-rank from the f32 rows)")
    p.add_argument("--gallery", type=int, default=None, help="gallery rows per GPU")
    p.add_argument("--gallery-dtype", choices=["fp32", "fp16"], default=None,
                   help="gallery rows: fp32 (configs 1-4), or fp16 (config 5: a native fp16 index, 2 B per element "
                        "on the device, exact f64 re-score from the fp16 rows)")
    p.add_argument("--dim", type=int, default=None)
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--model-type", choices=["multimodal", "text", "image", "both"], default=None,
                   help="joint-embedding head: multimodal (reference default, model.py:137; 5 fusion layers, "
                        "8 heads), text / image (one tower + its head), both (both single-modality heads)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--collective", action="store_true",
                   help="take the sharded RCCL search path (ShardedIndex: query all-gather, packed result "
                        "all-gather, device merge) even at one rank, to time it on one GPU")
    p.add_argument("--cpu-sample-queries", type=int, default=0)
    p.add_argument("--parity-queries", type=int, default=256,
                   help="queries re-embedded by the fp32 oracle for recall / P@10 vs the CPU path")
    a = p.parse_args(argv)
    pre = dict({"batch": 256, "gallery": 100_000, "k": 10, "model_type": "multimodal", "dim": 768,
                "tower_dtype": "bf16", "rerank": False, "gallery_dtype": "fp32"}, **PRESETS[a.preset])
    for key, v in pre.items():
        if getattr(a, key) is None:
            setattr(a, key, v)
    return a


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def usable_cpus():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup CPU quota
    (a GPU box exposes the whole machine's cores to os.cpu_count() but grants a share of them)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def launch_ranks(a):
    """--gpus N > 1 outside a launcher: start N ranks (one process per GPU) through
    torch.distributed.run on 127.0.0.1 and exit with its status.  Runs before anything touches the
    GPU, as a child process (never an exec)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if a.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}: refusing to report a mismatched run")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or a.collective:
        # the sharded path adds RCCL's stream to the towers' main / side streams and the fusion stack's
        # patch-side stream: past HIP's default 4 hardware queues the command processor time-slices the
        # queues and every kernel of the step ran ~4 % slower (one rank: 14.9 -> 15.6 ms per cfg2 step;
        # with 8 queues 14.9 again, profiles/r05_rccl_hw_queues_ab.txt).  Set before HIP initialises (the
        # pool's boxes export HIP's default 4 explicitly, so raise it rather than only default it).
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
            os.environ["GPU_MAX_HW_QUEUES"] = "8"

    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    coll = world > 1 or a.collective  # the sharded search path over RCCL
    if coll:
        if world == 1 and "MASTER_ADDR" not in os.environ:  # one rank without a launcher
            import socket
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]), RANK="0",
                                  WORLD_SIZE="1")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    import mmr_amd  # noqa: F401
    from mmr_amd import synthetic
    from mmr_amd.retrieval import GalleryIndex, check_status

    # gallery shard: rows [rank*n, (rank+1)*n) of a virtual (world*n, d) N(0,1) gallery
    n, d, K, B = a.gallery, a.dim, a.k, a.batch
    G = synthetic.gauss_gallery(n, d, synthetic.SEED + 17 * rank)
    if a.gallery_dtype == "fp16":  # config 5's fp16 gallery: a native fp16 index (fp16 scan only)
        G = G.astype(np.float16)
        a.knn_mode = "f16"
    index = GalleryIndex(G, device=local, idx_base=rank * n, mode=a.knn_mode)
    index.reserve(2 * B * world)

    model = None
    imgs = ids = mask = None
    if a.mode == "full":
        from mmr_amd.model import build_bench_model
        mt = "text" if a.model_type == "both" else a.model_type
        model = build_bench_model(device=dev, joint_dim=d, model_type=mt, tower_dtype=a.tower_dtype)
        if a.sequential_towers:
            set_streams(model, False)
        if a.model_type != "text":
            imgs = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, synthetic.SEED + rank))).to(dev)
        if a.model_type != "image":
            ids_np, mask_np = synthetic.reports(B, 128, synthetic.SEED + 100 + rank)
            ids, mask = torch.from_numpy(ids_np).to(dev), torch.from_numpy(mask_np).to(dev)
    else:
        qbatch = torch.from_numpy(synthetic.gauss_gallery(B, d, synthetic.SEED + 1 + rank)).to(dev)

    rr = None
    if a.rerank:
        # synthetic rerank tables (reranker.py:88-129 loads them from the KG directory / labels CSV):
        # 1-3 of 43 labels per row as uint64 bitsets, RERANK_DK-wide KG vectors.  Query tables cover
        # all world * nqr queries in all-gather order (same seed on every rank), gallery tables this
        # rank's shard rows
        nqr = B * (2 if a.model_type == "both" else 1)

        def bits(rows, gen):
            lab = torch.randint(0, synthetic.NUM_LABELS, (rows, 3), generator=gen, device=dev)
            keep = torch.rand((rows, 3), generator=gen, device=dev) < torch.tensor([1.0, 0.5, 0.3], device=dev)
            return ((torch.ones_like(lab) << lab) * keep).sum(1)
        gq = torch.Generator(device=dev).manual_seed(synthetic.SEED + 31)
        gg = torch.Generator(device=dev).manual_seed(synthetic.SEED + 32 + rank)
        rr = {"q_lab": bits(world * nqr, gq), "q_kg": torch.randn((world * nqr, RERANK_DK), generator=gq, device=dev),
              "g_lab": bits(n, gg), "g_kg": torch.randn((n, RERANK_DK), generator=gg, device=dev)}

    stream = torch.cuda.current_stream(dev)
    ev_pairs = []
    st_max = torch.zeros((), dtype=torch.int32, device=dev)  # max per-query status over all searches

    sh = None
    rec = {"on": False}
    if coll:  # the product's sharded path (mmr_amd.parallel.ShardedIndex) over RCCL
        from mmr_amd.parallel import ShardedIndex

        def local_search(qq, k):  # this rank's shard, events around the search call (kNN roofline)
            if rec["on"]:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            i, _, s64, st = index.search(qq, k, want_f64=True, want_status=True)
            if rec["on"]:
                e1.record(stream)
                ev_pairs.append((e0, e1))
            return i, s64, st
        sh = ShardedIndex(None, world * n, rank * n, local_search=local_search, status_out=st_max)
        rr_tables = (rr["q_lab"], rr["g_lab"], rr["q_kg"], rr["g_kg"]) if rr is not None else None
        if rr is not None:
            sh.local_components = lambda qq, cand: index.rerank_components(qq, cand, *rr_tables)

    def step(record):
        if model is not None:
            q = model.query_embeddings(imgs, ids, mask)            # (B or 2B, d) f32
        else:
            q = qbatch
        if coll:
            rec["on"] = record
            if rr is None:
                i, s, _ = sh.search(q, K)
            else:
                i = sh.search_rerank(q, K)[0]
                s = None
            return q, i, s
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        i, s, s64, st = index.search(q, K, want_f64=True, want_status=True)
        if record:
            e1.record(stream)
            ev_pairs.append((e0, e1))
        torch.maximum(st_max, st.max(), out=st_max)  # checked after the timed region (no sync here)
        if rr is not None:  # fused rerank of the K candidates (local = global row ids)
            i = index.rerank(q, i, rr["q_lab"], rr["g_lab"], rr["q_kg"], rr["g_kg"], K, want_components=False)[0]
        return q, i, s

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # every search of the timed region returned an exact list (status 0 for every query)
    check_status(st_max.view(1))
    ms_search = sum(e0.elapsed_time(e1) for e0, e1 in ev_pairs) / max(len(ev_pairs), 1)
    q_last, i_last, _ = out
    # HBM-bound regime probe (after the timed region): 16 resident queries — the f16 scan's one-tile
    # stream (knn_scan_f16_gmax<1>) or, in x3 mode, the skinny f32 stream — timed with events on the
    # launch stream, whole search call
    q16 = torch.from_numpy(synthetic.gauss_gallery(16, d, synthetic.SEED + 5 + rank)).to(dev)
    for _ in range(3):
        index.search(q16, K)
    hev = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # a short device-side spin ahead of e0 keeps the stream busy while the host enqueues the
        # call, so e0 -> e1 brackets the call's GPU work (prep / scan / select), not the host's
        # enqueue latency (~60 us of Python + ctypes per call, more than the call's GPU time)
        torch.cuda._sleep(1_000_000)
        e0.record(stream)
        _, _, st16 = index.search(q16, K, want_status=True)
        e1.record(stream)
        hev.append((e0, e1))
    torch.cuda.synchronize(dev)
    check_status(st16)
    lat_small = sum(e0.elapsed_time(e1) for e0, e1 in hev) / len(hev)
    # the same single search with the Infinity Cache (256 MB MALL) flushed first: a 512 MB write
    # between searches evicts the gallery copy, so the search streams it from HBM (the back-to-back
    # figure below re-reads a copy that fits the MALL when n*d*2 < 256 MB)
    flush = torch.empty((512 << 20) // 4, dtype=torch.float32, device=dev)
    hev = []
    for _ in range(10):
        flush.zero_()
        torch.cuda._sleep(1_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        _, _, st16 = index.search(q16, K, want_status=True)
        e1.record(stream)
        hev.append((e0, e1))
    torch.cuda.synchronize(dev)
    check_status(st16)
    lat_cold = sum(e0.elapsed_time(e1) for e0, e1 in hev) / len(hev)
    del flush
    # serving throughput: NB back-to-back 16-query searches between ONE event pair, all enqueued
    # behind a device spin longer than their host enqueue time (so the GPU never waits on the host);
    # every search does its full work (own outputs, status checked)
    NB = 20
    sts = []
    torch.cuda._sleep(12_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(NB):
        sts.append(index.search(q16, K, want_status=True)[2])
    e1.record(stream)
    torch.cuda.synchronize(dev)
    for st16 in sts:
        check_status(st16)
    ms_small = e0.elapsed_time(e1) / NB
    gemm_ms = {}
    if model is not None and a.model_type != "image":
        # per-launch GEMM timings (BERT QKV / O-proj / FFN1 / FFN2) in a short pass right after the
        # timed region with the towers in sequence: inside the timed steps the Swin tower runs
        # concurrently on a side stream, and events around one kernel would also count the
        # co-running kernels' share
        set_streams(model, False)
        model.backbones.bert.gemm_events = {}
        for _ in range(3):
            step(False)
        torch.cuda.synchronize(dev)
        set_streams(model, not a.sequential_towers)
        for name, evs in model.backbones.bert.gemm_events.items():
            gemm_ms[name] = sum(e0.elapsed_time(e1) for e0, e1 in evs) / max(len(evs), 1)
        model.backbones.bert.gemm_events = None

    # whole-job throughput: every rank embeds B queries; every query is scored against the whole
    # world*n gallery (each rank scores all world*B queries against its n rows)
    nq_step = (2 * B) if (model is not None and a.model_type == "both") else B
    q_per_s = world * nq_step * a.steps / elapsed
    pairs_per_s = (world * nq_step) * (world * n) * a.steps / elapsed
    Qs = world * nq_step
    ln_fold = bool(model is not None and a.model_type != "image" and getattr(model.backbones.bert, "ln_fold", False)
                   and (B * 128) % 256 == 0)
    roof, knn_roof = roofline(a, n, d, K, Qs, ms_search, ms_small, q16.shape[0], gemm_ms, B, lat_small, lat_cold,
                              ln_fold=ln_fold)

    cpu = cpu_knn = recall = p10 = x3_line = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        if model is None:
            cpu = cpu_baseline_knn(a, G, qbatch.cpu().numpy())
        else:
            cpu, emb_cpu = cpu_baseline_full(a, G, imgs, ids, mask)
            cpu_knn = cpu_baseline_knn(a, G, q_last[:64].cpu().numpy())
            nq_par = min(a.parity_queries, q_last.shape[0] if a.model_type != "both" else B)
            emb_par = oracle_embeddings(a, imgs, ids, mask, nq_par)
            q_par = q_last[:nq_par] if a.model_type != "both" else torch.cat([q_last[:nq_par], q_last[B:B + nq_par]])
            recall = recall_vs_cpu(index, q_par, emb_par, G, K)
            p10 = precision_vs_cpu(q_par, emb_par, d, a.knn_mode)
            del emb_cpu
            if a.tower_dtype != "x3" and not a.no_x3_line and a.model_type in ("multimodal", "text") and B <= 2048:
                x3_line = x3_block(a, index, G, imgs, ids, mask, emb_par, nq_par, K, dev, steps=10 if B <= 1024 else 3)

    if rank == 0:
        workload = {
            "multimodal": "Swin-T + BERT-base towers + 5-layer multimodal fusion head",
            "text": "text-only BERT-base tower + text head", "image": "Swin-T tower + image head",
            "both": "Swin-T + BERT-base towers + image and text heads"}[a.model_type]
        line = {
            "metric": "query embeddings/sec + cosine-pairs/sec @ Recall@10, 100k x 768 gallery",
            "value": q_per_s if a.mode == "full" else pairs_per_s,
            "unit": "query_embeddings/s" if a.mode == "full" else "cosine_pairs/s",
            "cosine_pairs_per_s": pairs_per_s,
            "query_embeddings_per_s": q_per_s if a.mode == "full" else None,
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": ({"fp8": "MX-fp8 (e4m3 + E8M0/32) tower linears, bf16 elsewhere / ",
                       "x3": "f32 towers (every contraction bf16x3 MFMA, f32 accumulate) / "}.get(a.tower_dtype, "bf16 towers / ")
                      if a.mode == "full" else "") + (
                "fp16 gallery (native fp16 index: the raw rows are the scan operand), exact f64 re-rank"
                if a.gallery_dtype == "fp16" else
                "f32 gallery, fp16 unit-row scan copy, exact f64 re-rank" if a.knn_mode == "f16"
                else "f32 gallery, bf16x3 scan, exact f64 re-rank"),
            "data": "synthetic (seeded N(0,1) gallery; random-init weights)",
            "config": {"workload": ("%s: %s%s, B=%d, top-%d over %dx%d %s per GPU%s" % (
                a.preset, workload, " (MX-fp8 BERT + Swin stage 3-4 linears)" if a.tower_dtype == "fp8" else "", B, K, n, d,
                "fp16" if a.gallery_dtype == "fp16" else "f32",
                " + fused KG/label rerank of the %d candidates" % K if a.rerank else ""))
                       if a.mode == "full" else ("%s kNN only: Q=%d, top-%d over %dx%d f32 per GPU" % (a.preset, B, K, n, d)),
                       "global_batch": world * B, "gallery_rows": world * n, "dim": d, "k": K,
                       "parallelism": (f"gallery row-shard x{world} + tower DP x{world}" if world > 1 else
                                       "single rank, sharded RCCL search path (--collective)" if coll else "single")},
            "roofline": roof,
            "knn_status_ok": True,
            "recall_at_10_vs_cpu": recall["recall_at_k"] if recall else None,
            "recall_vs_cpu": recall,
            "p_at_10": p10,
            "cpu_baseline": cpu,
            "cpu_baseline_knn": cpu_knn,
            "x3_mode": x3_line,
        }
        print(json.dumps(line), flush=True)
    if coll:
        dist.destroy_process_group()


def set_streams(model, on):
    """Side-stream overlap of the Swin tower (and of the fusion stack's patch-side work) on / off."""
    model.concurrent_towers = on
    if getattr(model, "fusion", None) is not None:
        model.fusion.side_streams = on


def roofline(a, n, d, K, Qs, ms_search, ms_small, q_small, gemm_ms, B, lat_small=None, lat_cold=None, ln_fold=False):
    """Roofline object of the dominant kernel (full: the BERT FFN1 GEMM, with the other BERT GEMM
    families beside it; knn: the search call) + the kNN search's own roofline."""
    # kNN search: algorithmic flops 2*Q*N*D; bytes = the scanned gallery copy once + norms + queries +
    # results.  f16: fp16 unit rows (N*D*2), one fp16 MFMA product per f32 product (dense fp16 peak =
    # bf16 peak), HBM-bound below Q ~ 312.  x3: hi/lo bf16 (N*D*4), 3 bf16 MFMA products per f32
    # product; Q <= 32 streams the f32 tile16 copy (N*D*4) on f32 MFMA (HBM-bound).
    peak_bf16, peak_hbm = 2.5e15, 8.0e12
    gbytes = 2 if a.knn_mode == "f16" else 4
    knn_flops = 2.0 * Qs * n * d
    knn_bytes = n * d * gbytes + n * 4 + Qs * d * 4 + Qs * K * 12
    mfma_work = knn_flops * (1 if a.knn_mode == "f16" else 3)
    if a.knn_mode == "f16":
        kname = "mmr_index_search (prep + fp16 MFMA scan + knn_select_t f64 re-rank)"
    elif Qs <= 32:
        kname = "mmr_index_search (prep + knn_scan_f32_gmax skinny f32 MFMA stream + knn_select_t)"
    else:
        kname = "mmr_index_search (prep + knn_scores_x3_gmax bf16x3 MFMA + knn_select_t)"
    t_hbm, t_mfma = knn_bytes / peak_hbm, mfma_work / peak_bf16
    if a.knn_mode == "x3" and Qs <= 32:
        t_mfma = 0.0
    knn_roof = {"kernel": kname, "scan_mode": a.knn_mode, "queries": Qs,
                "ms_per_launch": ms_search, "flops": knn_flops, "bytes": knn_bytes,
                "bound": "mfma" if t_mfma > t_hbm else "hbm",
                "bound_ms": max(t_hbm, t_mfma) * 1e3,
                "frac_of_bound": max(t_hbm, t_mfma) / (ms_search / 1e3),
                "achieved_tflops_f32_equiv": knn_flops / (ms_search / 1e3) / 1e12,
                "achieved_gbs": knn_bytes / (ms_search / 1e3) / 1e9}
    small_bytes = n * d * gbytes + n * 4 + q_small * d * 4 + q_small * K * 12
    knn_roof["hbm_regime"] = {
        "queries": int(q_small), "ms_per_search": ms_small, "bytes": small_bytes,
        "achieved_gbs": small_bytes / (ms_small / 1e3) / 1e9,
        "frac": small_bytes / (ms_small / 1e3) / peak_hbm,
        "timing": "20 back-to-back whole search calls between one event pair on the launch stream "
                  "(serving throughput; queued behind a device spin so the host enqueue is hidden); the "
                  "scanned copy (%d MB) %s the 256 MB Infinity Cache, so these re-reads may be partly "
                  "MALL-served: latency_ms_single_cold flushes it (512 MB write) before each search"
                  % (n * d * gbytes >> 20, "fits" if n * d * gbytes < (256 << 20) else "exceeds"),
        "latency_ms_single": lat_small,
        "latency_frac_single": (small_bytes / (lat_small / 1e3) / peak_hbm) if lat_small else None,
        "latency_ms_single_cold": lat_cold,
        "latency_frac_single_cold": (small_bytes / (lat_cold / 1e3) / peak_hbm) if lat_cold else None,
        "kernel": "whole search call: %s scan + knn_select_t"
                  % ("knn_scan_f16_gmax<1, RAW> (no prep launch)" if a.knn_mode == "f16"
                     else "prep + knn_scan_f32_gmax<1>")}
    fp8 = getattr(a, "tower_dtype", "bf16") == "fp8"
    x3 = getattr(a, "tower_dtype", "bf16") == "x3"
    peak_gemm = 5.0e15 if fp8 else peak_bf16  # dense MX-fp8 / bf16 MFMA peaks (MI355X_MICROARCH.md)
    wmul = 3.0 if x3 else 1.0  # x3: three bf16 MFMA products per f32 product (MFMA work = 3 x flops)
    if gemm_ms:
        M = B * 128
        shapes = {"qkv": (M, 2304, 768), "o": (M, 768, 768), "ffn1": (M, 3072, 768), "ffn2": (M, 768, 3072)}
        fam = {}
        for name, ms in gemm_ms.items():
            m_, n_, k_ = shapes[name]
            fl = 2.0 * m_ * n_ * k_
            fam[name] = {"shape_mnk": [m_, n_, k_], "ms_per_launch": ms, "tflops": fl / (ms / 1e3) / 1e12,
                         "frac": wmul * fl / (ms / 1e3) / peak_gemm}
        ms_ffn1 = gemm_ms["ffn1"]
        fl = 2.0 * M * 3072 * 768
        ln_fold = ln_fold and not (fp8 or x3)
        ffn1_kind = ("LayerNorm-folded mmr_linear_bf16_ln = gemm_bf16_tn_p8<4, 1, LNM=1>" if ln_fold
                     else "tuned variant")
        roof = {"bound": "mfma", "achieved": wmul * fl / (ms_ffn1 / 1e3) / 1e12, "peak": peak_gemm / 1e12,
                "unit": "TFLOP/s", "traffic": None,
                "kernel": (("BERT FFN1 bf16x3 GEMM + GELU (M=%d, N=3072, K=768; x3_gemm, f32 in / out; achieved = "
                            "MFMA work, 3 bf16 products per f32 product), " if x3 else
                            "BERT FFN1 MX-fp8 GEMM + GELU (M=%d, N=3072, K=768; the kernel the timed steps run: "
                            "mmr_linear_mxfp8_q8 = gemm_bf16_tn_p8<4, 1, FP8, OUT8>, emitting FFN2's fp8 operand), "
                            if fp8 else
                            "BERT FFN1 GEMM + GELU (M=%d, N=3072, K=768; %s), ") % ((M,) if (x3 or fp8) else (M, ffn1_kind))
                           + "timed per launch with HIP events in a towers-in-sequence pass after the timed region"),
                "ms_per_launch": ms_ffn1, "flops_per_launch": fl, "bert_gemms": fam, "knn": knn_roof}
    elif a.mode == "full":
        roof = dict(knn_roof, bound=knn_roof["bound"], unit="GB/s", achieved=knn_roof["achieved_gbs"],
                    peak=peak_hbm / 1e9)
    else:
        if knn_roof["bound"] == "mfma":
            roof = {"bound": "mfma", "achieved": mfma_work / (ms_search / 1e3) / 1e12, "peak": peak_bf16 / 1e12,
                    "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": knn_roof["achieved_gbs"], "peak": peak_hbm / 1e9, "unit": "GB/s"}
        roof.update({"traffic": None, "kernel": knn_roof["kernel"], "ms_per_launch": ms_search,
                     "bound_ms": knn_roof["bound_ms"], "frac_of_bound": knn_roof["frac_of_bound"],
                     "hbm_regime": knn_roof["hbm_regime"]})
    roof["frac"] = roof["achieved"] / roof["peak"]
    # HBM traffic per launch from the committed PMC pass (tools/pmc_traffic.py; FETCH_SIZE x2 per the
    # gfx950 correction + WRITE_SIZE), for the same kernels at the same shapes
    tr = pmc_traffic()
    if gemm_ms and (fp8 or x3):
        roof["variant"] = "mxfp8" if fp8 else "x3"
    elif gemm_ms and ln_fold and not (fp8 or x3):
        roof["variant"] = "ln_fold"
        rec = tr.get("bert_ffn1_ln_fold")
        if rec is not None:
            roof["traffic"] = rec["hbm_bytes"]
            roof["traffic_source"] = rec["source"]
    elif gemm_ms:
        from mmr_amd import _lib
        var = int(_lib.lib().mmr_linear_bf16_variant(B * 128, 3072, 768, 1, 1, 0))
        roof["variant"] = var
        rec = tr.get(f"bert_ffn1_v{var}") or tr.get("bert_ffn1")
        if rec is not None:
            roof["traffic"] = rec["hbm_bytes"]
            roof["traffic_source"] = rec["source"]
    elif a.mode == "knn" and B == 256 and n == 100_000 and d == 768:
        keys = ("knn_scan_f16", "knn_select_f16") if a.knn_mode == "f16" else ("knn_scores_x3", "knn_select")
        if all(k in tr for k in keys):
            roof["traffic"] = sum(tr[k]["hbm_bytes"] for k in keys)
            roof["traffic_source"] = tr[keys[0]]["source"]
    return roof, knn_roof


def pmc_traffic():
    """Latest per-round PMC traffic record (profiles/rNN_pmc_traffic.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    try:
        return json.load(open(paths[-1])) if paths else {}
    except (OSError, ValueError):
        return {}


def timed_median(fn, reps=5):
    """one warm-up run, then the median of `reps` timed runs (seconds)."""
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def _cores():
    import torch
    used = usable_cpus()
    torch.set_num_threads(used)
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(used)
    except Exception:
        pass
    return used


def cpu_baseline_knn(a, G, Q):
    """kNN-only baseline: the reference's exact path restated (oracle/knn.py sklearn_topk =
    retrieval_overlap.py:84-90: normalise + f32 sgemm + per-row argsort) on a bounded query sample
    against the same gallery, numpy BLAS on the usable host cores, median of 5 after a warm-up."""
    from oracle import knn as oknn
    used = _cores()
    nq = a.cpu_sample_queries or (16 if G.shape[0] > 200_000 else 64)
    nq = min(nq, Q.shape[0])
    t = timed_median(lambda: oknn.sklearn_topk(Q[:nq], G, a.k))
    return {"value": nq * G.shape[0] / t, "unit": "cosine_pairs/s", "cores": used, "cores_visible": os.cpu_count(),
            "kind": "port",
            "sample": f"{nq} queries x {G.shape[0]}x{G.shape[1]} gallery: numpy normalise + sgemm + argsort "
                      f"top-{a.k} (oracle/knn.py), median of 5 after one warm-up, {used} threads (usable CPUs of "
                      f"{os.cpu_count()} visible), CPU: {cpu_model()}"}


def cpu_baseline_full(a, G, imgs, ids, mask):
    """Oracle CPU path (tests-only infrastructure, timed here as the baseline) on a bounded sample of
    the bench's own inputs: Swin-T / BERT-base fp32 towers (torch CPU) + the same head + numpy cosine
    top-K over the same gallery — the reference's PyTorch-CPU path restated (oracle/towers.py).
    Returns (baseline dict, the sample's oracle joint embeddings) — the latter feed the recall."""
    import torch
    from mmr_amd.model import init_fusion_state, init_head_state
    from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
    from oracle import knn as oknn
    from oracle import towers as otw
    used = _cores()
    nb = a.cpu_sample_queries or 8
    ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
    hsd = init_head_state(768, 768, a.dim, 2711)
    if a.model_type == "multimodal":
        hsd.update(init_fusion_state(768, 768, a.dim, 8, 5, 2712))
    img = imgs[:nb].cpu() if imgs is not None else None
    ii = ids[:nb].cpu() if ids is not None else None
    mm = mask[:nb].cpu() if mask is not None else None
    res = {}

    def run():
        with torch.no_grad():
            if a.model_type == "text":
                t = otw.bert_forward(ii, mm, bsd, BERT_BASE["num_hidden_layers"], BERT_BASE["num_attention_heads"])
                q = otw.heads(None, None, t, hsd, "text")["joint_emb"]
            elif a.model_type == "image":
                g, p = otw.swin_image(img, ssd, SWIN_T)
                q = otw.heads(g, p, None, hsd, "image")["joint_emb"]
            else:
                (g, p), t = otw.backbones_forward(img, ii, mm, ssd, bsd, SWIN_T, BERT_BASE)
                if a.model_type == "multimodal":
                    q = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"]
                else:
                    q = torch.cat([otw.heads(g, p, t, hsd, "image")["joint_emb"],
                                   otw.heads(g, p, t, hsd, "text")["joint_emb"]])
        res["q"] = q.numpy()
        oknn.sklearn_topk(res["q"], G, a.k)
    t = timed_median(run)
    nq = nb * (2 if a.model_type == "both" else 1)
    heads = {"multimodal": "multimodal head", "text": "text tower + text head", "image": "image tower + image head",
             "both": "image and text heads"}[a.model_type]
    return ({"value": nq / t, "unit": "query_embeddings/s", "cores": used, "cores_visible": os.cpu_count(),
             "kind": "port",
             "sample": f"{nb} of the bench's own inputs: fp32 torch-CPU towers + {heads} + numpy cosine/argsort "
                       f"top-{a.k} over {G.shape[0]}x{G.shape[1]} (oracle/towers.py, oracle/knn.py), median of 5 "
                       f"after one warm-up, {used} threads (usable CPUs of {os.cpu_count()} visible), "
                       f"CPU: {cpu_model()}"}, res["q"])


def oracle_embeddings(a, imgs, ids, mask, nq):
    """fp32 oracle (the reference's CPU path restated, oracle/towers.py) joint embeddings of the
    first nq of the bench's own inputs (both: [image heads; text heads])."""
    import torch
    from mmr_amd.model import init_fusion_state, init_head_state
    from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
    from oracle import towers as otw
    _cores()
    ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
    hsd = init_head_state(768, 768, a.dim, 2711)
    if a.model_type == "multimodal":
        hsd.update(init_fusion_state(768, 768, a.dim, 8, 5, 2712))
    img = imgs[:nq].cpu() if imgs is not None else None
    ii = ids[:nq].cpu() if ids is not None else None
    mm = mask[:nq].cpu() if mask is not None else None
    out = []
    with torch.no_grad():
        for c0 in range(0, nq, 16):  # bounded host memory per chunk
            sl = slice(c0, min(nq, c0 + 16))
            if a.model_type == "text":
                t = otw.bert_forward(ii[sl], mm[sl], bsd, BERT_BASE["num_hidden_layers"], BERT_BASE["num_attention_heads"])
                q = otw.heads(None, None, t, hsd, "text")["joint_emb"]
            elif a.model_type == "image":
                g, p = otw.swin_image(img[sl], ssd, SWIN_T)
                q = otw.heads(g, p, None, hsd, "image")["joint_emb"]
            else:
                (g, p), t = otw.backbones_forward(img[sl], ii[sl], mm[sl], ssd, bsd, SWIN_T, BERT_BASE)
                if a.model_type == "multimodal":
                    q = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"]
                else:
                    q = (otw.heads(g, p, t, hsd, "image")["joint_emb"], otw.heads(g, p, t, hsd, "text")["joint_emb"])
            out.append(q)
    if a.model_type == "both":
        return torch.cat([torch.cat([o[0] for o in out]), torch.cat([o[1] for o in out])]).numpy()
    return torch.cat(out).numpy()


def x3_block(a, index, G, imgs, ids, mask, emb_par, nq_par, K, dev, steps=5):
    """The fp32-faithful tower mode (tower_dtype "x3") beside a bf16 / fp8 run: its throughput on the
    same step (same inputs, same index, same K) and its BASELINE.md s3 parity on the same parity
    queries (precision_vs_cpu: topk_equivalent + P@10 / R@10 under random labels)."""
    import torch
    from mmr_amd.model import build_bench_model
    m3 = build_bench_model(device=dev, joint_dim=a.dim, model_type=a.model_type, tower_dtype="x3")

    def st():
        q = m3.query_embeddings(imgs, ids, mask)
        index.search(q, K)
        return q
    # the headline's warm-up count (one step left the first timed steps ~5 % slow: clocks / side streams settle)
    for _ in range(max(1, a.warmup)):
        st()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        q = st()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    p10 = precision_vs_cpu(q[:nq_par], emb_par, a.dim, a.knn_mode)
    rec = recall_vs_cpu(index, q[:nq_par], emb_par, G, K)
    gemms = x3_bert_gemms(m3.backbones.bert, ids.numel(), dev) if a.model_type != "image" else None
    del m3
    torch.cuda.empty_cache()
    return {"tower_dtype": "x3", "query_embeddings_per_s": a.batch / el, "ms_per_step": el * 1e3, "steps": steps,
            "warmup": max(1, a.warmup),
            "bert_gemms_x3": gemms,
            "note": "same step as the headline (B=%d, top-%d over the same index) with f32 towers: every linear and "
                    "attention contraction as hi*hi + hi*lo + lo*hi bf16 MFMA (csrc/x3.hip)" % (a.batch, K),
            "p_at_10": p10, "recall_vs_cpu": rec}


def x3_bert_gemms(bert, rows, dev, reps=10):
    """The four BERT split GEMMs of the x3 step at its shapes (rows = B x L tokens), each launched as the step
    launches it (split-row operands; FFN1 writing FFN2's split rows; O-proj / FFN2 with the f32 residual),
    on layer 0's weights and N(0,1) activations: HIP events around `reps` back-to-back launches on the
    current stream.  frac = bf16 MFMA work (3 products per f32 product) / time / 2.5 PF."""
    import torch
    from mmr_amd import ops
    if not hasattr(bert, "layers") or rows % 256:
        return None
    ly = bert.layers[0]
    C, F = bert.hidden, ly["i_w"].w.shape[0]
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(rows, C, device=dev, generator=g)
    r = torch.randn(rows, C, device=dev, generator=g)
    xr = ops.x3_ln_split(x, ly["ln1_g"], ly["ln1_b"], 1e-12)
    if not isinstance(xr, ops.X3Rows) or F % 384:
        return None
    hr = ops.x3_linear_split_out(xr, ly["i_w"], ly["i_b"], act=1)
    fns = {"qkv": (lambda: ops.x3_linear(xr, ly["qkv_w"], ly["qkv_b"]), 3 * C * C),
           "o": (lambda: ops.x3_linear(xr, ly["o_w"], ly["o_b"], residual=r), C * C),
           "ffn1": (lambda: ops.x3_linear_split_out(xr, ly["i_w"], ly["i_b"], act=1), F * C),
           "ffn2": (lambda: ops.x3_linear(hr, ly["f_w"], ly["f_b"], residual=r), C * F)}
    out = {}
    stream = torch.cuda.current_stream(dev)
    for name, (fn, nk) in fns.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        work = 3 * 2.0 * rows * nk
        out[name] = {"ms_per_launch": ms, "bf16_mfma_flops": work, "frac_of_2p5pf": work / (ms * 1e-3) / 2.5e15}
    out["note"] = ("x3 split GEMMs at the step's shapes, M = %d: HIP events over %d launches each; the bf16 line's "
                   "bert_gemms are in roofline" % (rows, reps))
    return out


def recall_vs_cpu(index, q_gpu, emb_cpu, G, K):
    """Recall@K of the GPU path against the reference CPU path on the same inputs: top-K of the GPU
    (bf16-tower) embeddings through the GPU index vs top-K of the fp32 oracle embeddings through the
    oracle's sklearn-path ranking (retrieval_overlap.py:84-90); recall = |GPU ∩ CPU| / K per query
    (retrieval_eval.py:147-157 style overlap), plus the embedding cosine between the two paths."""
    import numpy as np
    from oracle import knn as oknn
    gi, _ = index.search(q_gpu.contiguous(), K)
    gi = gi.cpu().numpy() - index.idx_base
    ci, _ = oknn.sklearn_topk(emb_cpu, G, K)
    inter = [len(set(gi[r].tolist()) & set(ci[r].tolist())) / K for r in range(len(ci))]
    qg = q_gpu.double().cpu().numpy()
    cos = np.sum(qg * emb_cpu, 1) / (np.linalg.norm(qg, axis=1) * np.linalg.norm(emb_cpu, axis=1))
    return {"recall_at_k": float(np.mean(inter)), "k": K, "queries": int(len(ci)),
            "exact_list_match": float(np.mean([np.array_equal(gi[r], ci[r]) for r in range(len(ci))])),
            "min_embedding_cosine": float(cos.min()),
            "note": "GPU towers (bf16, or MX-fp8 linears at --tower-dtype fp8) + GPU exact kNN vs fp32 oracle towers + "
                    "sklearn-path kNN, same inputs, over the bench's N(0,1) gallery"}


def precision_vs_cpu(q_gpu, emb_cpu, d, knn_mode, K=10, n_gallery=100_000):
    """BASELINE.md §3 "identical Precision@10": the GPU path (GPU towers + GPU exact kNN) and the
    reference CPU path restated (fp32 oracle towers + sklearn-path ranking, retrieval_overlap.py:84-90)
    on the same queries over a LABELLED synthetic gallery (43 labels, 1-3 per row, row = sum of
    label centres + noise; relevance = shares >= 1 label, contructGT.py:69-81), P@10 with the
    reference's precision_at_k (retrieval_metrics.py:4-11) and R@10 / MRR per
    retrieval_overlap.py:84-115 / retrieval_eval.py:146-171."""
    import numpy as np
    from mmr_amd import metrics, synthetic
    from mmr_amd.retrieval import GalleryIndex
    from oracle import knn as oknn
    G, gl = synthetic.labelled_gallery(n_gallery, d, synthetic.SEED + 53)
    gbits = synthetic.labels_to_bits(gl)
    rng = np.random.default_rng(synthetic.SEED + 54)
    nq = q_gpu.shape[0]
    ql = np.zeros((nq, synthetic.NUM_LABELS), np.uint8)
    for r in range(nq):
        ql[r, rng.choice(synthetic.NUM_LABELS, size=int(rng.integers(1, 4)), replace=False)] = 1
    qbits = synthetic.labels_to_bits(ql)
    ix = GalleryIndex(G, mode=knn_mode)
    gi_t, gs_t = ix.search(q_gpu.contiguous(), K)[:2]
    gi, gs = gi_t.cpu().numpy(), gs_t.cpu().numpy()
    import torch
    gx = ix.search(torch.from_numpy(np.ascontiguousarray(emb_cpu, np.float32)).to(q_gpu.device), K)[0].cpu().numpy()
    ix.close()
    ci, cs = oknn.sklearn_topk(emb_cpu, G, K)
    teq, tmsg = oknn.topk_equivalent(ci, cs, gi, gs, tie_tol=1e-6, score_tol=1e-4)

    def pr(idx):
        rel = [[str(j) for j in np.nonzero(gbits & qbits[q])[0]] for q in range(nq)]
        p = float(np.mean([metrics.precision_at_k([str(j) for j in idx[q]], rel[q], K) for q in range(nq)]))
        mrr, _, rec = metrics.ranking_metrics(idx, qbits, gbits, K)
        return p, float(rec), float(mrr)
    pg, rg, mg = pr(gi)
    pc, rc, mc = pr(ci)
    xr_rand = pr(gx)
    qbits = gbits[ci[:, 0]]  # aligned relevance: the labels of the CPU path's nearest gallery item
    ag, arg_, _ = pr(gi)
    ac, arc, _ = pr(ci)
    xr_al = pr(gx)
    return {"queries": int(nq), "gallery": f"labelled {n_gallery}x{d}", "k": K,
            "topk_equivalent": bool(teq), "topk_equivalent_msg": tmsg,
            "topk_equivalent_rule": "oracle.knn.topk_equivalent: identical indices except runs of reference scores within "
                                    "1e-6 (compared as sets), scores within 1e-4 (BASELINE.md s3)",
            "p_at_10_gpu": pg, "p_at_10_cpu": pc, "r_at_10_gpu": rg, "r_at_10_cpu": rc, "mrr_gpu": mg, "mrr_cpu": mc,
            "identical_p_at_10": pg == pc, "identical_r_at_10": rg == rc,
            "relevance": "query labels drawn at random, independent of the embeddings (1-3 of 43; relevance = shares "
                         ">= 1 label, contructGT.py:69-81): any item the tower arithmetic moves across the cut can flip it",
            "retrieval_half_identical": bool(xr_rand[:2] == (pc, rc) and xr_al[:2] == (ac, arc)),
            "retrieval_half_note": "the GPU index fed the CPU path's own (fp32 oracle) embeddings: P@10 / R@10 vs the "
                                   "sklearn-path ranking, both relevance settings",
            "aligned_labels": {"p_at_10_gpu": ag, "p_at_10_cpu": ac, "r_at_10_gpu": arg_, "r_at_10_cpu": arc,
                               "identical_p_at_10": ag == ac, "identical_r_at_10": arg_ == arc,
                               "note": "secondary: query labels = the labels of the query's exact nearest gallery item "
                                       "on the CPU path (relevance consistent with the embedding space; saturates)"},
            "exact_list_match": float(np.mean([np.array_equal(gi[r], ci[r]) for r in range(nq)])),
    "top10_overlap": float(np.mean([len(set(gi[r]) & set(ci[r])) / K for r in range(nq)]))}


if __name__ == "__main__":
    main()
