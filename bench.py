"""Benchmark of the hot path (BASELINE.json metric: query embeddings/sec + cosine-pairs/sec,
100k x 768 gallery).

python bench.py --gpus N --steps K --warmup W [--mode full|knn]
  full (default): one step = Swin-T tower on B synthetic 224x224 images + ClinicalBERT-geometry
        tower on B synthetic 128-token reports (bf16) -> joint-embedding head (default: the
        reference's default model_type "multimodal", 5 fusion layers x 8 heads; --model-type
        text|image runs both single-modality heads) -> exact cosine top-10 of the query embeddings
        over the gallery (config 2: B=256, 100k x 768 f32).
  knn:  one step = exact cosine top-K of B resident queries over the gallery (kNN leg only).
N>1 (torch.distributed.run): the gallery is row-sharded (N x rows per rank: weak scaling), every
rank runs its own query batch through the towers and searches its shard for ALL ranks' queries
(all-gather of query embeddings), then per-shard top-K lists are all-gathered over RCCL and merged.
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", choices=["full", "knn"], default="full")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--knn-mode", choices=["x3", "f16"], default="f16",
                   help="gallery scan: f16 (fp16 unit-row copy, default) or x3 (bf16 split GEMM; skinny f32 "
                        "stream for Q <= 32); both exact (f64 re-rank from the f32 rows)")
    p.add_argument("--gallery", type=int, default=100_000, help="gallery rows per GPU")
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--model-type", choices=["multimodal", "text", "image"], default="multimodal",
                   help="joint-embedding head: multimodal (reference default, model.py:137; 5 fusion "
                        "layers, 8 heads) or the single-modality heads (text + image both run)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-queries", type=int, default=0)
    return p.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    import mmr_amd
    from mmr_amd import synthetic
    from mmr_amd.retrieval import GalleryIndex, merge_topk

    # gallery shard: rows [rank*n, (rank+1)*n) of a virtual (world*n, d) N(0,1) gallery
    n, d, K, B = a.gallery, a.dim, a.k, a.batch
    G = synthetic.gauss_gallery(n, d, synthetic.SEED + 17 * rank)
    index = GalleryIndex(G, device=local, idx_base=rank * n, mode=a.knn_mode)
    index.reserve(2 * B * world)

    model = None
    if a.mode == "full":
        from mmr_amd.model import build_bench_model
        model = build_bench_model(device=dev, joint_dim=d, model_type=a.model_type)
        imgs = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, synthetic.SEED + rank))).to(dev)
        ids_np, mask_np = synthetic.reports(B, 128, synthetic.SEED + 100 + rank)
        ids, mask = torch.from_numpy(ids_np).to(dev), torch.from_numpy(mask_np).to(dev)
    else:
        qbatch = torch.from_numpy(synthetic.gauss_gallery(B, d, synthetic.SEED + 1 + rank)).to(dev)

    stream = torch.cuda.current_stream(dev)
    ev_pairs = []

    def step(record):
        if model is not None:
            q = model.query_embeddings(imgs, ids, mask)            # (B, d) f32
        else:
            q = qbatch
        if world > 1:
            allq = torch.empty((world * q.shape[0], d), dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(allq, q.contiguous())
        else:
            allq = q
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        i, s, s64 = index.search(allq, K, want_f64=True)
        if record:
            e1.record(stream)
            ev_pairs.append((e0, e1))
        if world > 1:
            gi = torch.empty((world * i.shape[0], K), dtype=i.dtype, device=dev)
            gs = torch.empty((world * s64.shape[0], K), dtype=s64.dtype, device=dev)
            dist.all_gather_into_tensor(gi, i)
            dist.all_gather_into_tensor(gs, s64)
            i, s, _ = merge_topk(gs.view(world, -1, K), gi.view(world, -1, K), K)
        return i, s

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
    ms_search = sum(e0.elapsed_time(e1) for e0, e1 in ev_pairs) / max(len(ev_pairs), 1)
    # HBM-bound regime probe (after the timed region): searches of 16 resident queries run the
    # skinny scan (knn_scan_f32_gmax streams the gallery once), timed with events on the launch stream
    q16 = torch.from_numpy(synthetic.gauss_gallery(16, d, synthetic.SEED + 5 + rank)).to(dev)
    for _ in range(3):
        index.search(q16, K)
    hev = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        index.search(q16, K)
        e1.record(stream)
        hev.append((e0, e1))
    torch.cuda.synchronize(dev)
    ms_small = sum(e0.elapsed_time(e1) for e0, e1 in hev) / len(hev)
    if model is not None:
        # roofline kernel (BERT FFN1) timed in a short pass right after the timed region with the
        # towers in sequence: inside the timed steps the Swin tower runs concurrently on a side
        # stream, and events around one kernel would also count the co-running kernels' share
        saved = {k: os.environ.get(k) for k in ("MMR_TOWER_STREAMS", "MMR_FUSION_STREAMS")}
        os.environ.update({k: "0" for k in saved})
        model.backbones.bert.ffn1_events = []
        for _ in range(3):
            step(False)
        torch.cuda.synchronize(dev)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    # whole-job throughput: every rank embeds B queries; every query is scored against the whole
    # world*n gallery (each rank scores all world*B queries against its n rows)
    # full mode: one multimodal joint embedding per (image, report) pair, or image-head + text-head
    nq_step = (2 * B) if (model is not None and a.model_type != "multimodal") else B
    q_per_s = world * B * a.steps / elapsed
    pairs_per_s = (world * nq_step) * (world * n) * a.steps / elapsed
    # roofline of the dominant kernel, per launch on one GPU
    Qs = world * nq_step
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
        kname = "mmr_index_search (prep + knn_scan_f16_gmax fp16 MFMA stream + knn_select_groups f64 re-rank)"
    elif Qs <= 32:
        kname = "mmr_index_search (prep + knn_scan_f32_gmax skinny f32 MFMA stream + knn_select_groups)"
    else:
        kname = "mmr_index_search (prep + knn_scores_x3_gmax bf16x3 MFMA + knn_select_groups)"
    mfma_bound = a.knn_mode == "x3" and Qs > 32 and mfma_work / peak_bf16 > knn_bytes / peak_hbm
    if a.knn_mode == "f16":
        mfma_bound = mfma_work / peak_bf16 > knn_bytes / peak_hbm
    knn_roof = {"kernel": kname, "scan_mode": a.knn_mode,
                "ms_per_launch": ms_search, "flops": knn_flops, "bytes": knn_bytes,
                "bound": "mfma" if mfma_bound else "hbm",
                "achieved_tflops_f32_equiv": knn_flops / (ms_search / 1e3) / 1e12,
                "achieved_gbs": knn_bytes / (ms_search / 1e3) / 1e9}
    small_bytes = n * d * gbytes + n * 4 + q16.shape[0] * d * 4 + q16.shape[0] * K * 12
    knn_roof["hbm_regime"] = {
        "queries": int(q16.shape[0]), "ms_per_search": ms_small, "bytes": small_bytes,
        "achieved_gbs": small_bytes / (ms_small / 1e3) / 1e9,
        "frac": small_bytes / (ms_small / 1e3) / peak_hbm,
        "kernel": "whole search call: prep + %s scan + knn_select_groups (events on the launch stream)"
                  % ("knn_scan_f16_gmax" if a.knn_mode == "f16" else "knn_scan_f32_gmax")}
    if model is not None:
        evs = model.backbones.bert.ffn1_events
        ms_ffn1 = sum(e0.elapsed_time(e1) for e0, e1 in evs) / max(len(evs), 1)
        fl = 2.0 * B * 128 * 3072 * 768
        roof = {"bound": "mfma", "achieved": fl / (ms_ffn1 / 1e3) / 1e12, "peak": peak_bf16 / 1e12,
                "unit": "TFLOP/s", "traffic": None,
                "kernel": ("BERT FFN1 GEMM + GELU (M=%d, N=3072, K=768; tuned variant), %d launches timed in a "
                           "towers-in-sequence pass after the timed region" % (B * 128, len(evs))),
                "ms_per_launch": ms_ffn1, "flops_per_launch": fl, "knn": knn_roof}
    else:
        if knn_roof["bound"] == "mfma":
            roof = {"bound": "mfma", "achieved": mfma_work / (ms_search / 1e3) / 1e12, "peak": peak_bf16 / 1e12,
                    "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": knn_roof["achieved_gbs"], "peak": peak_hbm / 1e9, "unit": "GB/s"}
        roof.update({"traffic": None, "kernel": knn_roof["kernel"], "ms_per_launch": ms_search,
                     "hbm_regime": knn_roof["hbm_regime"]})
    roof["frac"] = roof["achieved"] / roof["peak"]
    # HBM traffic per launch from the committed PMC pass (tools/pmc_traffic.py; FETCH_SIZE x2 per the
    # gfx950 correction + WRITE_SIZE), for the same kernels at the same shapes
    tr = pmc_traffic()
    if model is not None:
        # the FFN1 launch variant the per-shape tuner settled on here; its PMC record if committed
        from mmr_amd import _lib
        var = int(_lib.lib().mmr_linear_bf16_variant(B * 128, 3072, 768, 1, 1, 0))
        roof["variant"] = var
        rec = tr.get(f"bert_ffn1_v{var}")
        if rec is not None:
            roof["traffic"] = rec["hbm_bytes"]
            roof["traffic_source"] = rec["source"]
    if (model is None and a.knn_mode == "x3" and "knn_scores_x3" in tr and "knn_select" in tr and B == 256
            and n == 100_000 and d == 768):
        roof["traffic"] = tr["knn_scores_x3"]["hbm_bytes"] + tr["knn_select"]["hbm_bytes"]
        roof["traffic_source"] = tr["knn_scores_x3"]["source"]
    if (model is None and a.knn_mode == "f16" and "knn_scan_f16" in tr and "knn_select_f16" in tr and B == 256
            and n == 100_000 and d == 768):
        roof["traffic"] = tr["knn_scan_f16"]["hbm_bytes"] + tr["knn_select_f16"]["hbm_bytes"]
        roof["traffic_source"] = tr["knn_scan_f16"]["source"]

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, G, qbatch) if model is None else cpu_baseline_full(a, G)

    if rank == 0:
        line = {
            "metric": "query embeddings/sec + cosine-pairs/sec @ Recall@10, 100k x 768 gallery",
            "value": q_per_s if a.mode == "full" else pairs_per_s,
            "unit": "query_embeddings/s" if a.mode == "full" else "cosine_pairs/s",
            "cosine_pairs_per_s": pairs_per_s,
            "query_embeddings_per_s": q_per_s if a.mode == "full" else None,
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": ("bf16 towers / " if a.mode == "full" else "") + (
                "f32 gallery, fp16 unit-row scan copy, exact f64 re-rank" if a.knn_mode == "f16"
                else "f32 gallery, bf16x3 scan, exact f64 re-rank"),
            "data": "synthetic (seeded N(0,1) gallery; random-init weights)",
            "config": {"workload": ("cfg2: Swin-T + BERT-base towers + %s head, B=%d, top-%d over %dx%d f32 per GPU"
                                    % ("5-layer multimodal fusion" if a.model_type == "multimodal" else "image+text",
                                       B, K, n, d))
                       if a.mode == "full" else ("kNN only: Q=%d, top-%d over %dx%d f32 per GPU" % (B, K, n, d)),
                       "global_batch": world * B, "gallery_rows": world * n, "dim": d, "k": K,
                       "parallelism": f"gallery row-shard x{world}" if world > 1 else "single"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic():
    """Latest per-round PMC traffic record (profiles/rNN_pmc_traffic.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    try:
        return json.load(open(paths[-1])) if paths else {}
    except (OSError, ValueError):
        return {}


def cpu_baseline(a, G, qbatch):
    """kNN-only baseline: the reference's exact path restated (oracle/knn.py sklearn_topk =
    retrieval_overlap.py:84-90: normalise + f32 sgemm + per-row argsort) on a bounded query sample
    against the same gallery, numpy BLAS on all host cores."""
    from oracle import knn as oknn
    nq = a.cpu_sample_queries or min(64, a.batch)
    Q = qbatch[:nq].cpu().numpy()
    oknn.sklearn_topk(Q[:1], G, a.k)
    t0 = time.perf_counter()
    oknn.sklearn_topk(Q, G, a.k)
    t = time.perf_counter() - t0
    try:
        from threadpoolctl import threadpool_info
        cores = max(int(p.get("num_threads", 1)) for p in threadpool_info() if p.get("user_api") == "blas")
    except Exception:
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": nq * G.shape[0] / t, "unit": "cosine_pairs/s", "cores": cores, "kind": "port",
            "sample": f"{nq} queries x {G.shape[0]}x{G.shape[1]} gallery: numpy normalise + sgemm + argsort "
                      f"top-{a.k} (oracle/knn.py), one timed run after warm-up, CPU: {cpu_model()}"}


def cpu_baseline_full(a, G):
    """Oracle CPU path (tests-only infrastructure, timed here as the baseline) on a bounded sample:
    Swin-T + BERT-base fp32 towers (torch CPU, all host cores) + text/image heads + numpy cosine
    top-K over the same gallery — the reference's PyTorch-CPU path restated (oracle/towers.py)."""
    import numpy as np
    import torch
    from mmr_amd import synthetic
    from mmr_amd.model import init_head_state
    from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
    from oracle import knn as oknn
    from oracle import towers as otw
    threads = torch.get_num_threads()
    nb = a.cpu_sample_queries or 8
    ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
    hsd = init_head_state(768, 768, a.dim, 2711)
    if a.model_type == "multimodal":
        from mmr_amd.model import init_fusion_state
        hsd.update(init_fusion_state(768, 768, a.dim, 8, 5, 2712))
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(nb, synthetic.SEED)))
    ids, mask = (torch.from_numpy(x) for x in synthetic.reports(nb, 128, synthetic.SEED + 100))

    def run(n):
        with torch.no_grad():
            (g, p), t = otw.backbones_forward(img[:n], ids[:n], mask[:n], ssd, bsd, SWIN_T, BERT_BASE)
            if a.model_type == "multimodal":
                qi = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"]
                qt = qi[:0]
            else:
                qi = otw.heads(g, p, t, hsd, "image")["joint_emb"]
                qt = otw.heads(g, p, t, hsd, "text")["joint_emb"]
        oknn.sklearn_topk(torch.cat([qi, qt]).numpy(), G, a.k)
    run(1)
    t0 = time.perf_counter()
    run(nb)
    t = time.perf_counter() - t0
    return {"value": nb / t, "unit": "query_embeddings/s", "cores": threads, "kind": "port",
            "sample": f"{nb} (image, 128-token report) pairs: fp32 torch-CPU Swin-T + BERT-base + {a.model_type} "
                      f"head(s) + numpy cosine/argsort top-{a.k} over {G.shape[0]}x{G.shape[1]} (oracle/towers.py, "
                      f"oracle/knn.py), one timed run after warm-up, CPU: {cpu_model()}"}


if __name__ == "__main__":
    main()
