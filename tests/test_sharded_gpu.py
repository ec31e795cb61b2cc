"""GPU, world_size 2 over gloo: ShardedIndex with the real libmmr GalleryIndex per rank (both ranks
on cuda:0; the per-shard lists are staged to host for gloo), in the f16 and x3 scan modes — the
merged result is bit-identical to one single-device index over the whole gallery (indices and f64
scores).  On the 8-GPU node the same class runs over RCCL (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mmr_amd import synthetic
from mmr_amd.parallel import ShardedIndex, shard_bounds
from mmr_amd.retrieval import GalleryIndex

pytestmark = pytest.mark.gpu

SMALL = (30_011, 384, 24, 16)
CFG4 = (2_000_000, 768, 128, 10)   # BASELINE cfg4's per-GPU shard (1M rows) at world 2


def _gallery(N, D):
    G = synthetic.gauss_gallery(N, D, 501)
    G[17] = G[N - 5]          # exact duplicate across the two shards: tie broken by global index
    G[40] = 0.0
    return G


def _worker(rank, world, port, mode, shape, out_q):
    N, D, B, K = shape
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        G = _gallery(N, D)
        Q = synthetic.gauss_gallery(world * B, D, 502)
        Q[0] = G[17]
        s, e = shard_bounds(N, world)[rank]
        ix = GalleryIndex(G[s:e], device=0, idx_base=s, mode=mode)

        def local(q, k):  # gloo exchanges host tensors: device search, lists staged to host
            i, _, s64, st = ix.search(q.cuda(), k, want_f64=True, want_status=True)
            return i.cpu(), s64.cpu(), st.cpu()

        sh = ShardedIndex(G[s:e], N, s, local_search=local)
        mi, ms, m64 = sh.search(torch.from_numpy(Q[rank * B:(rank + 1) * B]), K)
        out_q.put((rank, mi.numpy(), m64.numpy(), sh.reruns))
        ix.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,shape", [("f16", SMALL), ("x3", SMALL), ("f16", CFG4)])
def test_sharded_gallery_index_world2_equals_single_device(mode, shape):
    """Two ranks, each holding half the gallery (cfg4 case: 2 x 1M x 768, 128 queries per rank,
    top-10 on the 4-row-unit path), merged = one index over the whole gallery, bit for bit."""
    N, D, B, K = shape
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, shape, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    G = _gallery(N, D)
    Q = synthetic.gauss_gallery(world * B, D, 502)
    Q[0] = G[17]
    ix = GalleryIndex(G, mode=mode)
    si, _, s64 = ix.search(torch.from_numpy(Q).cuda(), K, want_f64=True)
    si, s64 = si.cpu().numpy(), s64.cpu().numpy()
    ix.close()
    assert si[0, :2].tolist() == [17, N - 5]
    for rank, mi, m64, reruns in res:
        assert reruns == 0
        np.testing.assert_array_equal(mi, si[rank * B:(rank + 1) * B])
        np.testing.assert_array_equal(m64, s64[rank * B:(rank + 1) * B])


def _worker_rerank(rank, world, port, out_q):
    """Sharded rerank over gloo with the real per-rank GalleryIndex: components computed on the
    owning shard, lists + components all-gathered (staged to host), host merge + host mix."""
    N, D, B, K, DK = 20_011, 256, 16, 12, 64
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        G, gb, qb, gk, qk = _rerank_data(N, D, world * B, DK)
        Q = synthetic.gauss_gallery(world * B, D, 512)
        s, e = shard_bounds(N, world)[rank]
        ix = GalleryIndex(G[s:e], device=0, idx_base=s, mode="f16")
        dev = torch.device("cuda:0")

        def local(q, k):
            i, _, s64, st = ix.search(q.cuda(), k, want_f64=True, want_status=True)
            return i.cpu(), s64.cpu(), st.cpu()

        def comps(q, cand):
            return ix.rerank_components(q.cuda(), cand.cuda(), _t(qb, dev), _t(gb[s:e], dev), _t(qk, dev),
                                        _t(gk[s:e], dev)).cpu()

        sh = ShardedIndex(G[s:e], N, s, local_search=local, local_components=comps)
        out = sh.search_rerank(torch.from_numpy(Q[rank * B:(rank + 1) * B]), K)
        out_q.put((rank,) + tuple(t.numpy() for t in out))
        ix.close()
    finally:
        dist.destroy_process_group()


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64) if a.dtype == np.uint64 else a).to(dev)


def _rerank_data(N, D, Q, DK):
    rng = np.random.default_rng(511)
    G = synthetic.gauss_gallery(N, D, 511)
    G[3] = G[N - 7]
    gb = rng.integers(0, 1 << 20, size=N).astype(np.uint64)
    qb = rng.integers(0, 1 << 20, size=Q).astype(np.uint64)
    return G, gb, qb, rng.standard_normal((N, DK), dtype=np.float32), rng.standard_normal((Q, DK), dtype=np.float32)


def test_sharded_rerank_world2_matches_single_index():
    """config 5's rerank at world > 1: (idx, final, emb_n, lab_n, kg_n) of the sharded path equal the
    single-index fused rerank (mmr_index_rerank) — order exactly, scores within f64 contraction
    rounding (the host mix vs the device's fused multiply-adds)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_worker_rerank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N, D, B, K, DK = 20_011, 256, 16, 12, 64
    G, gb, qb, gk, qk = _rerank_data(N, D, world * B, DK)
    Q = synthetic.gauss_gallery(world * B, D, 512)
    dev = torch.device("cuda:0")
    ix = GalleryIndex(G, mode="f16")
    qd = torch.from_numpy(Q).cuda()
    i = ix.search(qd, K)[0]
    ref = [t.cpu().numpy() for t in ix.rerank(qd, i, _t(qb, dev), _t(gb, dev), _t(qk, dev), _t(gk, dev), K)]
    ix.close()
    for rank, *got in res:
        sl = slice(rank * B, (rank + 1) * B)
        np.testing.assert_array_equal(got[0], ref[0][sl])
        for a, b in zip(got[1:], ref[1:]):
            np.testing.assert_allclose(a, b[sl], rtol=0, atol=1e-12)


def _simulated_gather(shards, Q, K, world, comps=None):
    """What the all-gather delivers on the 8-GPU node, built on one GPU: every shard searches ALL
    world*b queries, packs its lists (pack_lists) and the packs are stacked in rank order
    ([world][world*b][K][2 + P], the layout all_gather_into_tensor produces)."""
    from mmr_amd.parallel import pack_lists
    packs = []
    for r, ix in enumerate(shards):
        i, _, s64 = ix.search(Q, K, want_f64=True)
        packs.append(pack_lists(i, s64, comps[r](Q, i) if comps else None))
    return torch.stack(packs)


@pytest.mark.parametrize("mode", ["f16", "x3"])
def test_device_merge_simulated_world2_equals_single_index(mode):
    """The device branch of ShardedIndex.search (merge_gathered -> mmr_merge_topk_packed straight
    from the gathered buffer, each rank merging its own queries q0 = rank*b) on one GPU with a
    simulated 2-rank gather: bit-identical to one index over the whole gallery (indices, f32 and f64
    scores), exact duplicates across the shards tie-broken by global index."""
    from mmr_amd.parallel import merge_gathered
    N, D, B, K, world = 30_011, 384, 24, 16, 2
    G = _gallery(N, D)
    Q = synthetic.gauss_gallery(world * B, D, 502)
    Q[0] = G[17]
    Qd = torch.from_numpy(Q).cuda()
    shards = [GalleryIndex(G[s:e], device=0, idx_base=s, mode=mode) for s, e in shard_bounds(N, world)]
    g = _simulated_gather(shards, Qd, K, world)
    ix = GalleryIndex(G, mode=mode)
    si, ss, s64 = ix.search(Qd, K, want_f64=True)
    for rank in range(world):
        mi, ms, m64 = merge_gathered(g, rank * B, B, K)
        assert mi.is_cuda
        sl = slice(rank * B, (rank + 1) * B)
        assert torch.equal(mi, si[sl]) and torch.equal(m64, s64[sl]) and torch.equal(ms, ss[sl])
    assert si[0, :2].tolist() == [17, N - 5]
    for x in shards + [ix]:
        x.close()


def test_device_merge_simulated_world2_rerank_equals_single_index():
    """ShardedIndex.search_rerank's device branch (components ride in the same packed gather,
    merge_gathered with payload, then mmr_rerank_mix) on one GPU, simulated 2-rank gather:
    equal to the single-index fused rerank (order exactly, components within 1e-12)."""
    from mmr_amd.parallel import merge_gathered
    from mmr_amd.retrieval import rerank_mix
    N, D, B, K, DK, world = 20_011, 256, 16, 12, 64, 2
    G, gb, qb, gk, qk = _rerank_data(N, D, world * B, DK)
    Q = torch.from_numpy(synthetic.gauss_gallery(world * B, D, 512)).cuda()
    dev = torch.device("cuda:0")
    bounds = shard_bounds(N, world)
    shards = [GalleryIndex(G[s:e], device=0, idx_base=s, mode="f16") for s, e in bounds]
    comps = [(lambda q, cand, ix=ix, s=s, e=e: ix.rerank_components(q, cand, _t(qb, dev), _t(gb[s:e], dev),
                                                                     _t(qk, dev), _t(gk[s:e], dev)))
             for ix, (s, e) in zip(shards, bounds)]
    g = _simulated_gather(shards, Q, K, world, comps)
    ix = GalleryIndex(G, mode="f16")
    i = ix.search(Q, K)[0]
    ref = ix.rerank(Q, i, _t(qb, dev), _t(gb, dev), _t(qk, dev), _t(gk, dev), K)
    for rank in range(world):
        mi, _, _, mc = merge_gathered(g, rank * B, B, K, payload_width=3)
        out = rerank_mix(mi, mc, K)
        sl = slice(rank * B, (rank + 1) * B)
        assert torch.equal(out[0], ref[0][sl])
        for a, b in zip(out[1:], ref[1:]):
            assert (a - b[sl]).abs().max().item() <= 1e-12
    for x in shards + [ix]:
        x.close()


def test_set_mode_failure_keeps_index_usable():
    """a mode switch whose copies cannot be built (here a real device OOM: the free memory
    is taken first) must leave the index in its previous mode with its copies intact — the next
    search in that mode returns the exact list (it used to scan a freed fp16 copy)."""
    from mmr_amd._lib import MMRError
    N, D, B, K = 400_000, 1024, 16, 10
    G = synthetic.gauss_gallery(N, D, 601)
    Q = torch.from_numpy(synthetic.gauss_gallery(B, D, 602)).cuda()
    ix = GalleryIndex(G, mode="f16")
    ref_i, _, ref64 = ix.search(Q, K, want_f64=True)
    torch.cuda.synchronize()
    free, _ = torch.cuda.mem_get_info()
    # x3 copies need 3.3 GB; 1.5 GB stays free for the searches' kernel scratch
    hog = torch.empty(max(0, free - (1536 << 20)), dtype=torch.uint8, device="cuda")
    try:
        with pytest.raises(MMRError):
            ix.set_mode("x3")
        i, _, s64 = ix.search(Q, K, want_f64=True)
        assert torch.equal(i, ref_i) and torch.equal(s64, ref64)
        gb, _ = ix.device_bytes()
        assert gb <= N * D * 4 + N * 12 + 2 * (N + 256) * D * 2 + (1 << 20)  # f32 rows + fp16 copies only
    finally:
        del hog
        torch.cuda.empty_cache()
    ix.set_mode("x3")
    i, _, s64 = ix.search(Q, K, want_f64=True)
    assert torch.equal(i, ref_i) and torch.equal(s64, ref64)
    ix.close()


def _worker_rccl1(port, out_q):
    """One rank over RCCL (backend "nccl"): the product's device path exactly as the 8-GPU run takes it
    — device queries all-gathered by all_gather_into_tensor, the per-shard search on the GPU, ONE packed
    all-gather of the lists (+ rerank components), the device merge — at world 1 on this box's GPU."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        N, D, B, K, DK = 20_011, 256, 16, 12, 64
        G, gb, qb, gk, qk = _rerank_data(N, D, B, DK)
        Q = torch.from_numpy(synthetic.gauss_gallery(B, D, 512)).cuda()
        dev = torch.device("cuda:0")
        sh = ShardedIndex.from_full(G, device=0, mode="f16")
        assert dist.get_backend() == "nccl" and sh.world == 1
        mi, ms, m64 = sh.search(Q, K)
        tables = (_t(qb, dev), _t(gb, dev), _t(qk, dev), _t(gk, dev))
        rr = sh.search_rerank(Q, K, tables=tables)
        torch.cuda.synchronize()

        # the device status row through RCCL: a local search that flags one query with a
        # DEVICE status tensor — written into the packed all_gather_into_tensor buffer, read back by
        # gathered_status — makes search raise 'status 1' after the exchange; the group still works
        def flagged(q, k):
            i, s64, st = sh._index_search(q, k)
            st = st.clone()
            st[1] = 1
            return i, s64, st

        msg = "no error"
        try:
            ShardedIndex(None, sh.n_total, sh.start, local_search=flagged).search(Q, K)
        except RuntimeError as ex:
            msg = str(ex)
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        # with status_out the flag accumulates on the device instead (no host sync, no raise)
        so = torch.zeros((), dtype=torch.int32, device=dev)
        fi, _, _ = ShardedIndex(None, sh.n_total, sh.start, local_search=flagged, status_out=so).search(Q, K)
        torch.cuda.synchronize()
        out_q.put((mi.cpu().numpy(), m64.cpu().numpy(), [t_.cpu().numpy() for t_ in rr],
                   (msg, float(t.item()), int(so.item()), bool(torch.equal(fi, mi)))))
    finally:
        dist.destroy_process_group()


def test_sharded_index_over_rccl_world1_equals_single_index():
    """The RCCL branch of ShardedIndex on hardware (world 1: the collectives run through RCCL on this
    GPU; the 8-GPU scaling run takes the same calls): search and search_rerank equal the single index."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = ctx.Process(target=_worker_rccl1, args=(port, q))
    p.start()
    mi, m64, rr, (msg, red, so, same) = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert "status 1" in msg, msg
    assert red == 1.0 and so == 1 and same
    N, D, B, K, DK = 20_011, 256, 16, 12, 64
    G, gb, qb, gk, qk = _rerank_data(N, D, B, DK)
    dev = torch.device("cuda:0")
    ix = GalleryIndex(G, mode="f16")
    qd = torch.from_numpy(synthetic.gauss_gallery(B, D, 512)).cuda()
    si, _, s64 = ix.search(qd, K, want_f64=True)
    ref = [t.cpu().numpy() for t in ix.rerank(qd, si, _t(qb, dev), _t(gb, dev), _t(qk, dev), _t(gk, dev), K)]
    si, s64 = si.cpu().numpy(), s64.cpu().numpy()
    ix.close()
    np.testing.assert_array_equal(mi, si)
    np.testing.assert_array_equal(m64, s64)
    np.testing.assert_array_equal(rr[0], ref[0])
    for a, b in zip(rr[1:], ref[1:]):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)
