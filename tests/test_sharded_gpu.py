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

N, D, B, K = 30_011, 384, 24, 16


def _gallery():
    G = synthetic.gauss_gallery(N, D, 501)
    G[17] = G[N - 5]          # exact duplicate across the two shards: tie broken by global index
    G[40] = 0.0
    return G


def _worker(rank, world, port, mode, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        G = _gallery()
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


@pytest.mark.parametrize("mode", ["f16", "x3"])
def test_sharded_gallery_index_world2_equals_single_device(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    G = _gallery()
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
