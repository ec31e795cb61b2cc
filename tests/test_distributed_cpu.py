"""CPU, world_size 2 and 3 over gloo: the row-sharded search path (shard bounds, query all-gather,
per-shard list all-gather, deterministic merge) returns exactly the single-device exact top-K.
The per-shard search is stood in by the oracle here (no GPU); on the GPU box the same ShardedIndex
runs libmmr per rank (tests/test_knn_gpu.py::test_shard_merge_equals_single_index covers the
device merge kernel)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mmr_amd import synthetic
from mmr_amd.parallel import ShardedIndex, merge_topk_host, shard_bounds
from oracle import knn as oknn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, D, b, K, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, _ = synthetic.labelled_gallery(N, D, 77)
        G[5] = G[N - 3]           # an exact duplicate across shards: tie broken by global index
        Q, _ = synthetic.labelled_gallery(world * b, D, 78)
        s, e = shard_bounds(N, world)[rank]

        def local(q, k):
            i, sc = oknn.exact_topk(q.numpy(), G[s:e], k)
            i = np.where(i >= 0, i + s, -1)
            if i.shape[1] < k:  # shard smaller than k
                pad = k - i.shape[1]
                i = np.concatenate([i, np.full((i.shape[0], pad), -1)], 1)
                sc = np.concatenate([sc, np.full((sc.shape[0], pad), -np.inf)], 1)
            return torch.from_numpy(i.astype(np.int64)), torch.from_numpy(sc)

        sh = ShardedIndex(G[s:e], N, s, local_search=local)
        q_local = torch.from_numpy(Q[rank * b:(rank + 1) * b])
        mi, ms, m64 = sh.search(q_local, K)
        out_q.put((rank, mi.numpy(), m64.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 3001), (3, 25)])
def test_sharded_search_equals_single_device(world, N):
    D, b, K = 64, 5, 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, D, b, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    G, _ = synthetic.labelled_gallery(N, D, 77)
    G[5] = G[N - 3]
    Q, _ = synthetic.labelled_gallery(world * b, D, 78)
    ei, es = oknn.exact_topk(Q, G, K)
    for rank, mi, m64 in res:
        np.testing.assert_array_equal(mi, ei[rank * b:(rank + 1) * b])
        np.testing.assert_allclose(m64, es[rank * b:(rank + 1) * b], rtol=0, atol=1e-14)  # BLAS blocking


def test_shard_bounds_and_host_merge_edges():
    assert shard_bounds(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert shard_bounds(2, 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]
    # empty slots, equal scores across lists, fewer valid than k_out
    s = torch.tensor([[[0.9, 0.5, -np.inf]], [[0.9, 0.7, -np.inf]]], dtype=torch.float64)
    i = torch.tensor([[[7, 2, -1]], [[3, 9, -1]]])
    mi, ms, m64 = merge_topk_host(s, i, 5)
    assert mi.tolist() == [[3, 7, 9, 2, -1]]
    assert m64[0, :4].tolist() == [0.9, 0.9, 0.7, 0.5] and np.isneginf(m64[0, 4].item())
