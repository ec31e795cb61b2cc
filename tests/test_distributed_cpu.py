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


def _worker_status(rank, world, port, N, D, b, K, out_q):
    """local_search flags every other query as overflowed (status 1) and returns garbage for it;
    ShardedIndex must re-run exactly those through fallback_search before the exchange."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, _ = synthetic.labelled_gallery(N, D, 81)
        Q, _ = synthetic.labelled_gallery(world * b, D, 82)
        s, e = shard_bounds(N, world)[rank]
        calls = []

        def exact(q, k):
            i, sc = oknn.exact_topk(q.numpy(), G[s:e], k)
            return torch.from_numpy(np.where(i >= 0, i + s, -1).astype(np.int64)), torch.from_numpy(sc)

        def local(q, k):
            i, sc = exact(q, k)
            st = torch.zeros(q.shape[0], dtype=torch.int32)
            st[::2] = 1
            i[::2] = 0                 # garbage for the flagged queries
            sc[::2] = 9.0
            return i, sc, st

        def fallback(q, k):
            calls.append(q.shape[0])
            return exact(q, k)

        sh = ShardedIndex(G[s:e], N, s, local_search=local, fallback_search=fallback)
        mi, ms, m64 = sh.search(torch.from_numpy(Q[rank * b:(rank + 1) * b]), K)
        out_q.put((rank, mi.numpy(), m64.numpy(), sh.reruns, calls))
    finally:
        dist.destroy_process_group()


def test_sharded_search_reruns_flagged_queries():
    world, N, D, b, K = 2, 1500, 48, 5, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_status, args=(r, world, port, N, D, b, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    G, _ = synthetic.labelled_gallery(N, D, 81)
    Q, _ = synthetic.labelled_gallery(world * b, D, 82)
    ei, es = oknn.exact_topk(Q, G, K)
    for rank, mi, m64, reruns, calls in res:
        assert reruns == (world * b + 1) // 2 and calls == [(world * b + 1) // 2]
        np.testing.assert_array_equal(mi, ei[rank * b:(rank + 1) * b])
        np.testing.assert_allclose(m64, es[rank * b:(rank + 1) * b], rtol=0, atol=1e-14)


def _worker_status_raise(rank, world, port, N, D, b, K, out_q):
    """Rank 0's local search flags one query (status 1) and there is no fallback: the status rides in the
    packed result exchange and EVERY rank raises after it — none is left blocked in the collective."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, _ = synthetic.labelled_gallery(N, D, 83)
        Q, _ = synthetic.labelled_gallery(world * b, D, 84)
        s, e = shard_bounds(N, world)[rank]

        def local(q, k):
            i, sc = oknn.exact_topk(q.numpy(), G[s:e], k)
            st = torch.zeros(q.shape[0], dtype=torch.int32)
            if rank == 0:
                st[1] = 1
            return torch.from_numpy(np.where(i >= 0, i + s, -1).astype(np.int64)), torch.from_numpy(sc), st

        sh = ShardedIndex(G[s:e], N, s, local_search=local)
        try:
            sh.search(torch.from_numpy(Q[rank * b:(rank + 1) * b]), K)
            out_q.put((rank, "no error"))
        except RuntimeError as ex:
            out_q.put((rank, str(ex)))
        # the group is still usable afterwards (nobody was left inside a collective)
        t = torch.ones(1)
        dist.all_reduce(t)
        out_q.put((rank, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_sharded_search_status_raises_on_every_rank():
    world, N, D, b, K = 2, 800, 32, 4, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_status_raise, args=(r, world, port, N, D, b, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    msgs = [m for _, m in res if isinstance(m, str)]
    assert len(msgs) == world and all("status 1" in m for m in msgs), msgs
    assert [m for _, m in res if not isinstance(m, str)] == [float(world)] * world


def test_dls_cache_path_naming(tmp_path, monkeypatch):
    """DLS link-graph cache file (retrieval.py:72-79): explicit path, name / default stem inside the
    feature-DB directory, always .npz (np.savez appends it to any other name)."""
    from mmr_amd.retrieval import DLSRetrievalEngine
    f = str(tmp_path / "emb" / "train_joint_embeddings.npy")
    monkeypatch.delenv("MMR_FEATURE_DB_DIR", raising=False)
    cp = DLSRetrievalEngine.cache_path
    assert cp(f) == str(tmp_path / "emb" / "train_joint_embeddings_link_graph.npz")
    assert cp(f, name="graph_cache") == str(tmp_path / "emb" / "graph_cache.npz")
    assert cp(f, fdb_path=str(tmp_path / "x.pkl")) == str(tmp_path / "x.npz")
    assert cp(f, fdb_path=str(tmp_path / "y")) == str(tmp_path / "y.npz")
    monkeypatch.setenv("MMR_FEATURE_DB_DIR", str(tmp_path / "fdb"))
    assert cp(f) == str(tmp_path / "fdb" / "train_joint_embeddings_link_graph.npz")
    assert cp(None, name="g") == str(tmp_path / "fdb" / "g.npz")
    assert (tmp_path / "fdb").is_dir()
    monkeypatch.delenv("MMR_FEATURE_DB_DIR")
    assert cp(None) is None


def _rerank_fixture(N, D, Q, DK):
    rng = np.random.default_rng(91)
    G, _ = synthetic.labelled_gallery(N, D, 92)
    G[4] = G[N - 2]                        # duplicate across shards
    glab = [set(rng.choice(12, size=int(rng.integers(0, 4)), replace=False).tolist()) for _ in range(N)]
    qlab = [set(rng.choice(12, size=int(rng.integers(1, 3)), replace=False).tolist()) for _ in range(Q)]
    return G, glab, qlab, rng.standard_normal((N, DK)), rng.standard_normal((Q, DK))


def _worker_rerank(rank, world, port, N, D, b, K, DK, out_q):
    """Sharded rerank (config 5 at world > 1): the shard computes its candidates' raw components,
    they ride through the all-gather and the host payload merge, the mix runs on the merged list."""
    from oracle import dls as odls
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, glab, qlab, gkg, qkg = _rerank_fixture(N, D, world * b, DK)
        Q, _ = synthetic.labelled_gallery(world * b, D, 93)
        s, e = shard_bounds(N, world)[rank]

        def local(q, k):
            i, sc = oknn.exact_topk(q.numpy(), G[s:e], k)
            return torch.from_numpy(np.where(i >= 0, i + s, -1).astype(np.int64)), torch.from_numpy(sc)

        def comps(q, cand):
            out = np.zeros(tuple(cand.shape) + (3,))
            for qi in range(cand.shape[0]):
                for c in range(cand.shape[1]):
                    g = int(cand[qi, c])
                    if g >= 0:
                        assert s <= g < e  # a shard only scores its own rows
                        out[qi, c] = (odls._cos(q[qi].numpy().astype(np.float64), G[g].astype(np.float64)),
                                      odls._jac(qlab[qi], glab[g]), odls._cos(qkg[qi], gkg[g]))
            return torch.from_numpy(out)

        sh = ShardedIndex(G[s:e], N, s, local_search=local, local_components=comps)
        out = sh.search_rerank(torch.from_numpy(Q[rank * b:(rank + 1) * b]), K, topk=K - 2)
        out_q.put((rank,) + tuple(t.numpy() for t in out))
    finally:
        dist.destroy_process_group()


def test_sharded_rerank_world2_equals_single_list_rerank():
    """gloo world 2: the sharded rerank's (order, final, components) equal oracle/dls.rerank
    (reranker.py:240-333) over the single-device exact top-K list of every query."""
    from oracle import dls as odls
    world, N, D, b, K, DK = 2, 1501, 48, 6, 10, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_rerank, args=(r, world, port, N, D, b, K, DK, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    G, glab, qlab, gkg, qkg = _rerank_fixture(N, D, world * b, DK)
    Q, _ = synthetic.labelled_gallery(world * b, D, 93)
    ei, _ = oknn.exact_topk(Q, G, K)
    for rank, oi, fi, e, lab, kg in res:
        for r in range(b):
            qi = rank * b + r
            cand = ei[qi]
            order, final, re_, rl, rk = odls.rerank(Q[qi].astype(np.float64), G[cand], qlab[qi],
                                                    [glab[j] for j in cand], qkg[qi], gkg[cand], topk=K - 2)
            assert oi[r].tolist() == cand[order].tolist()
            np.testing.assert_allclose(fi[r], final, rtol=0, atol=1e-12)
            np.testing.assert_allclose(e[r], re_, rtol=0, atol=1e-12)
            np.testing.assert_allclose(lab[r], rl, rtol=0, atol=1e-12)
            np.testing.assert_allclose(kg[r], rk, rtol=0, atol=1e-12)
