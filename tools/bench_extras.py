"""Measurements of the SURVEY §8f rows beside the headline bench (one JSON line each):

  link_graph  DLS _build_link_graph (retrieval.py:121-138) as a GPU self-join over an N x D gallery
              (default 100k x 768, threshold 0.5, 10 links) -> cosine pairs/s and rows/s; CPU
              baseline = the reference's dense path restated (oracle/dls.py link_graph: f64 N x N
              cosine + per-row sort) on a bounded N.
  rerank      fused KG / label rerank (mmr_index_rerank) of Q queries x kc candidates -> queries/s;
              CPU baseline = oracle/dls.py rerank (the reference's per-query Python/numpy) on a sample.
usage: python tools/bench_extras.py [link_graph|rerank ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ev_time(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def bench_link_graph(n=100_000, d=768, thr=0.5, ml=10, cpu_n=4000):
    import numpy as np
    from mmr_amd import synthetic
    from mmr_amd.retrieval import GalleryIndex
    from oracle import dls as odls
    G, _ = synthetic.labelled_gallery(n, d, synthetic.SEED + 40)
    ix = GalleryIndex(G)
    t = ev_time(lambda: ix.link_graph(thr, ml), reps=3)
    nbr, cnt = ix.link_graph(thr, ml)
    avg_deg = float(cnt.float().mean().item())
    ix.close()
    t0 = time.perf_counter()
    odls.link_graph(G[:cpu_n], thr, ml)
    tc = time.perf_counter() - t0
    return {"bench": "link_graph", "n": n, "d": d, "threshold": thr, "max_links": ml, "seconds": t,
            "rows_per_s": n / t, "cosine_pairs_per_s": n * n / t, "avg_degree": avg_deg,
            "cpu_baseline": {"n": cpu_n, "seconds": tc, "cosine_pairs_per_s": cpu_n * cpu_n / tc,
                             "kind": "port", "what": "oracle/dls.py link_graph (f64 dense N x N + per-row sort)"}}


def bench_rerank(n=100_000, d=768, q=2048, kc=64, topk=10, dk=300, cpu_q=64):
    import numpy as np
    import torch
    from mmr_amd import synthetic
    from mmr_amd.retrieval import GalleryIndex
    from oracle import dls as odls
    rng = np.random.default_rng(7)
    G, gl = synthetic.labelled_gallery(n, d, synthetic.SEED + 41)
    ix = GalleryIndex(G)
    dev = torch.device("cuda")
    qe = torch.from_numpy(G[:q]).to(dev)
    cand, _ = ix.search(qe, kc)
    bits = torch.from_numpy(synthetic.labels_to_bits(gl).view(np.int64)).to(dev)
    kg = torch.from_numpy(rng.standard_normal((n, dk)).astype(np.float32)).to(dev)
    t = ev_time(lambda: ix.rerank(qe, cand, bits[:q], bits, kg[:q], kg, topk), reps=10)
    # CPU: the reference's per-query loop restated
    c = cand[:cpu_q].cpu().numpy()
    lsets = [set(np.nonzero(gl[i])[0].tolist()) for i in range(n)]
    kgh = kg.cpu().numpy()
    t0 = time.perf_counter()
    for i in range(cpu_q):
        odls.rerank(G[i], G[c[i]], lsets[i], [lsets[j] for j in c[i]], kgh[i], kgh[c[i]], topk=topk)
    tc = time.perf_counter() - t0
    ix.close()
    return {"bench": "rerank", "queries": q, "candidates": kc, "topk": topk, "d": d, "kg_dim": dk,
            "seconds": t, "queries_per_s": q / t,
            "cpu_baseline": {"queries": cpu_q, "queries_per_s": cpu_q / tc, "kind": "port",
                             "what": "oracle/dls.py rerank (per-query numpy, as reranker.py:240-333)"}}


if __name__ == "__main__":
    import torch
    torch.cuda.set_device(0)
    which = sys.argv[1:] or ["link_graph", "rerank"]
    for w in which:
        print(json.dumps({"link_graph": bench_link_graph, "rerank": bench_rerank}[w]()), flush=True)
