"""CPU: the DLS link-graph / walk / Reranker restatements (oracle/dls.py) against the reference's own
outputs (tests/golden/dls_rerank.npz, written by tests/golden/make_golden.py from
src/Retrieval/retrieval.py and src/Retrieval/reranker.py).  No GPU, no native library."""
import json
import os

import numpy as np
import pytest

from mmr_amd import synthetic
from oracle import dls as odls
from oracle import knn as oknn

from conftest import GOLDEN


def _fixture():
    f = np.load(os.path.join(GOLDEN, "dls_rerank.npz"), allow_pickle=False)
    G, gl = synthetic.dls_gallery()
    assert np.isclose(G.astype(np.float64).sum(), float(f["g_sum"]), rtol=0, atol=1e-6)
    return f, G, gl


def graph_from(f, tag):
    o, flat = f[f"graph_{tag}_offsets"], f[f"graph_{tag}_flat"]
    return [flat[o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)]


def graphs_equivalent(ref, got, G, threshold, tie_tol=1e-6):
    """Identical neighbour lists, except (a) runs of tied similarities (the reference's argsort is
    unstable) compared as sets and (b) neighbours within tie_tol of the threshold."""
    S = None
    for i, (a, b) in enumerate(zip(ref, got)):
        if a == b:
            continue
        if S is None:
            S = oknn.exact_scores(G, G)
        s = S[i]
        ok_a = {j for j in a if abs(s[j] - threshold) > tie_tol}
        ok_b = {j for j in b if abs(s[j] - threshold) > tie_tol}
        last = min(s[j] for j in a) if a else None
        # sets may only differ in elements tied with the list's last score (truncation at max_links)
        diff = ok_a ^ ok_b
        if any(last is None or abs(s[j] - last) > tie_tol for j in diff):
            return False, f"row {i}: {a} vs {b}"
        # order must agree outside tie runs
        sa = [round(s[j], 6) for j in a]
        sb = [round(s[j], 6) for j in b]
        if sa[:len(sb)] != sb[:len(sa)]:
            return False, f"row {i}: score order {sa} vs {sb}"
    return True, "ok"


@pytest.mark.parametrize("tag,thr,ml", [("t50_m10", 0.5, 10), ("t30_m8", 0.3, 8)])
def test_oracle_link_graph_matches_reference(tag, thr, ml):
    f, G, _ = _fixture()
    ref = graph_from(f, tag)
    got = odls.link_graph(G, thr, ml)
    ok, msg = graphs_equivalent(ref, got, G, thr)
    assert ok, msg
    # zero rows have no links; the duplicate pair link to each other first
    assert got[synthetic.DLS_ZERO[0]] == [] and got[synthetic.DLS_ZERO[1]] == []
    a, b = synthetic.DLS_DUP
    assert got[a][0] == b and got[b][0] == a


def test_oracle_walk_matches_reference():
    f, G, _ = _fixture()
    graph = graph_from(f, "t50_m10")
    Qm, _ = synthetic.labelled_gallery(synthetic.DLS_Q, synthetic.DLS_D, synthetic.SEED + 12)
    for qi in range(synthetic.DLS_Q):
        idx, sc = odls.walk_retrieve(G, graph, Qm[qi], K=5, seed=synthetic.SEED + qi)
        n = len(idx)
        assert idx == f["walk_idx"][qi][:n].tolist()
        np.testing.assert_allclose(sc, f["walk_score"][qi][:n], rtol=0, atol=1e-6)


def rerank_tables(f, G, gl):
    ids = [f"r{i}" for i in range(len(G))]
    lsets = odls.label_sets(gl, synthetic.LABEL_NAMES)
    node2id = json.loads(bytes(f["kg_node2id"]).decode())
    kg = odls.record_kg_vectors(ids, lsets, node2id, f["kg_node_emb"])
    return ids, lsets, kg


def test_oracle_rerank_matches_reference():
    f, G, gl = _fixture()
    ids, lsets, kg = rerank_tables(f, G, gl)
    for qn, qi in enumerate(f["rr_queries"]):
        cand = f["rr_cand"][qn]
        order, final, e, l, k = odls.rerank(G[qi], G[cand], lsets[qi], [lsets[j] for j in cand], kg[qi], kg[cand],
                                            topk=10)
        np.testing.assert_allclose(final, f["rr_final"][qn], rtol=0, atol=1e-6)
        np.testing.assert_allclose(e, f["rr_emb"][qn], rtol=0, atol=1e-6)
        np.testing.assert_allclose(l, f["rr_lab"][qn], rtol=0, atol=1e-12)
        np.testing.assert_allclose(k, f["rr_kg"][qn], rtol=0, atol=1e-6)
        got = cand[order].tolist()
        ref = f["rr_order"][qn].tolist()
        if got != ref:  # only runs of (near-)equal final scores may be permuted
            fr = f["rr_final"][qn]
            for p in range(len(ref)):
                if got[p] != ref[p]:
                    tied = np.abs(fr - fr[p]) <= 1e-9
                    assert set(np.array(got)[tied]) == set(np.array(ref)[tied]), (qn, got, ref)
