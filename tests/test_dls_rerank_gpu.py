"""GPU: DLS link graph (exact self-join, mmr_index_link_graph), the DLS engine (GPU graph + the
reference's host walk), the fused KG / label reranker (mmr_index_rerank) and the gallery writer —
against the reference's own outputs (tests/golden/dls_rerank.npz) and the oracle (oracle/dls.py).

Bars: link graphs identical to the oracle's exact-f64 graph (bit-exact neighbour lists) and
tie-aware equal to the reference's (its argsort order inside exact ties is unspecified); walk results
identical to the reference; rerank orders identical up to runs of equal final scores, scores within
1e-6 (the reference's own KG mean-pooling order noise is 6e-8)."""
import json
import os

import numpy as np
import pytest
import torch

import mmr_amd
from mmr_amd import synthetic
from mmr_amd.retrieval import GalleryIndex
from oracle import dls as odls
from oracle import knn as oknn

from conftest import GOLDEN
from test_oracle_dls import graph_from, graphs_equivalent, rerank_tables

pytestmark = pytest.mark.gpu


def _fixture():
    f = np.load(os.path.join(GOLDEN, "dls_rerank.npz"), allow_pickle=False)
    G, gl = synthetic.dls_gallery()
    return f, G, gl


@pytest.mark.parametrize("tag,thr,ml", [("t50_m10", 0.5, 10), ("t30_m8", 0.3, 8)])
@pytest.mark.parametrize("mode", ["x3", "f32"])
def test_link_graph_vs_reference_and_oracle(tag, thr, ml, mode):
    f, G, _ = _fixture()
    ix = GalleryIndex(G, mode=mode)
    nbr, cnt = ix.link_graph(thr, ml, batch=500)      # several row batches
    nbr, cnt = nbr.cpu().numpy(), cnt.cpu().numpy()
    got = [nbr[i, :cnt[i]].tolist() for i in range(len(G))]
    assert (nbr[np.arange(ml)[None, :] >= cnt[:, None]] == -1).all()
    assert got == odls.link_graph(G, thr, ml)
    ok, msg = graphs_equivalent(graph_from(f, tag), got, G, thr)
    assert ok, msg
    ix.close()


def test_link_graph_larger_vs_oracle():
    G, _ = synthetic.labelled_gallery(6000, 96, 31)       # d not a multiple of 64 (compact query copy)
    G[17] = 0.0
    G[100] = G[99]
    ix = GalleryIndex(G)
    nbr, cnt = ix.link_graph(0.4, 12)
    nbr, cnt = nbr.cpu().numpy(), cnt.cpu().numpy()
    got = [nbr[i, :cnt[i]].tolist() for i in range(len(G))]
    assert got == odls.link_graph(G, 0.4, 12)
    ix.close()


def test_dls_engine_walk_matches_reference(tmp_path):
    f, G, _ = _fixture()
    np.save(tmp_path / "g.npy", G)
    (tmp_path / "ids.json").write_text(json.dumps([f"r{i}" for i in range(len(G))]))
    eng = mmr_amd.make_retrieval_engine(str(tmp_path / "g.npy"), str(tmp_path / "ids.json"), method="dls",
                                        link_threshold=0.5, max_links=10, fdb_path=str(tmp_path / "graph.pkl"))
    assert os.path.exists(tmp_path / "graph.npz")          # cache written as .npz, never a pickle
    ref_graph = graph_from(f, "t50_m10")
    # the engine's own (GPU) graph is the reference's up to the order inside exact ties
    ok, msg = graphs_equivalent(ref_graph, eng.link_graph, G, 0.5)
    assert ok, msg
    own_graph = eng.link_graph
    # the walk is compared on the reference's own graph, so every query is compared (a tie-reordered
    # neighbour list may legitimately change the greedy walk's path)
    eng.link_graph = ref_graph
    Qm, _ = synthetic.labelled_gallery(synthetic.DLS_Q, synthetic.DLS_D, synthetic.SEED + 12)
    compared = 0
    for qi in range(synthetic.DLS_Q):
        ids, sc = eng.retrieve(Qm[qi], K=5, seed=synthetic.SEED + qi)
        n = len(ids)
        assert n == min(5, len(f["walk_idx"][qi]))
        assert [int(x[1:]) for x in ids] == f["walk_idx"][qi][:n].tolist()
        np.testing.assert_allclose(sc, f["walk_score"][qi][:n], rtol=0, atol=1e-6)
        compared += 1
    assert compared == synthetic.DLS_Q
    eng.link_graph = own_graph
    # the cache is re-used (same graph, no rebuild)
    eng2 = mmr_amd.DLSRetrievalEngine(str(tmp_path / "g.npy"), str(tmp_path / "ids.json"),
                                      fdb_path=str(tmp_path / "graph.pkl"))
    assert eng2.link_graph == eng.link_graph
    eng.close()
    eng2.close()


def _write_kg(tmp_path, f, gl):
    import pandas as pd
    kg = tmp_path / "kg"
    kg.mkdir()
    (kg / "node2id.json").write_text(bytes(f["kg_node2id"]).decode())
    np.save(kg / "node_embeddings_best.npy", f["kg_node_emb"])
    df = pd.DataFrame(gl.astype(np.int64), columns=synthetic.LABEL_NAMES)
    df.insert(0, "id", [f"r{i}" for i in range(len(gl))])
    df["report"] = ["text"] * len(gl)
    df.to_csv(tmp_path / "labels.csv", index=False)
    return kg, tmp_path / "labels.csv"


def _assert_rerank(order_idx, final, e, l, k, f, qn):
    np.testing.assert_allclose(final, f["rr_final"][qn], rtol=0, atol=1e-6)
    np.testing.assert_allclose(e, f["rr_emb"][qn], rtol=0, atol=1e-6)
    np.testing.assert_allclose(l, f["rr_lab"][qn], rtol=0, atol=1e-12)
    np.testing.assert_allclose(k, f["rr_kg"][qn], rtol=0, atol=1e-6)
    ref = f["rr_order"][qn].tolist()
    if list(order_idx) != ref:
        fr = f["rr_final"][qn]
        for p in range(len(ref)):
            if order_idx[p] != ref[p]:
                tied = np.abs(fr - fr[p]) <= 1e-9
                assert set(np.array(order_idx)[tied]) == set(np.array(ref)[tied])


def test_reranker_single_query_api_matches_reference(tmp_path):
    f, G, gl = _fixture()
    kg, csv = _write_kg(tmp_path, f, gl)
    R = mmr_amd.Reranker(kg_dir=kg, labels_csv=csv)
    ids = [f"r{i}" for i in range(len(G))]
    for qn, qi in enumerate(f["rr_queries"]):
        cand = f["rr_cand"][qn]
        cids = [ids[j] for j in cand]
        lookup = {c: G[j] for c, j in zip(cids, cand)}
        lookup[ids[qi]] = G[qi]
        out = R.rerank(ids[qi], cids, candidate_embs=G[cand], candidate_emb_lookup=lookup, topk=10)
        _assert_rerank([int(t[0][1:]) for t in out], [t[1] for t in out], [t[2] for t in out],
                       [t[3] for t in out], [t[4] for t in out], f, qn)


def test_fused_search_rerank_batch_matches_reference(tmp_path):
    """Device path: exact top-15 search -> fused rerank on device for all queries at once."""
    f, G, gl = _fixture()
    kg, csv = _write_kg(tmp_path, f, gl)
    ids = [f"r{i}" for i in range(len(G))]
    eng = mmr_amd.MI355XRetrievalEngine(embs=G, ids=ids)
    R = mmr_amd.Reranker(kg_dir=kg, labels_csv=csv).bind(eng)
    qrows = f["rr_queries"]
    q = torch.from_numpy(G[qrows]).cuda()
    cand, csc = eng.search(q, K=15)
    # (a) the fused rerank on the reference's own candidate lists: every query compared
    ref_cand = torch.from_numpy(np.ascontiguousarray(f["rr_cand"], np.int64)).cuda()
    oi, fi, e, l, k = R.rerank_batch(eng, q, [ids[i] for i in qrows], ref_cand, topk=10)
    oi, fi, e, l, k = (t.cpu().numpy() for t in (oi, fi, e, l, k))
    for qn in range(len(qrows)):
        _assert_rerank(oi[qn].tolist(), fi[qn], e[qn], l[qn], k[qn], f, qn)
    # (b) the device search's candidate sets equal the reference's top-15 except inside exact ties at
    # the cut; count how many needed the tie allowance
    ex = oknn.exact_scores(G[qrows], G)
    tied = 0
    for qn in range(len(qrows)):
        got, ref = set(cand[qn].tolist()), set(f["rr_cand"][qn].tolist())
        if got == ref:
            continue
        cut = float(csc[qn, -1])
        diff = got ^ ref
        assert all(abs(ex[qn, j] - cut) <= 1e-6 for j in diff), f"query {qn}: candidate sets differ off-tie"
        tied += 1
    assert tied <= 2
    # (c) the fused rerank on the device's own candidates vs the oracle on the same lists
    _, fi2, *_ = R.rerank_batch(eng, q, [ids[i] for i in qrows], cand, topk=10)
    fi2 = fi2.cpu().numpy()
    _, lsets, kgv = rerank_tables(f, G, gl)
    c = cand.cpu().numpy()
    for qn, qi in enumerate(qrows):
        order, final, *_ = odls.rerank(G[qi], G[c[qn]], lsets[qi], [lsets[j] for j in c[qn]], kgv[qi], kgv[c[qn]],
                                       topk=10)
        np.testing.assert_allclose(fi2[qn], final, rtol=0, atol=1e-9)
    eng.close()


def test_build_gallery_files(tmp_path):
    from mmr_amd.gallery import build_gallery, merge_galleries
    from mmr_amd.model import MultiModalRetrievalModel
    from mmr_amd.towers import BERT_BASE, SWIN_T
    scfg = dict(SWIN_T, embed_dim=32, depths=[2, 2, 2, 2], num_heads=[1, 2, 4, 8])
    bcfg = dict(BERT_BASE, vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                intermediate_size=512)
    m = MultiModalRetrievalModel(joint_dim=64, model_type="text", swin_cfg=scfg, bert_cfg=bcfg, device="cuda",
                                 training=True, pretrained=False)
    batches = []
    for b in range(3):
        img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(4, 50 + b)))
        ii, mm = (torch.from_numpy(x) for x in synthetic.reports(4, 128, 60 + b, vocab=1000))
        batches.append((img, ii, mm, [f"s{b}_{j}" for j in range(4)]))
    embs, ids = build_gallery(m, batches, tmp_path, split="train")
    build_gallery(m, batches[:1], tmp_path, split="val")
    ref = torch.cat([m(img.cuda(), ii.cuda(), mm.cuda())["joint_emb"].float().cpu() for img, ii, mm, _ in batches])
    assert torch.equal(torch.from_numpy(np.load(tmp_path / "train_joint_embeddings.npy")), ref)
    assert json.load(open(tmp_path / "train_ids.json")) == ids and len(ids) == 12
    me, mi = merge_galleries(tmp_path)
    assert me.shape == (16, 64) and mi == ids + ids[:4]
    eng = mmr_amd.make_retrieval_engine(str(tmp_path / "trainval_joint_embeddings.npy"),
                                        str(tmp_path / "trainval_ids.json"), method="mi355x")
    r_ids, r_sc = eng.retrieve(me[3], K=2)
    assert r_ids == [ids[3], ids[3]] and abs(r_sc[0] - 1.0) < 1e-6  # row 3 and its duplicate row 15
    eng.close()
