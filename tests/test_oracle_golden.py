"""CPU: the oracle (and the host-side metric code) against vectors produced by the reference
itself (tests/golden/make_golden.py).  No GPU, no native library."""
import json
import os

import numpy as np
import pytest
import torch

import mmr_amd
from mmr_amd import metrics, synthetic
from oracle import knn as oknn
from oracle import towers as otw

from conftest import GOLDEN


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def _regen(f):
    N, D, Q, seed, kind = int(f["N"]), int(f["D"]), int(f["Q"]), int(f["seed"]), str(f["kind"])
    if kind == "gauss":
        G = synthetic.gauss_gallery(N, D, seed)
        Qm = synthetic.gauss_gallery(Q, D, seed + 1)
    else:
        G, _ = synthetic.labelled_gallery(N, D, seed)
        Qm, _ = synthetic.labelled_gallery(Q, D, seed + 1)
        G[f["zero_rows"]] = 0.0
    assert np.isclose(G.astype(np.float64).sum(), float(f["g_sum"]), rtol=0, atol=1e-6)
    assert np.isclose(Qm.astype(np.float64).sum(), float(f["q_sum"]), rtol=0, atol=1e-6)
    return G, Qm


@pytest.mark.parametrize("name", ["knn_gauss_1k", "knn_gauss_10k", "knn_labelled_2k"])
def test_oracle_knn_matches_reference(name):
    f = _load(name + ".npz")
    G, Qm = _regen(f)
    for key in f.files:
        if not key.startswith("idx_k"):
            continue
        K = int(key[5:])
        ref_i, ref_s = f[key], f[f"score_k{K}"]
        # restated sklearn path: identical up to f32 rounding ties
        si, ss = oknn.sklearn_topk(Qm, G, K)
        ok, msg = oknn.topk_equivalent(ref_i, ref_s, si, ss, tie_tol=1e-6, score_tol=1e-5)
        assert ok, msg
        # exact f64 semantics (what the GPU implements): same ranking under the parity criterion
        ei, es = oknn.exact_topk(Qm, G, K)
        ok, msg = oknn.topk_equivalent(ref_i, ref_s, ei, es, tie_tol=1e-6, score_tol=1e-4)
        assert ok, msg


def test_exact_topk_ties_and_small_n():
    G = np.zeros((5, 4), np.float32)
    G[0] = [1, 0, 0, 0]
    G[2] = [1, 0, 0, 0]
    G[3] = [0, 1, 0, 0]
    q = np.array([[1, 0, 0, 0]], np.float32)
    i, s = oknn.exact_topk(q, G, 10)
    assert i.shape == (1, 5)
    assert i[0, :2].tolist() == [0, 2]          # exact tie -> lower index first
    assert i[0, 2:].tolist() == [1, 3, 4]       # zero rows score 0, tie with the orthogonal row
    assert np.allclose(s[0], [1, 1, 0, 0, 0])


def test_ranking_metrics_match_reference():
    g = json.load(open(os.path.join(GOLDEN, "ranking.json")))
    G, gl = synthetic.labelled_gallery(g["n_gallery"], g["D"], g["seed_g"])
    Qm, ql = synthetic.labelled_gallery(g["n_query"], g["D"], g["seed_q"])
    idx, _ = oknn.exact_topk(Qm, G, g["n_gallery"])  # full ranking for the first-relevant rank
    qb, gb = synthetic.labels_to_bits(ql), synthetic.labels_to_bits(gl)
    for k, want in g["cases"].items():
        mrr, hit, rec = metrics.ranking_metrics(idx, qb, gb, int(k))
        assert mrr == pytest.approx(want["mrr"], abs=1e-12)
        assert hit == pytest.approx(want["hit_at_k"], abs=1e-12)
        assert rec == pytest.approx(want["recall_at_k"], abs=1e-12)


def test_id_list_metrics_match_reference():
    m = json.load(open(os.path.join(GOLDEN, "ranking.json")))["metrics"]
    for (ret, rel), row in zip(m["lists"], m["per_list"]):
        rs = set(rel)
        for k in (1, 5, 10, 20):
            assert metrics.precision_at_k(ret, rel, k) == pytest.approx(row[f"p@{k}"], abs=1e-15)
            assert metrics.recall_at_k(ret, rel, k) == pytest.approx(row[f"r@{k}"], abs=1e-15)
            assert metrics.ndcg_at_k(ret, rel, k) == pytest.approx(row[f"ndcg@{k}"], abs=1e-12)
        assert metrics.average_precision(ret, rs) == pytest.approx(row["ap"], abs=1e-15)
        assert metrics.average_precision(ret, rs, 10) == pytest.approx(row["ap@10"], abs=1e-15)
    L = [r for r, _ in m["lists"]]
    S = [set(x) for _, x in m["lists"]]
    assert metrics.mean_average_precision(L, S) == pytest.approx(m["map"], abs=1e-15)
    assert metrics.mean_average_precision(L, S, 10) == pytest.approx(m["map@10"], abs=1e-15)
    assert metrics.mean_reciprocal_rank(L, S) == pytest.approx(m["mrr"], abs=1e-15)


def mini_towers():
    f = _load("towers_mini.npz")
    cfg = json.loads(bytes(f["cfg"]).decode())
    w = {k[2:]: torch.from_numpy(synthetic.bf16_bits_to_f32(f[k]).copy()) for k in f.files if k.startswith("w:")}
    swin = {k[5:]: v for k, v in w.items() if k.startswith("swin.")}
    bert = {k[5:]: v for k, v in w.items() if k.startswith("bert.")}
    head = {k[5:]: v for k, v in w.items() if k.startswith("head.")}
    image = torch.from_numpy(synthetic.image_from_u8(f["img_u8"]))
    ids = torch.from_numpy(f["input_ids"])
    mask = torch.from_numpy(f["attention_mask"])
    return f, cfg, swin, bert, head, image, ids, mask


def test_oracle_towers_match_reference():
    f, cfg, swin, bert, head, image, ids, mask = mini_towers()
    with torch.no_grad():
        (g, p), t = otw.backbones_forward(image, ids, mask, swin, bert, cfg["swin"], cfg["bert"])
    np.testing.assert_allclose(g.numpy(), f["img_global"], atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(p.numpy(), f["img_patches"], atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(t.numpy(), f["txt_feats"], atol=2e-4, rtol=1e-4)
    with torch.no_grad():
        for mt in ("text", "image"):
            o = otw.heads(torch.from_numpy(f["img_global"]), torch.from_numpy(f["img_patches"]),
                          torch.from_numpy(f["txt_feats"]), head, mt)
            np.testing.assert_allclose(o["joint_emb"].numpy(), f[f"{mt}_joint_emb"], atol=1e-5, rtol=1e-5)
            np.testing.assert_allclose(o["img_emb"].numpy(), f[f"{mt}_img_emb"], atol=1e-5, rtol=1e-5)
            np.testing.assert_allclose(o["txt_emb"].numpy(), f[f"{mt}_txt_emb"], atol=1e-5, rtol=1e-5)
        # multimodal: 2 fusion layers x CrossModalFusion + combiner (model.py:375-459)
        o = otw.heads(torch.from_numpy(f["img_global"]), torch.from_numpy(f["img_patches"]),
                      torch.from_numpy(f["txt_feats"]), head, "multimodal", mm_cfg={"num_heads": cfg["num_heads"]})
        np.testing.assert_allclose(o["joint_emb"].numpy(), f["multimodal_joint_emb"], atol=1e-5, rtol=1e-5)


def test_oracle_multimodal_cls_only_raises_like_reference():
    f, cfg, swin, bert, head, image, ids, mask = mini_towers()
    with pytest.raises(ValueError):
        otw.multimodal(torch.from_numpy(f["img_global"]), torch.from_numpy(f["img_patches"]),
                       torch.from_numpy(f["txt_feats"]), head, num_heads=4, use_cls_only=True)


def test_package_imports_without_gpu():
    assert hasattr(mmr_amd, "make_retrieval_engine")
    with pytest.raises(ValueError):
        mmr_amd.make_retrieval_engine("x.npy", "x.json", method="nope")


def test_mxfp8_oracle_rounding_matches_torch_float8():
    """The MX-fp8 oracle's e4m3 round-to-nearest-even and byte decode (oracle/mxfp8.py) equal torch's
    own float8_e4m3fn conversion on 200k values over 6 decades, and all 256 byte codes."""
    import torch
    from oracle import mxfp8 as mx
    rng = np.random.default_rng(0)
    v = np.clip((rng.standard_normal(200_000) * rng.choice([1e-3, 1.0, 30.0, 200.0], 200_000)).astype(np.float32),
                -448, 448)
    np.testing.assert_array_equal(mx.e4m3_round(v), torch.from_numpy(v).to(torch.float8_e4m3fn).float().numpy())
    b = np.arange(256, dtype=np.uint8)
    np.testing.assert_array_equal(mx.e4m3_decode(b), torch.from_numpy(b).view(torch.float8_e4m3fn).float().numpy())
    # block exponents: amax exactly 448 * 2^e -> e; one ulp above -> e + 1; zero block -> -127
    x = np.zeros((3, 32), np.float32)
    x[0, 5] = 448.0 * 4
    x[1, 7] = np.nextafter(np.float32(448.0 * 4), np.float32(1e9))
    np.testing.assert_array_equal(mx.block_exponents(x)[:, 0], [2, 3, -127])
