"""GPU: the native fp16 gallery index (mmr_index_create with MMR_F16, BASELINE config 5's "fp16
gallery").  The raw fp16 rows are the index's only device copy (tile32h: the operand of every fp16
scan, and the exact rows of the f64 re-score — fp16 is exact in f64), so an fp16 gallery costs 2 B per
element + norms on the device instead of f32 rows + fp16 copies.  The reference loads the gallery with
.astype("float32") (src/Retrieval/retrieval.py:24-32): the bar is bit-identical results to an index of
the f32-upcast rows (indices and f64 scores), on every scan path (lq / gmax / tile / p8 passes), with
exact duplicates, zero rows, K = 10 / 50, dims that are not chunk multiples and > 1024."""
import numpy as np
import pytest
import torch

from mmr_amd import synthetic
from mmr_amd.retrieval import GalleryIndex, MI355XRetrievalEngine
from oracle import knn as oknn

pytestmark = pytest.mark.gpu


def _gallery16(N, D, seed):
    G = synthetic.gauss_gallery(N, D, seed).astype(np.float16)
    G[5] = G[N - 3]           # exact duplicate: tie broken by the lower index
    G[11] = 0                 # zero row: score 0
    G[12] = G[13] * np.float16(2)  # parallel rows: equal cosine
    return G


@pytest.mark.parametrize("N,D", [(20_011, 768), (9_000, 200), (7_001, 100), (5_003, 1100)])
@pytest.mark.parametrize("K", [10, 50])
def test_native_f16_equals_f32_upcast_every_path(N, D, K):
    G16 = _gallery16(N, D, 700 + D)
    G32 = G16.astype(np.float32)
    ix16 = GalleryIndex(G16)
    assert ix16.native_f16 and ix16.mode == "f16"
    ixa = GalleryIndex(G32, mode="f16")
    ixb = GalleryIndex(G32, mode="x3")
    for Q in (1, 16, 17, 32, 33, 64, 129, 256, 300, 700, 1100):
        Qm = synthetic.gauss_gallery(Q, D, 800 + Q)
        Qm[0] = G32[13]
        q = torch.from_numpy(Qm).cuda()
        i16, _, s16, st = ix16.search(q, K, want_f64=True, want_status=True)
        ia, _, sa = ixa.search(q, K, want_f64=True)
        ib, _, sb = ixb.search(q, K, want_f64=True)
        assert int(st.max()) == 0
        assert torch.equal(i16, ia) and torch.equal(s16, sa), (Q, D, K)
        assert torch.equal(i16, ib) and torch.equal(s16, sb), (Q, D, K)
        if Q in (1, 33, 300):
            ei, es = oknn.exact_topk(Qm, G32, K)
            np.testing.assert_array_equal(i16.cpu().numpy(), ei)
    for x in (ix16, ixa, ixb):
        x.close()


def test_native_f16_explicit_other_mode_is_refused():
    """An fp16 gallery asked for an x3 / f32 index raises (it would otherwise become a silently f16-only
    index: ADVICE r04); the default mode of fp16 rows (numpy or torch) is f16."""
    G16 = _gallery16(3_000, 128, 7)
    for bad in ("x3", "f32"):
        with pytest.raises(ValueError, match="native fp16"):
            GalleryIndex(G16, mode=bad)
        with pytest.raises(ValueError, match="native fp16"):
            GalleryIndex(torch.from_numpy(G16).cuda(), mode=bad)
    ix = GalleryIndex(torch.from_numpy(G16).cuda())
    assert ix.native_f16 and ix.mode == "f16"
    ix.close()


def test_native_f16_device_bytes_and_modes():
    """1M x 1024 fp16 gallery: 2 B per element + f32 / f64 norms on the device (the f32 index needs
    4 B rows + the 2-B scan copy); x3 / f32 modes (which need f32 rows) are refused."""
    N, D = 1_000_000, 1024
    G16 = synthetic.gauss_gallery(N, D, synthetic.SEED + 70).astype(np.float16)
    ix = GalleryIndex(G16)
    g, _ = ix.device_bytes()
    Np = -(-N // 256) * 256
    assert g == Np * D * 2 + Np * 12
    with pytest.raises(ValueError):
        ix.set_mode("x3")
    with pytest.raises(ValueError):
        ix.set_mode("f32")
    q = torch.from_numpy(synthetic.gauss_gallery(2048, D, synthetic.SEED + 71)).cuda()
    i, _, s64 = ix.search(q, 10, want_f64=True)
    ix.close()
    # cfg5 shape against the f32-upcast index in its fp16 scan mode (same exact ranking)
    ixa = GalleryIndex(G16.astype(np.float32), mode="f16")
    ia, _, sa = ixa.search(q, 10, want_f64=True)
    ixa.close()
    assert torch.equal(i, ia) and torch.equal(s64, sa)


def test_native_f16_rerank_and_link_graph_equal_f32():
    """The fused KG / label rerank and the DLS link graph read the raw fp16 rows: equal to the
    f32-upcast index."""
    N, D, Q, K, DK = 12_007, 256, 64, 16, 32
    G16 = _gallery16(N, D, 710)
    G32 = G16.astype(np.float32)
    rng = np.random.default_rng(711)
    dev = torch.device("cuda")
    gb = torch.from_numpy(rng.integers(0, 1 << 20, size=N).astype(np.int64)).to(dev)
    qb = torch.from_numpy(rng.integers(0, 1 << 20, size=Q).astype(np.int64)).to(dev)
    gk = torch.from_numpy(rng.standard_normal((N, DK), dtype=np.float32)).to(dev)
    qk = torch.from_numpy(rng.standard_normal((Q, DK), dtype=np.float32)).to(dev)
    q = torch.from_numpy(synthetic.gauss_gallery(Q, D, 712)).to(dev)
    out = []
    for G in (G16, G32):
        ix = GalleryIndex(G, mode="f16")
        i = ix.search(q, K)[0]
        rr = ix.rerank(q, i, qb, gb, qk, gk, K)
        comp = ix.rerank_components(q, i, qb, gb, qk, gk)
        nbr, cnt = ix.link_graph(0.3, 8)
        out.append((i, rr, comp, nbr, cnt))
        ix.close()
    (i1, r1, c1, n1, k1), (i2, r2, c2, n2, k2) = out
    assert torch.equal(i1, i2) and torch.equal(c1, c2) and torch.equal(n1, n2) and torch.equal(k1, k2)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


def test_engine_fp16_npy_builds_native_index(tmp_path):
    """make_retrieval_engine-style construction from an fp16 .npy (cfg5's gallery file): the engine
    builds the native index, exposes the reference's f32 `embs`, and retrieves exactly what the fp32
    engine over the upcast rows retrieves."""
    import json
    N, D = 4_001, 384
    G16 = _gallery16(N, D, 720)
    fp, ip = tmp_path / "g16.npy", tmp_path / "ids.json"
    np.save(fp, G16)
    ip.write_text(json.dumps([f"r{i}" for i in range(N)]))
    e16 = MI355XRetrievalEngine(str(fp), str(ip), dtype="fp16")
    e32 = MI355XRetrievalEngine(embs=G16.astype(np.float32), ids=[f"r{i}" for i in range(N)], dtype="fp32")
    assert e16.index.native_f16 and e16.embs.dtype == np.float32
    Qm = synthetic.gauss_gallery(40, D, 721)
    a, sa = e16.search(Qm, 10)
    b, sb = e32.search(Qm, 10)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(sa, sb)
    assert e16.retrieve(Qm[3], K=5) == e32.retrieve(Qm[3], K=5)
    e16.close()
    e32.close()
