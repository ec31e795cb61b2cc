"""GPU parity: libmmr batched-cosine top-K (mmr_index_search / mmr_merge_topk through the C ABI)
against the oracle (exact f64, bit-exact indices) and the reference's sklearn vectors (golden,
tie-aware).  Tolerances: indices bit-exact vs the exact oracle; scores within 1e-4 of sklearn and
within 1e-6 of the exact f64 scores (they are f64 rounded to f32)."""
import os

import numpy as np
import pytest
import torch

from mmr_amd import metrics, synthetic
from mmr_amd.retrieval import GalleryIndex, MI355XRetrievalEngine, merge_topk
from oracle import knn as oknn

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _search(G, Q, K, **kw):
    ix = GalleryIndex(G, **kw)
    q = torch.from_numpy(np.ascontiguousarray(Q, np.float32)).cuda()
    i, s, s64, st = ix.search(q, K, want_f64=True, want_status=True)
    torch.cuda.synchronize()
    ix.close()
    return i.cpu().numpy(), s.cpu().numpy(), s64.cpu().numpy(), st.cpu().numpy()


def _exact_check(G, Q, K, mode="x3"):
    gi, gs, g64, st = _search(G, Q, K, mode=mode)
    assert (st == 0).all()
    ei, es = oknn.exact_topk(Q, G, K)
    kk = ei.shape[1]
    np.testing.assert_array_equal(gi[:, :kk], ei)
    np.testing.assert_allclose(g64[:, :kk], es, rtol=0, atol=1e-12)
    np.testing.assert_allclose(gs[:, :kk], es.astype(np.float32), rtol=0, atol=0)
    if kk < K:
        assert (gi[:, kk:] == -1).all() and np.isneginf(gs[:, kk:]).all()
    return gi, gs


@pytest.mark.parametrize("name", ["knn_gauss_1k", "knn_gauss_10k", "knn_labelled_2k"])
def test_knn_matches_reference_golden(name):
    f = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    N, D, Q, seed, kind = int(f["N"]), int(f["D"]), int(f["Q"]), int(f["seed"]), str(f["kind"])
    if kind == "gauss":
        G, Qm = synthetic.gauss_gallery(N, D, seed), synthetic.gauss_gallery(Q, D, seed + 1)
    else:
        G, _ = synthetic.labelled_gallery(N, D, seed)
        Qm, _ = synthetic.labelled_gallery(Q, D, seed + 1)
        G[f["zero_rows"]] = 0.0
    for key in f.files:
        if key.startswith("idx_k"):
            K = int(key[5:])
            gi, gs = _exact_check(G, Qm, K)
            ok, msg = oknn.topk_equivalent(f[key], f[f"score_k{K}"], gi, gs, tie_tol=1e-6, score_tol=1e-4)
            assert ok, msg


@pytest.mark.parametrize("mode", ["x3", "f32", "f16"])
def test_knn_scan_modes_agree(mode):
    G = synthetic.gauss_gallery(20000, 768, 41)
    Qm = synthetic.gauss_gallery(200, 768, 42)
    _exact_check(G, Qm, 50, mode=mode)


@pytest.mark.parametrize("N,D,Q,K", [(1, 8, 3, 5), (7, 100, 1, 10), (300, 64, 65, 256), (1000, 1024, 129, 50),
                                     (5000, 768, 300, 10), (257, 24, 2, 1)])
def test_knn_shapes_and_edges(N, D, Q, K):
    rng = np.random.default_rng(N + D + Q + K)
    G = rng.standard_normal((N, D), dtype=np.float32)
    Qm = rng.standard_normal((Q, D), dtype=np.float32)
    _exact_check(G, Qm, K)


def test_knn_ties_zero_rows_and_duplicates():
    rng = np.random.default_rng(5)
    G = rng.standard_normal((2000, 128), dtype=np.float32)
    G[100:110] = G[50]          # exact duplicates -> equal scores -> index order
    G[200:205] = 0.0            # zero rows -> score 0
    Qm = np.concatenate([G[50:51] * 3.0, np.zeros((1, 128), np.float32),
                         -G[60:61], rng.standard_normal((5, 128), dtype=np.float32)])
    gi, gs = _exact_check(G, Qm, 20)
    assert gi[0, :11].tolist() == [50] + list(range(100, 110))
    assert gi[1].tolist() == list(range(20))  # zero query: every score 0 -> lowest indices


def test_knn_negative_scores_and_clustered():
    G, _ = synthetic.labelled_gallery(4000, 256, 11)
    G = -np.abs(G)                       # many negative cosines
    Qm = np.abs(synthetic.gauss_gallery(40, 256, 12))
    _exact_check(G, Qm, 64)


@pytest.mark.parametrize("Q", [1, 5, 16, 17, 32, 33, 64])
def test_knn_skinny_scan_query_tiles(Q):
    """Q <= 64 runs the HBM-streaming f32 skinny scan (1, 2 or 4 query tiles of 16); duplicates and
    padding rows (N not a multiple of 64) included."""
    rng = np.random.default_rng(100 + Q)
    G = rng.standard_normal((20_003, 768), dtype=np.float32)
    G[7000:7016] = G[3]
    Qm = np.concatenate([G[3:4] * 0.5, rng.standard_normal((Q - 1, 768), dtype=np.float32)])
    gi, _ = _exact_check(G, Qm, 25)
    assert gi[0, :17].tolist() == [3] + list(range(7000, 7016))


@pytest.mark.parametrize("Q", [1, 64])
def test_knn_100k_skinny_exact(Q):
    G = synthetic.gauss_gallery(100_000, 768, synthetic.SEED)
    Qm = synthetic.gauss_gallery(Q, 768, synthetic.SEED + 2)
    _exact_check(G, Qm, 10)


@pytest.mark.parametrize("Q", [1, 16, 17, 33, 64, 65, 128, 256, 300])
def test_knn_f16_scan_query_tiles(Q):
    """fp16 scan (mode f16): every QT in {1,2,4,8,16} and a second 256-query pass; duplicates,
    padding rows and a zero row; exact indices and f64 scores as the other modes."""
    rng = np.random.default_rng(300 + Q)
    G = rng.standard_normal((10_007, 768), dtype=np.float32)
    G[5000:5008] = G[3]
    G[9000] = 0.0
    Qm = np.concatenate([G[3:4] * 2.0, rng.standard_normal((Q - 1, 768), dtype=np.float32)])
    gi, _ = _exact_check(G, Qm, 20, mode="f16")
    assert gi[0, :9].tolist() == [3] + list(range(5000, 5008))


@pytest.mark.parametrize("D", [8, 24, 150, 200, 1000])
@pytest.mark.parametrize("Q", [1, 20, 40, 130])
def test_knn_f16_dims_not_multiple_of_chunk(D, Q):
    """fp16 scan with padded dims Dp = 64 / 192 / 256 / 1024: every chunk width must divide Dp."""
    rng = np.random.default_rng(D * 1000 + Q)
    G = rng.standard_normal((3000 + D, D), dtype=np.float32)
    Qm = rng.standard_normal((Q, D), dtype=np.float32)
    _exact_check(G, Qm, 10, mode="f16")


@pytest.mark.parametrize("D", [8, 150])
def test_knn_skinny_dims(D):
    rng = np.random.default_rng(D)
    G = rng.standard_normal((2500, D), dtype=np.float32)
    _exact_check(G, rng.standard_normal((5, D), dtype=np.float32), 10)
    _exact_check(G, rng.standard_normal((30, D), dtype=np.float32), 10)


def test_knn_f16_labelled_and_negative():
    G, _ = synthetic.labelled_gallery(4000, 256, 11)
    Qm, _ = synthetic.labelled_gallery(50, 256, 12)
    _exact_check(G, Qm, 64, mode="f16")
    _exact_check(-np.abs(G), np.abs(Qm), 10, mode="f16")


def test_knn_100k_f16_exact():
    G = synthetic.gauss_gallery(100_000, 768, synthetic.SEED)
    Qm = synthetic.gauss_gallery(256, 768, synthetic.SEED + 1)
    _exact_check(G, Qm, 10, mode="f16")


def test_engine_fp16_gallery_matches_fp32_engine():
    G, _ = synthetic.labelled_gallery(3000, 128, 21)
    G[100:140] = G[7]                     # 40 exact ties: f16 margin may overflow -> x3 redo
    Qm = np.concatenate([G[7:8], synthetic.labelled_gallery(20, 128, 22)[0]])
    ids = [str(i) for i in range(len(G))]
    e32 = MI355XRetrievalEngine(embs=G, ids=ids)
    e16 = MI355XRetrievalEngine(embs=G, ids=ids, dtype="fp16")
    a_i, a_s = e32.search(Qm, K=50)
    b_i, b_s = e16.search(Qm, K=50)
    np.testing.assert_array_equal(a_i, b_i)
    np.testing.assert_array_equal(a_s, b_s)
    e32.close()
    e16.close()


def test_knn_100k_full_size_exact():
    G = synthetic.gauss_gallery(100_000, 768, synthetic.SEED)
    Qm = synthetic.gauss_gallery(256, 768, synthetic.SEED + 1)
    _exact_check(G, Qm, 10)


def test_shard_merge_equals_single_index():
    G, _ = synthetic.labelled_gallery(6000, 192, 21)
    Qm, _ = synthetic.labelled_gallery(70, 192, 22)
    K = 10
    si, ss, s64, _ = _search(G, Qm, K)
    bounds = [0, 1000, 1001, 4000, 6000]   # ragged shards, one with a single row (< K)
    idxs, scs = [], []
    q = torch.from_numpy(Qm).cuda()
    for a, b in zip(bounds[:-1], bounds[1:]):
        ix = GalleryIndex(G[a:b], idx_base=a)
        i, s, sd = ix.search(q, K, want_f64=True)
        idxs.append(i)
        scs.append(sd)
    mi, ms, m64 = merge_topk(torch.stack(scs), torch.stack(idxs), K)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mi.cpu().numpy(), si)
    np.testing.assert_array_equal(m64.cpu().numpy(), s64)


def test_engine_retrieve_contract_and_precision_at_10(tmp_path):
    G, gl = synthetic.labelled_gallery(3000, 768, 31)
    Qm, ql = synthetic.labelled_gallery(64, 768, 32)
    ids = [f"case{i}" for i in range(len(G))]
    np.save(tmp_path / "g.npy", G)
    (tmp_path / "ids.json").write_text(__import__("json").dumps(ids))
    from mmr_amd import make_retrieval_engine
    eng = make_retrieval_engine(str(tmp_path / "g.npy"), str(tmp_path / "ids.json"), method="mi355x")
    r_ids, r_scores = eng.retrieve(Qm[0], K=5)
    assert len(r_ids) == 5 and all(isinstance(x, str) for x in r_ids)
    assert r_scores == sorted(r_scores, reverse=True)
    gi, gs = eng.search(Qm, K=10)
    si, ss = oknn.sklearn_topk(Qm, G, 10)
    qb, gb = synthetic.labels_to_bits(ql), synthetic.labels_to_bits(gl)
    # identical P@10 / R@10 to the reference's sklearn ranking
    for k in (1, 5, 10):
        assert metrics.ranking_metrics(gi, qb, gb, k)[1:] == metrics.ranking_metrics(si, qb, gb, k)[1:]
    p_ref = [metrics.precision_at_k([ids[j] for j in si[q]], [ids[j] for j in np.nonzero(gb & qb[q])[0]], 10)
             for q in range(len(Qm))]
    p_got = [metrics.precision_at_k([ids[j] for j in gi[q]], [ids[j] for j in np.nonzero(gb & qb[q])[0]], 10)
             for q in range(len(Qm))]
    assert p_ref == p_got
    eng.close()


@pytest.mark.parametrize("mode", ["x3", "f32", "f16"])
def test_knn_massive_ties_batched_exact(mode):
    """More exact ties inside the candidate margin than the selection buffer holds (2048 rows /
    512 groups): the selection kernel merges the candidates batch by batch into an exact top-K —
    status stays 0 and the lists equal the oracle's (ties by lower index), no host re-run."""
    rng = np.random.default_rng(77)
    G = rng.standard_normal((12_000, 128), dtype=np.float32)
    G[1000:7000] = G[5]                      # 6001 identical rows
    G[9000:9003] = G[5] * 2.0                # same direction, other norms: equal cosine too
    Qm = np.concatenate([G[5:6], G[5:6] * -1.0, rng.standard_normal((3, 128), dtype=np.float32)])
    for K in (10, 256):
        gi, _ = _exact_check(G, Qm, K, mode=mode)
        assert gi[0, 0] == 5 and gi[0, 1:K].tolist() == list(range(1000, 999 + K))


def test_knn_f16_dim_above_1024():
    """d > 1024 (Dp = 1536): the strided query prep and the d > 1024 re-score branch; the f16
    margin term 2 sqrt(Dp) 2^-25 is computed from Dp."""
    rng = np.random.default_rng(1536)
    G = rng.standard_normal((4000, 1536), dtype=np.float32)
    G[10:14] = G[2]
    Qm = np.concatenate([G[2:3], rng.standard_normal((40, 1536), dtype=np.float32)])
    for mode in ("f16", "x3", "f32"):
        gi, _ = _exact_check(G, Qm, 16, mode=mode)
        assert gi[0, :5].tolist() == [2, 10, 11, 12, 13]


def _exact_topk_chunked(Q, G, K, chunk=131072):
    """oracle.knn.exact_topk semantics over a large gallery in row chunks (f64 scores, score desc
    then index asc) without an N x Q f64 matrix of the whole gallery."""
    Q64 = np.asarray(Q, np.float64)
    qn = np.linalg.norm(Q64, axis=1)
    best_s = np.full((len(Q), 0), -np.inf)
    best_i = np.zeros((len(Q), 0), np.int64)
    for c0 in range(0, len(G), chunk):
        Gc = np.asarray(G[c0:c0 + chunk], np.float64)
        gn = np.linalg.norm(Gc, axis=1)
        den = qn[:, None] * gn[None, :]
        with np.errstate(invalid="ignore", divide="ignore"):
            s = np.where(den > 0, (Q64 @ Gc.T) / np.where(den > 0, den, 1.0), 0.0)
        cs = np.concatenate([best_s, s], 1)
        ci = np.concatenate([best_i, np.broadcast_to(np.arange(c0, c0 + len(Gc)), s.shape)], 1)
        order = np.lexsort((ci, -cs), axis=1)[:, :K]
        best_s, best_i = np.take_along_axis(cs, order, 1), np.take_along_axis(ci, order, 1)
    return best_i, best_s


def test_knn_cfg3_1m_text_queries_top50():
    """BASELINE cfg3's kNN leg: 1024 queries, top-50 over 1M x 768.  f16 and x3 scans return the
    same exact lists for all 1024 queries; 32 of them equal the oracle's exact top-50."""
    G = synthetic.gauss_gallery(1_000_000, 768, synthetic.SEED + 3)
    G[123_456:123_460] = G[777]
    Qm = synthetic.gauss_gallery(1024, 768, synthetic.SEED + 4)
    Qm[0] = G[777] * 0.25
    ix = GalleryIndex(G, mode="f16")
    q = torch.from_numpy(Qm).cuda()
    i16, _, s16, st16 = ix.search(q, 50, want_f64=True, want_status=True)
    ix.set_mode("x3")
    i3, _, s3, st3 = ix.search(q, 50, want_f64=True, want_status=True)
    torch.cuda.synchronize()
    assert int(st16.max()) == 0 and int(st3.max()) == 0
    assert torch.equal(i16, i3) and torch.equal(s16, s3)
    sub = np.r_[0, np.arange(1, 1024, 33)][:32]
    ei, es = _exact_topk_chunked(Qm[sub], G, 50)
    np.testing.assert_array_equal(i16.cpu().numpy()[sub], ei)
    np.testing.assert_allclose(s16.cpu().numpy()[sub], es, rtol=0, atol=1e-12)
    assert i16[0, :5].tolist() == [777, 123_456, 123_457, 123_458, 123_459]
    ix.close()


def test_knn_two_streams_share_one_index():
    """Searches on one index from two streams: the workspace follows the stream (event hand-off),
    so concurrent enqueues return the same lists as sequential ones."""
    G = synthetic.gauss_gallery(50_000, 256, 91)
    Qa = torch.from_numpy(synthetic.gauss_gallery(200, 256, 92)).cuda()
    Qb = torch.from_numpy(synthetic.gauss_gallery(40, 256, 93)).cuda()
    for mode in ("f16", "x3"):
        ix = GalleryIndex(G, mode=mode)
        ra = ix.search(Qa, 20)[0].clone()
        rb = ix.search(Qb, 20)[0].clone()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = []
        for _ in range(4):
            with torch.cuda.stream(s1):
                oa = ix.search(Qa, 20)[0]
            with torch.cuda.stream(s2):
                ob = ix.search(Qb, 20)[0]
            outs.append((oa, ob))
        torch.cuda.synchronize()
        for oa, ob in outs:
            assert torch.equal(oa, ra) and torch.equal(ob, rb)
        ix.close()


def test_knn_f16_raw_query_range():
    """Q <= 32 f16 searches score the caller's unnormalised rows in fp16 (no prep launch): a zero
    query (every score 0 -> rows 0..K-1), tiny and large norms (per-query margin), a component beyond
    fp16's safe range (the exact every-row path), and a query view that is not 16-B aligned (prep
    path) all return the oracle's exact lists; the prep path agrees bit for bit."""
    rng = np.random.default_rng(808)
    G = rng.standard_normal((6000, 256), dtype=np.float32)
    G[3000:3004] = G[17]
    Qm = rng.standard_normal((12, 256), dtype=np.float32)
    Qm[0] = 0.0
    Qm[1] = G[17] * 1e-7             # |q| ~ 1.6e-6: fp16 subnormals, margin dominated by delta_abs
    Qm[2] = G[17] * 3e3              # large but in range
    Qm[3] = rng.standard_normal(256).astype(np.float32)
    Qm[3, 5] = 5e4                   # beyond the fp16-safe range -> every-row path
    Qm[4] = G[17] * 1e-3
    gi, _ = _exact_check(G, Qm, 12, mode="f16")
    assert gi[0].tolist() == list(range(12))
    for r in (1, 2, 4):
        assert gi[r, :5].tolist() == [17, 3000, 3001, 3002, 3003]
    # unaligned view: 1 float in, same rows -> prep + normalised scan, same exact lists
    buf = torch.from_numpy(np.concatenate([np.zeros(1, np.float32), Qm.ravel()])).cuda()
    qv = buf[1:].view(12, 256)
    ix = GalleryIndex(G, mode="f16")
    i2, _, s2, st2 = ix.search(qv, 12, want_f64=True, want_status=True)
    i3, _, s3, _ = ix.search(torch.from_numpy(Qm).cuda(), 12, want_f64=True, want_status=True)
    torch.cuda.synchronize()
    ix.close()
    assert int(st2.max()) == 0
    np.testing.assert_array_equal(i2.cpu().numpy(), gi)
    np.testing.assert_array_equal(i3.cpu().numpy(), gi)
    assert torch.equal(s2, s3)


@pytest.mark.parametrize("Q", [5, 40, 256])
@pytest.mark.parametrize("K", [10, 100])
def test_knn_f16_coarse_select_clusters(Q, K):
    """The f16 selection reads per-(query, 64-row block) maxima first: tight clusters put hundreds of
    rows inside the margin (the tightening pass) and a run of near-duplicates inside one block (a
    loose thread-max bound); lists stay exact."""
    rng = np.random.default_rng(Q * 1000 + K)
    G = rng.standard_normal((30_000, 128), dtype=np.float32)
    c = rng.standard_normal(128).astype(np.float32)
    G[4096:6096] = c + 0.05 * rng.standard_normal((2000, 128), dtype=np.float32)   # 2000-row cluster
    G[20_000:20_064] = G[7] + 1e-4 * rng.standard_normal((64, 128), dtype=np.float32)  # one block
    Qm = rng.standard_normal((Q, 128), dtype=np.float32)
    Qm[0] = c
    Qm[1] = G[7]
    Qm[2] = -c
    _exact_check(G, Qm, K, mode="f16")


@pytest.mark.parametrize("Q", [3, 64])
@pytest.mark.parametrize("K", [10, 50])
def test_knn_f16_scattered_cluster_block_tightening(Q, K):
    """A cluster scattered over many 64-row blocks: more than 2K + 32 blocks clear the first
    (thread-max) bound, so the selection tightens it with the exact K-th largest of the collected
    blocks' maxima before reading their unit maxima (knn_select_t COARSE); lists stay exact."""
    rng = np.random.default_rng(7000 + Q * 10 + K)
    N, D = 60_000, 256
    G = rng.standard_normal((N, D), dtype=np.float32)
    c = rng.standard_normal(D).astype(np.float32)
    rows = rng.choice(N // 64, size=800, replace=False) * 64 + rng.integers(0, 64, size=800)
    G[rows] = c + 0.08 * rng.standard_normal((800, D), dtype=np.float32)
    Qm = rng.standard_normal((Q, D), dtype=np.float32)
    Qm[0] = c
    Qm[1] = c + 0.01 * rng.standard_normal(D).astype(np.float32)
    _exact_check(G, Qm, K, mode="f16")


@pytest.mark.parametrize("N", [1, 100, 255, 256, 257, 513])
@pytest.mark.parametrize("Q", [129, 256, 600])
def test_knn_f16_p8_small_galleries(N, Q):
    """129-512-query f16 passes on the 8-phase GEMM scan with fewer gallery tiles than workgroups
    (one 256-row tile, or a few: most XCD slots idle) and padded rows inside the last tile; Q = 600:
    a 512-query pass (two query tiles per gallery tile) + an 88-query tile-scan pass."""
    rng = np.random.default_rng(N * 7 + Q)
    G = rng.standard_normal((N, 128), dtype=np.float32)
    Qm = rng.standard_normal((Q, 128), dtype=np.float32)
    _exact_check(G, Qm, 10, mode="f16")


@pytest.mark.parametrize("Q", [200, 300, 700])
def test_knn_f16_p8_four_row_units(Q):
    """Galleries above 2^18 rows at K < 32: the 8-phase GEMM scan writes 4-row unit maxima
    (knn_select_t<2>) instead of 2-row ones, in passes of up to 1024 queries (query tiles sharing
    each gallery tile: Q = 300 two tiles, the second padded; 700 three tiles); exact vs the oracle,
    with a duplicate run and the padded last tile."""
    rng = np.random.default_rng(4444)
    G = rng.standard_normal((300_001, 128), dtype=np.float32)
    G[200_000:200_006] = G[11]
    Qm = rng.standard_normal((Q, 128), dtype=np.float32)
    Qm[0] = G[11]
    gi, _ = _exact_check(G, Qm, 10, mode="f16")
    assert gi[0, :7].tolist() == [11] + list(range(200_000, 200_006))
