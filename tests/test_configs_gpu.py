"""GPU: BASELINE.json configs 3-5 at their per-GPU size, against the oracle.

cfg4 (8M x 768 over 8 GPUs = 1M rows per shard, K=10, Q=256): one shard's search on the 4-row-unit
    p8 path (> 2^18 rows, K < 32), all queries equal between the f16 and x3 scans, 32 against the
    chunked exact oracle (oracle.knn.exact_topk semantics).  The 2 x 1M world-2 merge is in
    test_sharded_gpu.py.
cfg5 (fp8 towers, B=2048, 8M x 1024 fp16 gallery = 1M rows per GPU, K=10, KG rerank fused):
    the 1M x 1024 f16 search of 2048 queries (8 passes of 256), the fused rerank in the step on the
    device's own candidates vs oracle/dls.rerank (reranker.py:240-333), the sharded rerank (shard
    components -> payload merge -> mix) bit-identical to the fused one, and the B=2048 MX-fp8 tower
    step with 16 of its embeddings against the fp32 oracle.
cfg3 (text-only BERT, B=1024): the text tower + head at B=1024 (GEMM M=131072) vs the oracle.
"""
import numpy as np
import pytest
import torch

from mmr_amd import synthetic
from mmr_amd.retrieval import GalleryIndex, merge_topk, rerank_mix
from oracle import dls as odls

pytestmark = pytest.mark.gpu


def _exact_topk_chunked(Q, G, K, chunk=131072):
    """oracle.knn.exact_topk semantics (f64 cosine, 0 for zero norms; score desc, index asc) over a
    gallery too large for one N x Q f64 matrix."""
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


def test_cfg4_shard_1m_x_768_q256_k10():
    """One cfg4 shard: 1M x 768, 256 queries, top-10 (the p8 GEMM scan with 4-row unit maxima and
    knn_select_t<2>), duplicates across the shard and a zero row."""
    G = synthetic.gauss_gallery(1_000_000, 768, synthetic.SEED + 40)
    G[900_000:900_005] = G[31]
    G[77] = 0.0
    Qm = synthetic.gauss_gallery(256, 768, synthetic.SEED + 41)
    Qm[0] = G[31] * 2.0
    ix = GalleryIndex(G, mode="f16")
    q = torch.from_numpy(Qm).cuda()
    i16, _, s16, st16 = ix.search(q, 10, want_f64=True, want_status=True)
    ix.set_mode("x3")
    i3, _, s3, st3 = ix.search(q, 10, want_f64=True, want_status=True)
    torch.cuda.synchronize()
    ix.close()
    assert int(st16.max()) == 0 and int(st3.max()) == 0
    assert torch.equal(i16, i3) and torch.equal(s16, s3)
    sub = np.r_[0, np.arange(1, 256, 8)][:32]
    ei, es = _exact_topk_chunked(Qm[sub], G, 10)
    np.testing.assert_array_equal(i16.cpu().numpy()[sub], ei)
    np.testing.assert_allclose(s16.cpu().numpy()[sub], es, rtol=0, atol=1e-12)
    assert i16[0, :6].tolist() == [31] + list(range(900_000, 900_005))


def _rerank_tables(n, nq, dk, seed):
    """uint64 label bitsets (0-3 of 43 labels per record) + f32 KG vectors, vectorised."""
    rng = np.random.default_rng(seed)

    def bits(rows):
        lab = rng.integers(0, synthetic.NUM_LABELS, size=(rows, 3)).astype(np.uint64)
        keep = rng.random((rows, 3)) < np.array([0.8, 0.5, 0.3])
        return np.bitwise_or.reduce(np.where(keep, np.uint64(1) << lab, np.uint64(0)), axis=1)
    return bits(n), bits(nq), rng.standard_normal((n, dk), dtype=np.float32), \
        rng.standard_normal((nq, dk), dtype=np.float32)


def _lset(b):
    return {j for j in range(64) if (int(b) >> j) & 1}


def test_cfg5_search_1m_x_1024_q2048_rerank_fused_and_sharded():
    """cfg5's retrieval leg per GPU: 2048 queries, top-10 over 1M x 1024 on the fp16 scan copy
    (exact f64 ranking), then the KG / label rerank of the 10 candidates (alpha .6 / beta .25 /
    gamma .15, reranker.py:240-333):
      * 16 queries' top-10 equal the chunked exact oracle;
      * the fused rerank (mmr_index_rerank) on the device's own candidates equals oracle/dls.rerank
        on the same lists for 32 queries (order up to runs of equal finals, components 1e-9);
      * the sharded form — two shard indexes, per-shard top-10 + raw components, the payload merge
        and mmr_rerank_mix — returns bit-identical idx / final / components for all 2048 queries."""
    N, D, Q, K, DK = 1_000_000, 1024, 2048, 10, 128
    G = synthetic.gauss_gallery(N, D, synthetic.SEED + 50)
    G[500_000:500_003] = G[9]
    Qm = synthetic.gauss_gallery(Q, D, synthetic.SEED + 51)
    Qm[0] = G[9]
    gbits, qbits, gkg, qkg = _rerank_tables(N, Q, DK, 52)
    dev = torch.device("cuda")
    q = torch.from_numpy(Qm).to(dev)
    tq = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64) if a.dtype == np.uint64 else a).to(dev)  # noqa: E731
    ix = GalleryIndex(G, mode="f16")
    i, _, s64, st = ix.search(q, K, want_f64=True, want_status=True)
    assert int(st.max()) == 0
    fi, ff, fe, fl, fk = ix.rerank(q, i, tq(qbits), tq(gbits), tq(qkg), tq(gkg), K)
    torch.cuda.synchronize()
    ix.close()
    ic = i.cpu().numpy()
    sub = np.r_[0, np.arange(1, Q, 131)][:16]
    ei, es = _exact_topk_chunked(Qm[sub], G, K)
    np.testing.assert_array_equal(ic[sub], ei)
    assert ic[0, :4].tolist() == [9, 500_000, 500_001, 500_002]
    fic, ffc = fi.cpu().numpy(), ff.cpu().numpy()
    for qn in np.r_[0, np.arange(5, Q, 64)][:32]:
        cand = ic[qn]
        order, final, e, l, k = odls.rerank(Qm[qn], G[cand], _lset(qbits[qn]), [_lset(gbits[j]) for j in cand],
                                            qkg[qn].astype(np.float64), gkg[cand].astype(np.float64), topk=K)
        np.testing.assert_allclose(ffc[qn], final, rtol=0, atol=1e-9)
        got = fic[qn].tolist()
        ref = cand[order].tolist()
        for p in range(K):
            if got[p] != ref[p]:
                tied = np.abs(final - final[p]) <= 1e-12
                assert set(np.array(got)[tied]) == set(np.array(ref)[tied])
    # sharded: two shard indexes, components on the owning shard, merge with payload, mix
    half = N // 2
    lists_i, lists_s, comps = [], [], []
    for s0, s1 in ((0, half), (half, N)):
        sx = GalleryIndex(G[s0:s1], idx_base=s0, mode="f16")
        li, _, ls, lst = sx.search(q, K, want_f64=True, want_status=True)
        assert int(lst.max()) == 0
        comps.append(sx.rerank_components(q, li, tq(qbits), tq(gbits[s0:s1]), tq(qkg), tq(gkg[s0:s1])))
        lists_i.append(li)
        lists_s.append(ls)
        torch.cuda.synchronize()
        sx.close()
    mi, _, m64, mc = merge_topk(torch.stack(lists_s), torch.stack(lists_i), K, payload=torch.stack(comps))
    assert torch.equal(mi, i) and torch.equal(m64, s64)
    si, sf, se, sl, sk = rerank_mix(mi, mc, K)
    for a, b in ((si, fi), (sf, ff), (se, fe), (sl, fl), (sk, fk)):
        assert torch.equal(a, b)


def test_cfg5_fp8_towers_batch_2048_vs_oracle():
    """cfg5's tower step at its batch: B=2048 (BERT GEMMs M=262,144; Swin stage 3-4 fp8 linears),
    multimodal head at joint_dim 1024; 16 of the 2048 embeddings against the fp32 oracle
    (e4m3 tolerance: cosine >= 0.99 per embedding, as test_e2e_gpu's fp8 case)."""
    from mmr_amd.model import build_bench_model, init_fusion_state, init_head_state
    from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
    from oracle import towers as otw
    m = build_bench_model(device="cuda", joint_dim=1024, model_type="multimodal", tower_dtype="fp8")
    B = 2048
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 71)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(B, 128, 72))
    m.query_embeddings(img.cuda(), ids.cuda(), mask.cuda())
    q = m.query_embeddings(img.cuda(), ids.cuda(), mask.cuda())
    assert q.shape == (B, 1024) and bool(torch.isfinite(q).all())
    sub = np.r_[0, np.arange(7, B, 136)][:16]
    ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
    hsd = init_head_state(768, 768, 1024, 2711)
    hsd.update(init_fusion_state(768, 768, 1024, 8, 5, 2712))
    with torch.no_grad():
        (g, p), t = otw.backbones_forward(img[sub], ids[sub], mask[sub], ssd, bsd, SWIN_T, BERT_BASE)
        ref = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"].double()
    got = q[torch.from_numpy(sub).cuda()].double().cpu()
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=1)
    print({"fp8_b2048_min_cos": float(cos.min()), "mean": float(cos.mean())})
    assert float(cos.min()) >= 0.99


@pytest.mark.parametrize("B", [1, 7])
def test_fp8_towers_ragged_batches(B):
    """MX-fp8 operands take 256-row panels: batches whose token rows are not multiples of 256
    (B = 1 serving, B = 7) run the fp8 path on zero-padded rows (towers._pad_rows) and match the
    fp32 oracle with the B = 256 case's fp8 bar (cosine >= 0.99), multimodal and text-only."""
    from mmr_amd.model import build_bench_model, init_fusion_state, init_head_state
    from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
    from oracle import towers as otw
    m = build_bench_model(device="cuda", joint_dim=1024, model_type="multimodal", tower_dtype="fp8")
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 81)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(B, 128, 82))
    q = m.query_embeddings(img.cuda(), ids.cuda(), mask.cuda())
    ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
    hsd = init_head_state(768, 768, 1024, 2711)
    hsd.update(init_fusion_state(768, 768, 1024, 8, 5, 2712))
    with torch.no_grad():
        (g, p), t = otw.backbones_forward(img, ids, mask, ssd, bsd, SWIN_T, BERT_BASE)
        ref = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"].double()
    cos = torch.nn.functional.cosine_similarity(q.double().cpu(), ref, dim=1)
    assert q.shape == (B, 1024) and float(cos.min()) >= 0.99
    # the text-only fp8 head through the same padding (BERT rows B * 128)
    mt = build_bench_model(device="cuda", joint_dim=768, model_type="text", tower_dtype="fp8")
    qt = mt.query_embeddings(None, ids.cuda(), mask.cuda())
    hs2 = init_head_state(768, 768, 768, 2711)
    with torch.no_grad():
        t2 = otw.bert_forward(ids, mask, bsd, 12, 12)
        ref2 = otw.heads(None, None, t2, hs2, "text")["joint_emb"].double()
    cos2 = torch.nn.functional.cosine_similarity(qt.double().cpu(), ref2, dim=1)
    assert float(cos2.min()) >= 0.99


def test_cfg3_text_tower_batch_1024_vs_oracle():
    """cfg3's tower at its batch: text-only BERT-base B=1024 x 128 tokens (GEMM M=131,072) + text head;
    16 embeddings against the fp32 oracle (bf16 bar: cosine >= 0.999)."""
    from mmr_amd.model import build_bench_model, init_head_state
    from mmr_amd.towers import BERT_BASE, init_bert_state
    from oracle import towers as otw
    m = build_bench_model(device="cuda", joint_dim=768, model_type="text")
    B = 1024
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(B, 128, 91))
    m.query_embeddings(None, ids.cuda(), mask.cuda())
    q = m.query_embeddings(None, ids.cuda(), mask.cuda())
    sub = np.r_[0, np.arange(3, B, 68)][:16]
    bsd = init_bert_state(BERT_BASE, 2710)
    hs = init_head_state(768, 768, 768, 2711)
    with torch.no_grad():
        t = otw.bert_forward(ids[sub], mask[sub], bsd, 12, 12)
        ref = otw.heads(None, None, t, hs, "text")["joint_emb"].double()
    cos = torch.nn.functional.cosine_similarity(q[torch.from_numpy(sub).cuda()].double().cpu(), ref, dim=1)
    assert float(cos.min()) >= 0.999


def test_index_device_bytes_per_mode():
    """Scan copies exist only in the mode that reads them: f32 rows + norms always; x3 adds the bf16
    hi/lo split + tile16 f32 copies (8 B per element); f16 the ONE tile32h fp16 copy every fp16 scan
    reads (2 B per element; round 4: the p8 scan reads it too, no row-major copy) and frees the x3 ones.
    (An fp16 gallery builds the native fp16 index instead: 2 B per element in all,
    test_knn_f16_native_gpu.py.)"""
    N, D = 1_000_000, 1024
    G = synthetic.gauss_gallery(N, D, synthetic.SEED + 60)
    base = N * D * 4 + N * 12
    ix = GalleryIndex(G, mode="f16")
    g16, _ = ix.device_bytes()
    assert base + N * D * 2 <= g16 <= base + N * D * 2 + 512 * D * 6 + 512 * 12
    ix.set_mode("x3")
    g3, _ = ix.device_bytes()
    assert base + N * D * 8 <= g3 <= base + N * D * 8 + 512 * D * 12
    ix.set_mode("f32")
    g32, _ = ix.device_bytes()
    assert g32 <= base + 512 * D * 4 + 512 * 12
    # results do not depend on which copies exist
    q = torch.from_numpy(synthetic.gauss_gallery(64, D, synthetic.SEED + 61)).cuda()
    a = ix.search(q, 10)[0]
    ix.set_mode("f16")
    b = ix.search(q, 10)[0]
    torch.cuda.synchronize()
    ix.close()
    assert torch.equal(a, b)
