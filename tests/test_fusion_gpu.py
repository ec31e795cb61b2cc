"""GPU parity of the multimodal fusion stack (model_type="multimodal", model.py:375-459) and its
kernels against plain-torch fp32 (oracle/towers.py: mha / cross_modal_fusion / multimodal, pinned to
the reference by tests/golden/towers_mini.npz in test_oracle_golden.py).

Tolerances: attention core (bf16 q/k/v, bf16 P) max|err| <= 2e-2 * max|ref|; exact-f32 kernels
(linear_f32, ln_rows f32) 1e-5; end-to-end multimodal joint embeddings cosine >= 0.999 per row and
max|err| <= 4e-2 * max|ref| (bf16 token activations through the stack).  MX-fp8 stack (config 5:
e4m3 operands of the enhancer in_proj and cross-projection GEMMs): cosine >= 0.995 per row,
max|err| <= 1e-1 * max|ref| — e4m3 keeps 3 mantissa bits per operand element."""
import math

import pytest
import torch
import torch.nn.functional as F

from mmr_amd import ops, synthetic
from mmr_amd.model import Backbones, MultiModalRetrievalModel, init_fusion_state, init_head_state
from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
from oracle import towers as otw

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(got, ref):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-12)


def bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("B,lq,lk,heads,dh", [(2, 128, 128, 8, 96), (3, 49, 128, 8, 96), (2, 128, 49, 4, 16),
                                              (2, 51, 51, 8, 96), (2, 1, 1, 4, 32), (1, 77, 300, 2, 64),
                                              (2, 40, 512, 3, 128), (1, 33, 65, 1, 192), (2, 300, 512, 8, 96)])
def test_mha_strided_and_mean(B, lq, lk, heads, dh):
    """mmr_mha == softmax(q k^T / sqrt(dh)) v on strided row views of packed projections; mean over
    the query rows; ragged lq / lk (padded to 32 in-kernel)."""
    g = torch.Generator().manual_seed(B * 1000 + lq + lk + dh)
    E = heads * dh
    qp = bf(torch.randn(B * lq, 3 * E, generator=g))          # q in cols [E, 2E) of a packed row
    kvp = bf(torch.randn(B * lk, 2 * E + 16, generator=g))    # k | v | pad (row stride 2E + 16)
    q, k, v = qp[:, E:2 * E], kvp[:, :E], kvp[:, E:2 * E]
    hd = lambda t, L: t.float().reshape(B, L, heads, dh).transpose(1, 2)  # noqa: E731
    ref = ((hd(q, lq) @ hd(k, lk).transpose(-1, -2)) / math.sqrt(dh)).softmax(-1) @ hd(v, lk)
    ref = ref.transpose(1, 2).reshape(B * lq, E)
    qd, kvd = qp.to(DEV), kvp.to(DEV)
    out = torch.empty((B * lq, E), dtype=torch.bfloat16, device=DEV)
    mean = torch.empty((B, E), dtype=torch.float32, device=DEV)
    ops.mha(qd[:, E:2 * E], kvd[:, :E], kvd[:, E:2 * E], B, lq, lk, heads, dh, 1 / math.sqrt(dh), out=out,
            mean_out=mean)
    assert rel_err(out, ref) < 2e-2
    assert rel_err(mean, ref.view(B, lq, E).mean(1)) < 2e-2
    # mean-only launch gives the same mean
    mean2 = torch.empty_like(mean)
    ops.mha(qd[:, E:2 * E], kvd[:, :E], kvd[:, E:2 * E], B, lq, lk, heads, dh, 1 / math.sqrt(dh), mean_out=mean2)
    if lq <= 128:  # single query chunk: deterministic LDS reduction
        assert torch.equal(mean, mean2)
    else:
        assert rel_err(mean2, mean.cpu()) < 1e-5


@pytest.mark.parametrize("B,cin,cout,act,bias,res", [(256, 768, 1536, 1, True, False), (256, 1536, 768, 0, True, True),
                                                  (256, 768, 384, 1, True, False), (256, 384, 768, 0, True, True),
                                                  (1280, 768, 768, 0, True, False), (7, 1024, 2048, 1, False, False)])
def test_linear_x3(B, cin, cout, act, bias, res):
    """mmr_linear_x3 (bf16x3 MFMA: hi*hi + hi*lo + lo*hi of the bf16 splits, f32 accumulation) vs an f64
    reference: within 2e-5 * max|ref| (f32 linear_f32: 1e-5), ragged row counts, residual in place."""
    g = torch.Generator().manual_seed(B + cin + cout)
    x = torch.randn(B, cin, generator=g)
    w = torch.randn(cout, cin, generator=g) * cin ** -0.5
    b = torch.randn(cout, generator=g) if bias else None
    r = torch.randn(B, cout, generator=g) if res else None
    ref = x.double() @ w.double().T
    if b is not None:
        ref = ref + b.double()
    if act == 1:
        ref = torch.nn.functional.gelu(ref)
    if r is not None:
        ref = ref + r.double()
    y = r.to(DEV) if r is not None else None
    out = ops.linear_x3(x.to(DEV), ops.X3W(w.to(DEV)), b.to(DEV) if b is not None else None, residual=y, act=act,
                        out=y)
    err = (out.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5, err


def test_linear_x3_wave_split():
    """The 8-wave K split (small launches) and the 4-wave one agree with the f64 reference alike."""
    g = torch.Generator().manual_seed(11)
    x, w = torch.randn(96, 1536, generator=g), torch.randn(768, 1536, generator=g) * 1536 ** -0.5
    b = torch.randn(768, generator=g)
    ref = x.double() @ w.double().T + b.double()
    for nw in (4, 8):
        with ops.pinned(ops.PIN_X3_WAVES, nw):
            out = ops.linear_x3(x.to(DEV), ops.X3W(w.to(DEV)), b.to(DEV))
        err = (out.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-5, (nw, err)


def test_linear_x3_batched_strided():
    """The batched form over strided row views (the fusion head's phase-2 layout: x rows of nl*C with
    per-problem column offsets, residual per problem) == per-problem linear_f32 within 2e-5."""
    g = torch.Generator().manual_seed(5)
    nl, B, C, D = 5, 64, 768, 768
    G = torch.randn(B, nl * C, generator=g).to(DEV)
    w = (torch.randn(nl, D, C, generator=g) * C ** -0.5).to(DEV)
    b = torch.randn(nl, D, generator=g).to(DEV)
    r = torch.randn(nl, B, D, generator=g).to(DEV)
    y = ops.linear_x3_batched(G, ops.X3W(w), b, nl, B, residual=r, ldx=nl * C, bsx=C)
    for i in range(nl):
        ref = ops.linear_f32(G[:, i * C:(i + 1) * C], w[i], b[i], residual=r[i])
        err = (y[i] - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-5, (i, err)


def test_linear_f32_strided_residual_inplace():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(70, 200, generator=g)
    w, b = torch.randn(96, 128, generator=g) * 0.1, torch.randn(96, generator=g)
    r = torch.randn(70, 96, generator=g)
    xd = x.to(DEV)
    y = r.to(DEV).clone()
    ops.linear_f32(xd[:, 16:144], w.to(DEV), b.to(DEV), residual=y, out=y)     # strided x, in-place residual
    ref = x[:, 16:144] @ w.T + b + r
    assert rel_err(y, ref) < 1e-5
    y2 = ops.linear_f32(xd[:, 16:144], w.to(DEV), b.to(DEV), act=1)
    assert rel_err(y2, F.gelu(x[:, 16:144] @ w.T + b)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ln_rows(dtype):
    g = torch.Generator().manual_seed(7)
    x, r = torch.randn(37, 768, generator=g).to(dtype), torch.randn(37, 768, generator=g).to(dtype)
    ga, be = 1 + 0.1 * torch.randn(768, generator=g), 0.1 * torch.randn(768, generator=g)
    post = torch.randn(37, 768, generator=g)
    a, ps = torch.tensor([0.7]), torch.tensor([1.3])
    ref = F.layer_norm(a * x.float() + r.float(), (768,), ga, be, 1e-5)
    y = ops.ln_rows(x.to(DEV), ga.to(DEV), be.to(DEV), 1e-5, alpha=a.to(DEV), residual=r.to(DEV))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(y, ref) < tol
    if dtype == torch.float32:
        y = ops.ln_rows(x.to(DEV), ga.to(DEV), be.to(DEV), 1e-5, post=post.to(DEV), post_scale=ps.to(DEV))
        assert rel_err(y, F.layer_norm(x, (768,), ga, be, 1e-5) + 1.3 * post) < 1e-5


@pytest.mark.parametrize("c,ld,groups", [(768, 768, 1), (384, 384, 3), (1024, 1024, 1), (96, 96, 1), (768, 770, 2),
                                         (256, 258, 1), (192, 192, 2), (200, 201, 1), (520, 521, 1), (40, 40, 1)])
def test_ln_rows_f32_widths(c, ld, groups):
    """f32 rows at the widths the vector forms take (c % 256: 4-wide, c % 128: 2-wide), the short-row form
    (c <= 256: 16 / 32 lanes per row) and the scalar form (longer rows at an odd stride), grouped
    parameters, residual + post, a row count that leaves dead lanes: vs torch fp32 within 1e-5."""
    g = torch.Generator().manual_seed(c + ld + groups)
    rows = 6 * groups + 1
    xb = torch.randn(rows, ld, generator=g)
    x, r, post = xb[:, :c], torch.randn(rows, c, generator=g), torch.randn(rows, c, generator=g)
    ga, be = 1 + 0.1 * torch.randn(groups, c, generator=g), 0.1 * torch.randn(groups, c, generator=g)
    a, ps = 0.5 + torch.rand(groups, generator=g), torch.rand(groups, generator=g)
    y = ops.ln_rows(xb.to(DEV)[:, :c], ga.to(DEV), be.to(DEV), 1e-5, alpha=a.to(DEV), residual=r.to(DEV),
                    post=post.to(DEV), post_scale=ps.to(DEV), groups=groups)
    gi = torch.arange(rows) % groups
    ref = F.layer_norm(a[gi, None] * x + r, (c,), None, None, 1e-5) * ga[gi] + be[gi] + ps[gi, None] * post
    assert rel_err(y, ref) < 1e-5


def test_add_pos_and_assemble():
    g = torch.Generator().manual_seed(9)
    x = torch.randn(3, 49, 96, generator=g)
    pos = torch.randn(512, 96, generator=g)
    y = ops.add_pos(x.to(DEV), pos.to(DEV), 49)
    assert rel_err(y, x + pos[:49]) < 1e-2
    x1, x2 = torch.randn(3, 64, generator=g), torch.randn(3, 64, generator=g)
    pf = bf(torch.randn(3 * 5, 64, generator=g))
    pe = torch.randn(10, 64, generator=g)
    s = ops.assemble_seq(x1.to(DEV), pf.to(DEV), x2.to(DEV), pe.to(DEV), 5)
    ref = torch.cat([x1[:, None], pf.float().view(3, 5, 64), x2[:, None]], 1) + pe[:7]
    assert rel_err(s, ref) < 1e-2


def _check_emb(got, ref, tol=4e-2):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    cos = F.cosine_similarity(got, ref, dim=1)
    assert cos.min().item() >= 0.999, cos
    assert rel_err(got, ref) <= tol


@pytest.mark.parametrize("text", [True, False])
def test_fusion_stack_vs_oracle_on_backbone_features(text):
    """FusionStack on fixed backbone features (B=3, L=128, joint 768, 8 heads, 3 layers) vs the
    oracle restatement; text=False exercises the learnable default text token (fusion.py:404-407)."""
    g = torch.Generator().manual_seed(11)
    B, Lt, Np, C, D = 3, 128, 49, 768, 768
    hs = init_head_state(C, C, D, 21)
    hs.update(init_fusion_state(C, C, D, 8, 3, 22))
    G = torch.randn(B, C, generator=g)
    P = torch.randn(B, Np, C, generator=g)
    T = bf(torch.randn(B, Lt, C, generator=g)).float() if text else None
    with torch.no_grad():
        ref = otw.multimodal(G, P, T, hs, num_heads=8)
    from mmr_amd.fusion import FusionStack
    fs = FusionStack(hs, 8, device=DEV)
    got = fs.forward(G.to(DEV), P.to(DEV), T.to(DEV) if text else None)
    _check_emb(got, ref)


@pytest.mark.parametrize("tower_dtype", ["bf16", "fp8", "x3"])
def test_fusion_stack_side_stream_bitwise(tower_dtype):
    """The patch-side layer work on a side stream (FusionStack.side_streams; bf16, MX-fp8 and x3
    paths) runs the same kernels on the same operands as one stream: bitwise-equal joint embeddings
    (first call in sequence, then with and without the side stream), at B = 256 where the patch
    GEMMs take the 8-phase route."""
    g = torch.Generator().manual_seed(17)
    B, Lt, Np, C, D = 256, 128, 49, 768, 768
    hs = init_head_state(C, C, D, 27)
    hs.update(init_fusion_state(C, C, D, 8, 5, 28))
    G = torch.randn(B, C, generator=g).to(DEV)
    P = torch.randn(B, Np, C, generator=g).to(DEV)
    T = bf(torch.randn(B, Lt, C, generator=g)).float().to(DEV)
    from mmr_amd.fusion import FusionStack
    fs = FusionStack(hs, 8, device=DEV, tower_dtype=tower_dtype)
    first = fs.forward(G, P, T).clone()      # warm call: one stream
    fs.side_streams = True
    two = fs.forward(G, P, T).clone()
    fs.side_streams = False
    one = fs.forward(G, P, T).clone()
    torch.cuda.synchronize()
    assert torch.equal(two, one) and torch.equal(first, one)


@pytest.mark.parametrize("tower_dtype", ["bf16", "x3"])
def test_model_early_patch_work_bitwise(tower_dtype):
    """MultiModalRetrievalModel.query_embeddings with the towers concurrent and the fusion stack's
    patch-side work started on the towers' side stream right after the image tower (patch_work):
    bitwise-equal joint embeddings to the first (in-sequence) call and to a call with the towers in
    sequence (B = 64)."""
    from mmr_amd.model import build_bench_model
    B = 64
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 81))).to(DEV)
    ids, mask = (torch.from_numpy(a).to(DEV) for a in synthetic.reports(B, 128, 82))
    m = build_bench_model(device=DEV, joint_dim=768, model_type="multimodal", tower_dtype=tower_dtype)
    first = m.query_embeddings(img, ids, mask).clone()
    early = m.query_embeddings(img, ids, mask).clone()
    m.concurrent_towers = False
    seq = m.query_embeddings(img, ids, mask).clone()
    torch.cuda.synchronize()
    assert torch.equal(early, seq) and torch.equal(first, seq)


def test_fusion_stack_exact_query_linears():
    """exact_query_linears=True routes the per-query linears (global enhancer, out-projections, the
    joint chain) to exact f32 (mmr_linear_f32*): both routes match the oracle; they differ from each
    other by ~1e-4 relative (the per-query vectors feed the bf16 fused sequence, where a 2^-17
    difference can flip a bf16 rounding)."""
    g = torch.Generator().manual_seed(13)
    B, Lt, Np, C, D = 3, 128, 49, 768, 768
    hs = init_head_state(C, C, D, 25)
    hs.update(init_fusion_state(C, C, D, 8, 3, 26))
    G = torch.randn(B, C, generator=g)
    P = torch.randn(B, Np, C, generator=g)
    T = bf(torch.randn(B, Lt, C, generator=g)).float()
    with torch.no_grad():
        ref = otw.multimodal(G, P, T, hs, num_heads=8)
    from mmr_amd.fusion import FusionStack
    fs = FusionStack(hs, 8, device=DEV)
    x3 = fs.forward(G.to(DEV), P.to(DEV), T.to(DEV))
    fs.exact_query_linears = True
    ex = fs.forward(G.to(DEV), P.to(DEV), T.to(DEV))
    assert FusionStack(hs, 8, device=DEV, exact_query_linears=True).exact_query_linears
    _check_emb(ex, ref)
    assert rel_err(ex.cpu(), x3.cpu()) <= 1e-3
    assert not torch.equal(ex, x3)  # the two routes really differ (bf16x3 vs f32 products)


def test_full_size_multimodal_vs_oracle():
    """Swin-T + BERT-base + 5-layer multimodal head (joint 768, 8 heads) end to end, B=2."""
    ssd, bsd = init_swin_state(SWIN_T, 5), init_bert_state(BERT_BASE, 6)
    hs = init_head_state(768, 768, 768, 7)
    hs.update(init_fusion_state(768, 768, 768, 8, 5, 8))
    bb = Backbones(swin_state=ssd, bert_state=bsd, device=DEV)
    m = MultiModalRetrievalModel(joint_dim=768, num_heads=8, model_type="multimodal", backbones=bb,
                                 head_state=hs, device=DEV, use_shared_ffn=False)
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(2, 9)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(2, 128, 10))
    o = m(img.to(DEV), ids.to(DEV), mask.to(DEV))
    q = m.query_embeddings(img.to(DEV), ids.to(DEV), mask.to(DEV))
    with torch.no_grad():
        (rg, rp), rt = otw.backbones_forward(img, ids, mask, ssd, bsd, SWIN_T, BERT_BASE)
        ref = otw.heads(rg, rp, rt, hs, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"]
    _check_emb(o["joint_emb"], ref)
    assert torch.equal(o["joint_emb"], q)


@pytest.mark.parametrize("text", [True, False])
def test_fusion_stack_reference_joint_dim_1024(text):
    """The reference's configured head geometry (configs/config.yaml:14 joint_dim 1024, num_heads 8
    -> head_dim 128, num_fusion_layers 5) on 768-wide backbone features, vs the oracle."""
    g = torch.Generator().manual_seed(12)
    B, Lt, Np, C, D = 3, 128, 49, 768, 1024
    hs = init_head_state(C, C, D, 23)
    hs.update(init_fusion_state(C, C, D, 8, 5, 24))
    G = torch.randn(B, C, generator=g)
    P = torch.randn(B, Np, C, generator=g)
    T = bf(torch.randn(B, Lt, C, generator=g)).float() if text else None
    with torch.no_grad():
        ref = otw.multimodal(G, P, T, hs, num_heads=8)
    from mmr_amd.fusion import FusionStack
    fs = FusionStack(hs, 8, device=DEV)
    got = fs.forward(G.to(DEV), P.to(DEV), T.to(DEV) if text else None)
    assert got.shape == (B, D)
    _check_emb(got, ref)


def test_full_size_multimodal_joint_dim_1024_batch_256_vs_oracle():
    """Swin-T + BERT-base + 5-layer multimodal head at joint_dim 1024 (config.yaml:14), B=256 through
    query_embeddings (the bench's stream-overlapped path), compared with the oracle on 4 rows."""
    ssd, bsd = init_swin_state(SWIN_T, 15), init_bert_state(BERT_BASE, 16)
    hs = init_head_state(768, 768, 1024, 17)
    hs.update(init_fusion_state(768, 768, 1024, 8, 5, 18))
    bb = Backbones(swin_state=ssd, bert_state=bsd, device=DEV)
    m = MultiModalRetrievalModel(joint_dim=1024, num_heads=8, model_type="multimodal", backbones=bb,
                                 head_state=hs, device=DEV, use_shared_ffn=False)
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(256, 19)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(256, 128, 20))
    q = m.query_embeddings(img.to(DEV), ids.to(DEV), mask.to(DEV))      # first call: towers in sequence
    q2 = m.query_embeddings(img.to(DEV), ids.to(DEV), mask.to(DEV))     # overlapped streams
    torch.cuda.synchronize()
    assert q.shape == (256, 1024) and torch.equal(q, q2)
    rows = [0, 77, 128, 255]
    with torch.no_grad():
        (rg, rp), rt = otw.backbones_forward(img[rows], ids[rows], mask[rows], ssd, bsd, SWIN_T, BERT_BASE)
        ref = otw.heads(rg, rp, rt, hs, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"]
    _check_emb(q[rows], ref)


def test_fusion_stack_fp8_vs_oracle():
    """tower_dtype="fp8": the enhancer in_proj and folded cross-projection GEMMs on MX-fp8 operands
    emitted by the add-pos / LayerNorm kernels.  B=256 so both the text (B*128) and the patch
    (B*49) token rows are 256 multiples (both sides take the fp8 path); 8 rows vs the oracle."""
    g = torch.Generator().manual_seed(13)
    B, Lt, Np, C, D = 256, 128, 49, 768, 1024
    hs = init_head_state(C, C, D, 25)
    hs.update(init_fusion_state(C, C, D, 8, 2, 26))
    G = torch.randn(B, C, generator=g)
    P = torch.randn(B, Np, C, generator=g)
    T = bf(torch.randn(B, Lt, C, generator=g)).float()
    from mmr_amd.fusion import FusionStack
    fs8 = FusionStack(hs, 8, device=DEV, tower_dtype="fp8")
    assert all(L["txt"].fp8_ok(B * Lt) and L["patch"].fp8_ok(B * Np) for L in fs8.layers)
    got8 = fs8.forward(G.to(DEV), P.to(DEV), T.to(DEV))
    got = FusionStack(hs, 8, device=DEV).forward(G.to(DEV), P.to(DEV), T.to(DEV))
    rows = [0, 1, 63, 100, 128, 200, 254, 255]
    with torch.no_grad():
        ref = otw.multimodal(G[rows], P[rows], T[rows], hs, num_heads=8)
    _check_emb(got[rows], ref)
    got8 = got8.detach().float().cpu()[rows]
    cos = F.cosine_similarity(got8, ref.float(), dim=1)
    assert cos.min().item() >= 0.995, cos
    assert rel_err(got8, ref) <= 1e-1
    assert not torch.equal(got8, got.detach().float().cpu()[rows])  # the fp8 path really ran


def test_fusion_stack_fp8_head_dim_not_multiple_of_32_falls_back():
    """tower_dtype="fp8" with D = 768 and 16 heads (head_dim 48): the MX-fp8 attention
    output needs head_dim % 32 == 0, so every enhancer / o2 path stays bf16 (no MMRError) and the
    result matches the oracle like the bf16 stack."""
    g = torch.Generator().manual_seed(14)
    B, Lt, Np, C, D, H = 256, 128, 49, 768, 768, 16
    hs = init_head_state(C, C, D, 27)
    hs.update(init_fusion_state(C, C, D, H, 2, 28))
    G = torch.randn(B, C, generator=g)
    P = torch.randn(B, Np, C, generator=g)
    T = bf(torch.randn(B, Lt, C, generator=g)).float()
    from mmr_amd.fusion import FusionStack
    fs8 = FusionStack(hs, H, device=DEV, tower_dtype="fp8")
    assert not any(L["txt"].fp8_ok(B * Lt) or L["patch"].fp8_ok(B * Np) for L in fs8.layers)
    got8 = fs8.forward(G.to(DEV), P.to(DEV), T.to(DEV))
    rows = [0, 100, 255]
    with torch.no_grad():
        ref = otw.multimodal(G[rows], P[rows], T[rows], hs, num_heads=H)
    _check_emb(got8[rows], ref)
