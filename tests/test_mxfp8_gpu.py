"""GPU: MX-fp8 quantiser and block-scaled GEMM (the fp8 tower linears of BASELINE.json config 5)
against the numpy restatement in oracle/mxfp8.py.

Quantiser: bit-exact — every e4m3 value and every E8M0 scale byte (read back through the image-order
offsets) equals the oracle's, including zero blocks, zero-padded K and both scale layouts.
GEMM: the products of e4m3 x e4m3 x 2^(ea+eb) are exact in f32, so the only differences from an f64
GEMM of the dequantised operands are the f32 accumulation order and the bf16 output rounding:
tolerance |y - ref| <= 2^-8 |ref| + 1e-3 * max|ref| (bf16 half-ulp plus accumulation slack)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mmr_amd import ops
from oracle import mxfp8 as mx

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf16_input(rows, k, seed, zero_block=True):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((rows, k)).astype(np.float32)
    x *= np.exp(rng.uniform(-6, 6, (rows, 1))).astype(np.float32)   # per-row magnitudes over 5 decades
    if zero_block:
        x[3, 32:64] = 0.0
    t = torch.from_numpy(x).to(torch.bfloat16)
    return t, t.float().numpy()


def _decode(x8, rows, layout):
    q = mx.e4m3_decode(x8.q.cpu().numpy())
    off = mx.scale_offsets(rows, x8.kp, layout)
    e = x8.s.cpu().numpy()[off].astype(np.int32) - 127
    return q, e


@pytest.mark.parametrize("rows,k,layout", [(256, 768, 0), (512, 384, 0), (384, 768, 1), (192, 3072, 1), (512, 768, 2)])
def test_quantize_bit_exact(rows, k, layout):
    xt, xf = _bf16_input(rows, k, 11 + rows + k)
    x8 = ops.quantize_mxfp8(xt.to(DEV), layout=layout)
    torch.cuda.synchronize()
    q, e = _decode(x8, rows, layout)
    qo, eo = mx.quantize(xf, x8.kp)
    np.testing.assert_array_equal(e, eo)
    np.testing.assert_array_equal(q, qo)
    assert x8.kp >= k and np.all(q[:, k:] == 0)


def _ref(x8, w8, rows, n, bias, res, act):
    qx, ex = _decode(x8, rows, 0)
    qw, ew = _decode(w8, n, w8.layout)
    y = mx.dequantize(qx, ex) @ mx.dequantize(qw, ew).T
    if bias is not None:
        y = y + bias.cpu().numpy().astype(np.float64)[None, :]
    if act:
        y = F.gelu(torch.from_numpy(y)).numpy()
    if res is not None:
        y = y + res.float().cpu().numpy()
    return y


@pytest.mark.parametrize("M,N,K,act,res,wl", [(256, 192, 768, 0, False, 1), (512, 384, 384, 1, False, 1),
                                              (1024, 576, 768, 0, True, 1), (8192, 2304, 768, 0, False, 1),
                                              (4096, 768, 3072, 0, True, 1), (2048, 3072, 768, 1, False, 1),
                                              (256, 256, 768, 0, False, 2), (8192, 2304, 768, 0, False, 2),
                                              (4096, 768, 3072, 0, False, 2), (1024, 512, 512, 1, True, 2)])
def test_linear_mxfp8_matches_dequantised_gemm(M, N, K, act, res, wl):
    """wl: weight layout 1 (256 x 192 tiles) or 2 (256 x 256 tiles)."""
    xt, _ = _bf16_input(M, K, 7 + M)
    wt, _ = _bf16_input(N, K, 8 + N, zero_block=False)
    x8 = ops.quantize_mxfp8(xt.to(DEV), layout=0)
    w8 = ops.quantize_mxfp8((wt * 0.05).to(DEV), layout=wl)
    g = torch.Generator().manual_seed(M + N)
    bias = torch.randn(N, generator=g).to(DEV)
    r = (torch.randn(M, N, generator=g) * 3).to(torch.bfloat16).to(DEV) if res else None
    y = ops.linear_mxfp8(x8, w8, bias, r, act=act)
    torch.cuda.synchronize()
    ref = _ref(x8, w8, M, N, bias, r, act)
    d = np.abs(y.float().cpu().numpy() - ref)
    tol = 2.0 ** -8 * np.abs(ref) + 1e-3 * np.abs(ref).max()
    assert np.all(d <= tol), f"max excess {np.max(d - tol)}"


def test_linear_mxfp8_rejects_bad_shapes():
    x8 = ops.quantize_mxfp8(torch.zeros(256, 768, dtype=torch.bfloat16, device=DEV), layout=0)
    w8 = ops.quantize_mxfp8(torch.zeros(200, 768, dtype=torch.bfloat16, device=DEV)[:192], layout=1)
    with pytest.raises(Exception):
        ops.quantize_mxfp8(torch.zeros(100, 768, dtype=torch.bfloat16, device=DEV), layout=0)
    bad = ops.MXFP8(w8.q[:100], w8.s, 768, 1)
    with pytest.raises(Exception):
        ops.linear_mxfp8(x8, bad)


@pytest.mark.parametrize("M,N,K,act", [(512, 3072, 768, 1), (1024, 1536, 512, 1), (256, 512, 768, 0)])
def test_linear_mxfp8_q8_equals_quantised_bf16_output(M, N, K, act):
    """The fused fp8-output epilogue (BERT FFN1 -> FFN2, Swin fc1 -> fc2) is bit-identical to
    quantising the bf16 output of the same GEMM with mmr_quantize_mxfp8 (values and scale bytes)."""
    xt, _ = _bf16_input(M, K, 3 + M)
    wt, _ = _bf16_input(N, K, 4 + N, zero_block=False)
    x8 = ops.quantize_mxfp8(xt.to(DEV), layout=0)
    w8 = ops.quantize_mxfp8((wt * 0.05).to(DEV), layout=2)
    bias = torch.randn(N, generator=torch.Generator().manual_seed(N)).to(DEV)
    y8 = ops.linear_mxfp8_q8(x8, w8, bias, act=act)
    if act == 0:
        ref8 = ops.quantize_mxfp8(ops.linear_mxfp8(x8, w8, bias, act=act), layout=0)
        torch.cuda.synchronize()
        assert torch.equal(y8.q, ref8.q)
        assert torch.equal(y8.s, ref8.s)
        return
    # GELU: the e4m3 epilogue runs the cheap sigmoid form (common.h gelu_q8x2 = oracle.mxfp8.gelu_q8, bounded in
    # tests/test_gelu_q8_cpu.py) — against the oracle's MX-fp8 of the f64 GEMM + erf GELU, rounded to bf16 as
    # the epilogue rounds: bit-exact wherever the bound allows, i.e. a code differs only where the erf value
    # lies within |gelu_q8 - gelu_erf| (+ one bf16 ulp — both sides round to bf16 before e4m3 — and the f32
    # accumulation) of an e4m3 rounding boundary, and then by one step plus that bound; the scale bytes equal
    # but for blocks whose amax moved across a binade
    z = _ref(x8, w8, M, N, bias, None, 0)                                  # f64 pre-activation
    ref = _ref(x8, w8, M, N, bias, None, act)                              # erf GELU
    refb = torch.from_numpy(ref).float().to(torch.bfloat16).float().numpy()
    qo, eo = mx.quantize(refb, N)
    torch.cuda.synchronize()
    q, e = _decode(y8, M, 0)
    assert np.mean(e != eo) < 2e-3, np.mean(e != eo)
    same = np.repeat(e == eo, 32, axis=1)
    er = np.ldexp(1.0, -np.repeat(e, 32, axis=1))                          # 2^-e: real -> scaled units
    qx, ex_ = _decode(x8, M, 0)
    qw, ew = _decode(w8, N, w8.layout)
    absdot = np.abs(mx.dequantize(qx, ex_)) @ np.abs(mx.dequantize(qw, ew)).T
    acc = K * 2.0 ** -24 * absdot + 2.0 ** -24 * np.abs(z)                 # f32 accumulation (+ the bias add)
    ulp16 = np.ldexp(1.0, np.floor(np.log2(np.maximum(np.abs(ref), 1e-30))).astype(int) - 7)  # bf16 ulp of ref
    slack = (np.abs(mx.gelu_q8(z).astype(np.float64) - ref) + ulp16 + 1.13 * acc) * er
    diff = (q != qo) & same
    mid = (q.astype(np.float64) + qo) / 2                                  # the boundary between the two codes
    near = np.abs(refb * er - mid) <= slack * 1.0001
    assert np.all(near[diff]), f"{np.count_nonzero(diff & ~near)} codes differ away from a rounding boundary"
    a = np.maximum(np.abs(q), np.abs(qo))
    ex = np.floor(np.log2(np.maximum(a, 2.0 ** -30)))
    step = np.where(ex >= -6, 2.0 ** (ex - 3), 2.0 ** -9)
    assert np.all(np.abs(q - qo)[diff] <= (step + 2 * slack)[diff] * 1.0001)  # one step (more only in a block's
    #                                                  subnormal range, where the GELU's 2.7e-4 spans several)
    print(f"codes differing at a rounding boundary: {diff.mean():.4%}")


@pytest.mark.parametrize("rows,c,add", [(512, 768, True), (256, 768, False), (256, 1536, True)])
def test_layernorm_q8_equals_quantised_layernorm(rows, c, add):
    """LayerNorm with the fused MX-fp8 output: y equals the plain LayerNorm bit for bit, and the fp8
    operand equals mmr_quantize_mxfp8 of y (values and scale bytes)."""
    xt, _ = _bf16_input(rows, c, 5 + rows)
    rt, _ = _bf16_input(rows, c, 6 + rows)
    g = torch.Generator().manual_seed(c)
    gam, bet = (torch.randn(c, generator=g) * 0.5 + 1).to(DEV), (torch.randn(c, generator=g) * 0.1).to(DEV)
    x, r = xt.to(DEV), (rt.to(DEV) if add else None)
    y, y8 = ops.layernorm_q8(x, r, gam, bet, 1e-12)
    ref = ops.add_layernorm(x, r, gam, bet, 1e-12) if add else ops.layernorm(x, gam, bet, 1e-12)
    ref8 = ops.quantize_mxfp8(ref, layout=0)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert torch.equal(y8.q, ref8.q)
    assert torch.equal(y8.s, ref8.s)


@pytest.mark.parametrize("rows,c,kp,want_y", [(512, 384, 512, False), (256, 384, 512, True), (256, 96, 256, False),
                                             (256, 768, 768, False)])
def test_layernorm_q8_padded_k(rows, c, kp, want_y):
    """The fp8 Swin stages' LayerNorm operand with K padded to the weight's kp (stage 3: C = 384 -> 512):
    bytes and scale bytes equal mmr_quantize_mxfp8(LayerNorm(x), kp) including the zero padding; with
    want_y=False no bf16 rows are written."""
    xt, _ = _bf16_input(rows, c, 7 + rows + c)
    g = torch.Generator().manual_seed(c + 1)
    gam, bet = (torch.randn(c, generator=g) * 0.5 + 1).to(DEV), (torch.randn(c, generator=g) * 0.1).to(DEV)
    x = xt.to(DEV)
    y, y8 = ops.layernorm_q8(x, None, gam, bet, 1e-5, kp=kp, want_y=want_y)
    ref = ops.layernorm(x, gam, bet, 1e-5)
    ref8 = ops.quantize_mxfp8(ref, layout=0, kp=kp)
    torch.cuda.synchronize()
    assert (y is None) == (not want_y)
    if want_y:
        assert torch.equal(y, ref)
    assert y8.kp == kp and y8.k == c
    assert torch.equal(y8.q, ref8.q)
    assert torch.equal(y8.s, ref8.s)


@pytest.mark.parametrize("rows,c,l,f32in", [(512, 768, 128, False), (256, 768, 49, True), (768, 1024, 51, False)])
def test_add_pos_q8_and_scaled_ln_q8_equal_quantised_outputs(rows, c, l, f32in):
    """The fusion stack's fp8 operand producers (config 5): x + pos and LayerNorm(alpha*x + r) with the
    fused MX-fp8 output — y equal to the plain kernels bit for bit, the operand equal to
    mmr_quantize_mxfp8 of y (values and scale bytes)."""
    xt, _ = _bf16_input(rows, c, 31 + rows)
    rt, _ = _bf16_input(rows, c, 32 + rows)
    g = torch.Generator().manual_seed(c + l)
    pos = (torch.randn(max(l, 64), c, generator=g) * 0.2).to(DEV)
    x = xt.to(DEV).float() if f32in else xt.to(DEV)
    y, y8 = ops.add_pos(x, pos, l, q8=True)
    ref = ops.add_pos(x, pos, l)
    ref8 = ops.quantize_mxfp8(ref, layout=0)
    torch.cuda.synchronize()
    assert torch.equal(y, ref) and torch.equal(y8.q, ref8.q) and torch.equal(y8.s, ref8.s)
    gam, bet = (torch.randn(c, generator=g) * 0.5 + 1).to(DEV), (torch.randn(c, generator=g) * 0.1).to(DEV)
    alpha = torch.tensor([0.7], device=DEV)
    r = rt.to(DEV)
    z, z8 = ops.scaled_add_layernorm(ref, alpha, r, gam, bet, 1e-5, q8=True)
    zr = ops.scaled_add_layernorm(ref, alpha, r, gam, bet, 1e-5)
    zr8 = ops.quantize_mxfp8(zr, layout=0)
    torch.cuda.synchronize()
    assert torch.equal(z, zr) and torch.equal(z8.q, zr8.q) and torch.equal(z8.s, zr8.s)


def test_q8_producers_reject_ragged_rows():
    x = torch.zeros(100, 768, dtype=torch.bfloat16, device=DEV)
    pos = torch.zeros(128, 768, device=DEV)
    with pytest.raises(Exception, match="mmr_add_pos_bf16_q8"):
        ops.add_pos(x, pos, 50, q8=True)


@pytest.mark.parametrize("B,L,heads,dh", [(2, 128, 12, 64), (4, 64, 8, 96)])
def test_bert_attention_q8_equals_quantised_context(B, L, heads, dh):
    """The attention kernel's fused MX-fp8 context (config 5's O-proj operand): the bf16 context equals
    the plain kernel's bit for bit and the operand equals mmr_quantize_mxfp8 of it; bf16=False
    writes the same operand without the bf16 copy."""
    g = torch.Generator().manual_seed(B * L + dh)
    C = heads * dh
    qkv = (torch.randn(B, L, 3 * C, generator=g) * 2).to(torch.bfloat16).to(DEV)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[0, L // 2:] = 0
    mask = mask.to(DEV)
    ref = ops.bert_attention(qkv, mask, heads, dh)
    ctx, c8 = ops.bert_attention(qkv, mask, heads, dh, q8=True)
    _, c8b = ops.bert_attention(qkv, mask, heads, dh, q8=True, bf16=False)
    ref8 = ops.quantize_mxfp8(ref.view(B * L, C), layout=0)
    torch.cuda.synchronize()
    assert torch.equal(ctx, ref)
    for x8 in (c8, c8b):
        assert torch.equal(x8.q, ref8.q) and torch.equal(x8.s, ref8.s)


@pytest.mark.parametrize("B,lq,lk,heads,dh", [(256, 49, 128, 8, 96), (4, 128, 128, 8, 128), (512, 49, 64, 8, 96)])
def test_mha_q8_equals_quantised_output(B, lq, lk, heads, dh):
    """mmr_mha_q8 (the fusion head's fp8 out-projection operands, strided Q / K / V views of packed
    projections, ragged lq = 49 with the mean output beside it): the operand equals mmr_quantize_mxfp8 of
    the plain kernel's bf16 output bit for bit, and the mean is unchanged."""
    g = torch.Generator().manual_seed(B + lq + lk + dh)
    C = heads * dh
    qp = (torch.randn(B * lq, 3 * C, generator=g) * 2).to(torch.bfloat16).to(DEV)
    kv = (torch.randn(B * lk, 3 * C, generator=g) * 2).to(torch.bfloat16).to(DEV)
    sc = 1.0 / dh ** 0.5
    out = torch.empty(B * lq, C, dtype=torch.bfloat16, device=DEV)
    m_ref = torch.empty(B, C, device=DEV)
    ops.mha(qp[:, 2 * C:], kv[:, C:2 * C], kv[:, 2 * C:], B, lq, lk, heads, dh, sc, out=out, mean_out=m_ref)
    m8 = torch.empty(B, C, device=DEV)
    _, _, a8 = ops.mha(qp[:, 2 * C:], kv[:, C:2 * C], kv[:, 2 * C:], B, lq, lk, heads, dh, sc, mean_out=m8, q8=True)
    ref8 = ops.quantize_mxfp8(out, layout=0)
    torch.cuda.synchronize()
    assert torch.equal(a8.q, ref8.q) and torch.equal(a8.s, ref8.s)
    assert torch.equal(m8, m_ref)


@pytest.mark.parametrize("B,np_,c", [(256, 49, 256), (1280, 49, 1024)])
def test_assemble_seq_q8_equals_quantised_sequence(B, np_, c):
    """The combiner's fp8 QKV operand (config 5) written by the sequence assembly itself equals
    mmr_quantize_mxfp8 of the bf16 sequence bit for bit (values and scale bytes); B*(np_+2) % 256 == 0."""
    g = torch.Generator().manual_seed(B + c)
    x1 = (torch.randn(B, c, generator=g) * 3).to(DEV)
    x2 = (torch.randn(B, c, generator=g) * 0.5).to(DEV)
    pf = (torch.randn(B * np_, c, generator=g) * 2).to(torch.bfloat16).to(DEV)
    pe = (torch.randn(np_ + 2, c, generator=g) * 0.1).to(DEV)
    seq = ops.assemble_seq(x1, pf, x2, pe, np_).view(B * (np_ + 2), c)
    s8 = ops.assemble_seq(x1, pf, x2, pe, np_, q8=True)
    ref8 = ops.quantize_mxfp8(seq, layout=0)
    torch.cuda.synchronize()
    assert torch.equal(s8.q, ref8.q) and torch.equal(s8.s, ref8.s)


@pytest.mark.parametrize("B,L,C", [(2, 128, 768), (4, 64, 256), (8, 96, 1024)])
def test_bert_embed_q8_equals_quantised_embedding(B, L, C):
    """The fp8 BERT tower's embedding LayerNorm writes the first QKV operand: y equal to bert_embed bit
    for bit, the operand equal to quantize_mxfp8(y) (values and scale bytes)."""
    g = torch.Generator().manual_seed(B * L + C)
    word = (torch.randn(1000, C, generator=g) * 0.05).to(DEV)
    pos = (torch.randn(512, C, generator=g) * 0.02).to(DEV)
    type0 = (torch.randn(C, generator=g) * 0.02).to(DEV)
    gam, bet = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV), (torch.randn(C, generator=g) * 0.1).to(DEV)
    ids = torch.randint(0, 1000, (B, L), generator=g).to(DEV)
    y, y8 = ops.bert_embed_q8(ids, word, pos, type0, gam, bet, 1e-12)
    ref = ops.bert_embed(ids, word, pos, type0, gam, bet, 1e-12)
    ref8 = ops.quantize_mxfp8(ref.reshape(-1, C), layout=0)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert torch.equal(y8.q, ref8.q)
    assert torch.equal(y8.s, ref8.s)
