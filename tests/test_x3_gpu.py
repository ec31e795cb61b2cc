"""GPU parity of the fp32-faithful tower mode (tower_dtype="x3", csrc/x3.hip, towers_x3.py).

The reference computes its towers and heads in fp32 (src/Model/fusion.py:198-199, 322-325,
model.py:365-479); the x3 mode keeps f32 activations and runs every contraction as
a_hi.b_hi + a_hi.b_lo + a_lo.b_hi on bf16 MFMA (~2^-17 relative per product, f32 accumulation).

Bars (written per test):
  * kernels vs f64 of the same f32 inputs: linear |err| <= 2^-15 * (|x| @ |w|^T) + 1e-6 * max|ref|
    (the split's per-product bound with margin), attention max|err| <= 5e-5 * max|ref|;
  * towers vs the f64 oracle (oracle/towers.py run in double): max|err| <= 5e-4 * max|ref| — an
    order below the bf16 towers' 4e-2 — and vs the reference's own fp32 goldens (towers_mini.npz);
  * end to end: x3 towers + GPU exact kNN against the fp32 oracle towers + the
    sklearn-path top-10 (src/Evaluate/retrieval_overlap.py:84-115) on EVERY query of a B = 256 batch
    over the 100k x 768 labelled gallery: oracle.knn.topk_equivalent (tie_tol 1e-6, scores within
    1e-4) and identical P@10 / R@10 / MRR under random labels.
"""
import json
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mmr_amd import _lib, metrics, ops, synthetic
from mmr_amd.model import Backbones, MultiModalRetrievalModel, build_bench_model
from mmr_amd.retrieval import MI355XRetrievalEngine
from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
from mmr_amd.towers_x3 import BertTowerX3, SwinTowerX3
from oracle import knn as oknn
from oracle import towers as otw

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(got, ref):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)


@pytest.mark.parametrize("M,N,K,act,bias,res", [(1000, 96, 96, 0, True, False), (513, 2304, 768, 0, True, False),
                                                (300, 3072, 768, 1, True, False), (257, 768, 3072, 0, True, True),
                                                (77, 288, 64, 1, True, True), (4096, 200, 384, 0, False, False),
                                                (20000, 384, 1536, 0, False, False),
                                                # M % 256 == 0, N % 192 / 256 == 0: the K' = 3 kp split GEMM on the
                                                # 8-phase kernel (mmr_x3_linear_p8), K padded to 128 where needed
                                                (4096, 2304, 768, 0, True, False), (2048, 3072, 768, 1, True, False),
                                                (2048, 768, 3072, 0, True, True), (8192, 384, 96, 1, True, False),
                                                (4096, 192, 384, 0, False, True), (256, 1152, 200, 0, True, True),
                                                (65536, 576, 192, 0, True, False),
                                                # N not a multiple of 192 / 256: weight rows zero-padded to 192s,
                                                # the f32 epilogue drops the padded columns (buffer range check)
                                                (2048, 96, 384, 0, True, True), (2048, 288, 96, 1, True, False),
                                                (1024, 200, 64, 0, True, True)])
def test_x3_linear_vs_f64(M, N, K, act, bias, res):
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g) if bias else None
    r = torch.randn(M, N, generator=g) if res else None
    ref = x.double() @ w.double().T
    if b is not None:
        ref = ref + b.double()
    if act == 1:
        ref = F.gelu(ref)
    if r is not None:
        ref = ref + r.double()
    y = ops.x3_linear(x.to(DEV), ops.X3W(w.to(DEV)), b.to(DEV) if b is not None else None,
                      residual=r.to(DEV) if r is not None else None, act=act)
    err = (y.double().cpu() - ref).abs()
    absdot = x.double().abs() @ w.double().abs().T
    bound = 2.0 ** -15 * absdot + 1e-6 * ref.abs().max()
    f32 = x @ w.T  # the reference's own f32 GEMM, for scale
    print(json.dumps({"x3_max_err": err.max().item(), "f32_gemm_max_err": (f32.double() - x.double() @ w.double().T)
                      .abs().max().item()}))
    assert (err <= bound).all(), (err - bound).max().item()


def test_x3_linear_p8_inplace_residual_and_route():
    """The split-GEMM route with the residual in place (residual = out, as the towers call it) equals
    the out-of-place result bit for bit, and agrees with the 128 x 128 x3 kernel (the rows-not-a-
    multiple-of-256 route) within the split's error."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 1024, 768, 768
    x = torch.randn(M, K, generator=g).to(DEV)
    wx = ops.X3W((torch.randn(N, K, generator=g) * 0.05).to(DEV))
    b = torch.randn(N, generator=g).to(DEV)
    r = torch.randn(M, N, generator=g).to(DEV)
    y = ops.x3_linear(x, wx, b, residual=r)
    r2 = r.clone()
    ops.x3_linear(x, wx, b, residual=r2, out=r2)
    assert torch.equal(y, r2)
    # the first M - 1 rows through the 128 x 128 kernel (M - 1 is not a multiple of 256)
    y_old = ops.x3_linear(x[:M - 1], wx, b, residual=r[:M - 1])
    assert (y_old - y[:M - 1]).abs().max().item() <= 1e-5 * y.abs().max().item()


@pytest.mark.parametrize("M,C,Fw,res", [(2048, 768, 3072, False),   # BERT FFN (fc1 -> fc2, no residual)
                                       (1024, 96, 384, True),      # Swin stage-1 MLP: fc2 N = 96 (one padded tile)
                                       (2048, 192, 768, True),     # Swin stage-2 MLP, residual in fc2
                                       (512, 768, 3072, True), (768, 384, 1536, True),
                                       (1000, 768, 3072, False)])  # rows not a multiple of 256: unfused
def test_x3_ffn_split_handoff_bitwise(M, C, Fw, res):
    """x3_ffn (fc1 writes fc2's [hi | lo] operand rows, fc2 reads them as they are)
    equals x3_linear(GELU) -> x3_linear bit for bit where fc2 alone takes the 8-phase route (N >= 192;
    N = 96 runs the 128 x 128 x3 kernel alone: same products, another summation order -> 1e-5 of max),
    and stays within the x3 bound of f64."""
    g = torch.Generator().manual_seed(M + C + Fw)
    x = torch.randn(M, C, generator=g).to(DEV)
    w1 = ops.X3W((torch.randn(Fw, C, generator=g) * C ** -0.5).to(DEV))
    b1 = (torch.randn(Fw, generator=g) * 0.1).to(DEV)
    w2 = ops.X3W((torch.randn(C, Fw, generator=g) * Fw ** -0.5).to(DEV))
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    r = torch.randn(M, C, generator=g).to(DEV) if res else None
    y = ops.x3_ffn(x, w1, b1, w2, b2, residual=r)
    ref = ops.x3_linear(ops.x3_linear(x, w1, b1, act=1), w2, b2, residual=r)
    torch.cuda.synchronize()
    if C >= 192 or M % 256:
        assert torch.equal(y, ref)
    else:
        assert (y - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    h64 = F.gelu(x.double() @ w1.w.double().T + b1.double())
    y64 = h64 @ w2.w.double().T + b2.double() + (r.double() if r is not None else 0)
    assert _rel(y, y64) < 1e-5


@pytest.mark.parametrize("T,C", [(4096, 96), (1000, 96), (2048, 192), (77, 192)])
def test_x3_swin_mlp_vs_f64(T, C):
    """The fused x3 Swin MLP (LN -> fc1 -> erf GELU -> fc2 -> + x, hidden on chip) against f64, and against
    the unfused x3 chain (x3_ln_split -> x3_ffn) within the x3 bound; ragged token counts."""
    g_ = torch.Generator().manual_seed(T + C)
    x = (torch.randn(T, C, generator=g_) * 1.5 + 0.3).to(DEV)
    gm = (1 + 0.1 * torch.randn(C, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(C, generator=g_)).to(DEV)
    w1 = (torch.randn(4 * C, C, generator=g_) * C ** -0.5).to(DEV)
    b1 = (0.1 * torch.randn(4 * C, generator=g_)).to(DEV)
    w2 = (torch.randn(C, 4 * C, generator=g_) * (4 * C) ** -0.5).to(DEV)
    b2 = (0.1 * torch.randn(C, generator=g_)).to(DEV)
    pack = ops.x3_swin_mlp_pack(w1, w2)
    y = ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)
    xd = x.double().cpu()
    z = (xd - xd.mean(-1, keepdim=True)) / torch.sqrt(xd.var(-1, unbiased=False, keepdim=True) + 1e-5)
    z = z * gm.double().cpu() + bt.double().cpu()
    hid = F.gelu(z @ w1.double().cpu().T + b1.double().cpu())
    y64 = xd + hid @ w2.double().cpu().T + b2.double().cpu()
    assert _rel(y, y64) < 1e-5
    h = ops.x3_ln_split(x, gm, bt, 1e-5)
    y_chain = ops.x3_ffn(h, ops.X3W(w1), b1, ops.X3W(w2), b2, residual=x)
    assert _rel(y, y_chain) < 1e-5


@pytest.mark.parametrize("T", [4096, 1000, 33])
def test_x3_swin_mlp_workgroup_forms_bit_identical(T):
    """The C = 96 MLP's 4-wave workgroups (the default) and 8-wave ones run the same per-token products in the
    same order: bit-identical outputs, ragged token counts (partial last workgroup)."""
    C = 96
    g_ = torch.Generator().manual_seed(T + 7)
    x = (torch.randn(T, C, generator=g_) * 1.5 + 0.3).to(DEV)
    gm = (1 + 0.1 * torch.randn(C, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(C, generator=g_)).to(DEV)
    w1 = (torch.randn(4 * C, C, generator=g_) * C ** -0.5).to(DEV)
    b1 = (0.1 * torch.randn(4 * C, generator=g_)).to(DEV)
    w2 = (torch.randn(C, 4 * C, generator=g_) * (4 * C) ** -0.5).to(DEV)
    b2 = (0.1 * torch.randn(C, generator=g_)).to(DEV)
    pack = ops.x3_swin_mlp_pack(w1, w2)
    with ops.pinned(ops.PIN_X3_MLP, 0):
        y0 = ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)
    with ops.pinned(ops.PIN_X3_MLP, 1):
        y1 = ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)
    y = ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(y, y1)


@pytest.mark.parametrize("T,C,N,mode", [(4096, 96, 288, "ln"), (1000, 96, 96, "xs"), (2048, 192, 576, "ln"),
                                         (300, 192, 192, "xs"), (512, 96, 96, "ln_res")])
def test_x3_rowlin_vs_f64(T, C, N, mode):
    """The streamed x3 row-linear: LN(x) W^T + b (the Swin norm1 + qkv) and xs W^T + b + r (proj over the
    window attention's split rows) against f64, and against the x3 GEMM route within the x3 bound."""
    g_ = torch.Generator().manual_seed(T + C + N)
    x = (torch.randn(T, C, generator=g_) * 1.5 + 0.2).to(DEV)
    gm = (1 + 0.1 * torch.randn(C, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(C, generator=g_)).to(DEV)
    w = (torch.randn(N, C, generator=g_) * C ** -0.5).to(DEV)
    b = (0.1 * torch.randn(N, generator=g_)).to(DEV)
    r = torch.randn(T, N, generator=g_).to(DEV) if mode != "ln" else None
    pack = ops.x3_rowlin_pack(w)
    xd = x.double().cpu()
    if mode.startswith("ln"):
        y = ops.x3_rowlin(x, pack, b, N, ln=(gm, bt, 1e-5), residual=r)
        z = (xd - xd.mean(-1, keepdim=True)) / torch.sqrt(xd.var(-1, unbiased=False, keepdim=True) + 1e-5)
        z = z * gm.double().cpu() + bt.double().cpu()
        y_gemm = ops.x3_linear(ops.x3_ln_split(x, gm, bt, 1e-5), ops.X3W(w), b, residual=r)
    else:
        kp = _lib.lib().mmr_x3_p8_kpad(C)
        xr = ops.X3Rows(_split_bits(x, kp).view(torch.bfloat16), C, kp, (T,))
        y = ops.x3_rowlin(xr, pack, b, N, residual=r)
        z = xr.t[:, :C].double().cpu() + xr.t[:, kp:kp + C].double().cpu()  # the split rows' exact value
        y_gemm = ops.x3_linear(x, ops.X3W(w), b, residual=r)
    y64 = z @ w.double().cpu().T + b.double().cpu() + (r.double().cpu() if r is not None else 0)
    assert y.shape == (T, N)
    assert _rel(y, y64) < 1e-5
    assert _rel(y, y_gemm) < 1e-5


@pytest.mark.parametrize("rows,c,res", [(1024, 96, True), (512, 192, False), (768, 384, True), (256, 768, True),
                                        (256, 100, False), (13, 768, True), (7, 96, False)])
def test_ln_rows_split(rows, c, res):
    """mmr_ln_rows_split: the f32 LayerNorm within f32 rounding of ln_rows and of f64, and the split
    rows bit-identical to splitting its own f32 output (zero columns c..kp); ragged row counts."""
    g_ = torch.Generator().manual_seed(rows + c)
    x = (torch.randn(rows, c, generator=g_) * 3 + 1).to(DEV)
    r = torch.randn(rows, c, generator=g_).to(DEV) if res else None
    g = (1 + 0.1 * torch.randn(c, generator=g_)).to(DEV)
    b = (0.1 * torch.randn(c, generator=g_)).to(DEV)
    L = _lib.lib()
    kp = L.mmr_x3_p8_kpad(c)
    y = torch.empty(rows, c, device=DEV)
    xs = torch.full((rows, 2 * kp), 12345, dtype=torch.int16, device=DEV).view(torch.bfloat16)
    s = _lib.stream_ptr()
    assert L.mmr_ln_rows_split(_lib.ptr(x), c, None, _lib.ptr(r), c if res else 0, _lib.ptr(g), _lib.ptr(b),
                               _lib.ptr(y), c, _lib.ptr(xs), rows, c, 1e-5, s) == 0
    torch.cuda.synchronize()
    ref = ops.ln_rows(x, g, b, 1e-5, residual=r)
    z = x.double() + (r.double() if res else 0)
    z64 = (z - z.mean(-1, keepdim=True)) / torch.sqrt(z.var(-1, unbiased=False, keepdim=True) + 1e-5) * g.double() + b.double()
    assert (y - ref).abs().max().item() <= 2e-6 * ref.abs().max().item()
    assert _rel(y, z64) < 2e-6
    hi = y.to(torch.bfloat16)
    lo = (y - hi.float()).to(torch.bfloat16)
    u = xs.view(torch.int16)
    assert torch.equal(u[:, :c], hi.view(torch.int16)) and torch.equal(u[:, kp:kp + c], lo.view(torch.int16))
    assert (u[:, c:kp] == 0).all() and (u[:, kp + c:] == 0).all()
    # y optional: the split alone
    xs2 = torch.empty_like(xs)
    assert L.mmr_ln_rows_split(_lib.ptr(x), c, None, _lib.ptr(r), c if res else 0, _lib.ptr(g), _lib.ptr(b), None, 0,
                               _lib.ptr(xs2), rows, c, 1e-5, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(xs2.view(torch.int16), u)


@pytest.mark.parametrize("rows,c", [(512, 768), (256, 96), (300, 96), (256, 100), (64, 1024)])
def test_ln_alpha_product_rounded(rows, c):
    """LN(alpha * x + r) (PreFusionEnhancer, reference src/Model/fusion.py:33): the kernels round the
    product, then add — bit for bit the same as feeding torch's own rounded alpha * x with no alpha, for
    ln_rows and for the split LayerNorm (f32 output and split rows); hipcc may not contract the product
    into the residual add."""
    g_ = torch.Generator().manual_seed(rows * 7 + c)
    x = (torch.randn(rows, c, generator=g_) * 3 + 0.5).to(DEV)
    r = torch.randn(rows, c, generator=g_).to(DEV)
    gm = (1 + 0.1 * torch.randn(c, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(c, generator=g_)).to(DEV)
    alpha = torch.tensor([0.7377123], device=DEV)
    xa = alpha * x
    assert torch.equal(ops.ln_rows(x, gm, bt, 1e-5, alpha=alpha, residual=r), ops.ln_rows(xa, gm, bt, 1e-5, residual=r))
    y1, s1 = ops.x3_ln_split(x, gm, bt, 1e-5, residual=r, keep_f32=True, alpha=alpha)
    y0, s0 = ops.x3_ln_split(xa, gm, bt, 1e-5, residual=r, keep_f32=True)
    torch.cuda.synchronize()
    assert torch.equal(y1, y0)
    if isinstance(s1, ops.X3Rows):
        assert torch.equal(s1.t.view(torch.int16), s0.t.view(torch.int16))


@pytest.mark.parametrize("M,C,Fw", [(1024, 96, 384), (512, 768, 3072), (768, 384, 1536)])
def test_x3_split_rows_operand_bitwise(M, C, Fw):
    """A LayerNorm's split rows (x3_ln_split -> X3Rows) feed x3_linear / x3_ffn with the same bits as
    the f32 LayerNorm output does (the x3 towers' LN -> QKV / FFN pairs)."""
    g_ = torch.Generator().manual_seed(M + Fw)
    x = torch.randn(M, C, generator=g_).to(DEV)
    r = torch.randn(M, C, generator=g_).to(DEV)
    g = (1 + 0.1 * torch.randn(C, generator=g_)).to(DEV)
    b = (0.1 * torch.randn(C, generator=g_)).to(DEV)
    wq = ops.X3W((torch.randn(3 * C, C, generator=g_) * C ** -0.5).to(DEV))
    bq = torch.randn(3 * C, generator=g_).to(DEV)
    w1 = ops.X3W((torch.randn(Fw, C, generator=g_) * C ** -0.5).to(DEV))
    b1 = (torch.randn(Fw, generator=g_) * 0.1).to(DEV)
    w2 = ops.X3W((torch.randn(C, Fw, generator=g_) * Fw ** -0.5).to(DEV))
    b2 = (torch.randn(C, generator=g_) * 0.1).to(DEV)
    y, xr = ops.x3_ln_split(x, g, b, 1e-5, residual=r, keep_f32=True)
    assert isinstance(xr, ops.X3Rows)
    assert torch.equal(ops.x3_linear(xr, wq, bq), ops.x3_linear(y, wq, bq))
    assert torch.equal(ops.x3_linear(xr, w1, b1, act=1), ops.x3_linear(y, w1, b1, act=1))
    assert torch.equal(ops.x3_ffn(xr, w1, b1, w2, b2, residual=x), ops.x3_ffn(y, w1, b1, w2, b2, residual=x))
    # no bias (a zero bias on the split-input kernel) and a strided output: the same bits
    assert torch.equal(ops.x3_linear(xr, wq), ops.x3_linear(y, wq))
    o = torch.empty(3 * C, M, device=DEV).t()
    ops.x3_linear(xr, wq, bq, out=o)
    assert torch.equal(o, ops.x3_linear(y, wq, bq))
    torch.cuda.synchronize()


def test_x3_linear_p8_split_flags_rejected():
    """The split GEMM's preconditions fail loudly at the C-ABI."""
    L = _lib.lib()
    x = torch.zeros(256, 2 * 384, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(384, 2 * 384, dtype=torch.bfloat16, device=DEV)
    b = torch.zeros(384, dtype=torch.float32, device=DEV)
    y = torch.zeros(256, 2 * 384, dtype=torch.bfloat16, device=DEV)
    s = _lib.stream_ptr()
    P = _lib.ptr
    # split output with a residual / n not a multiple of 384; a NULL weight image; m not a multiple of
    # 256; k past 4096; the split LayerNorm with c % 4 != 0 / misaligned rows
    assert L.mmr_x3_linear_p8(P(x), P(w), P(b), P(b), P(y), 256, 384, 384, 0, 1, s) != 0
    assert L.mmr_x3_linear_p8(P(x), P(w), P(b), None, P(y), 256, 192, 384, 0, 1, s) != 0
    assert L.mmr_x3_linear_p8(P(x), None, P(b), None, P(y), 256, 384, 384, 0, 0, s) != 0
    assert L.mmr_x3_linear_p8(P(x), P(w), P(b), None, P(y), 255, 384, 384, 0, 0, s) != 0
    assert L.mmr_x3_linear_p8(P(x), P(w), P(b), None, P(y), 256, 384, 4097, 0, 0, s) != 0
    f = torch.zeros(8, 100, device=DEV)
    assert L.mmr_ln_rows_split(P(f), 100, None, None, 0, P(b), P(b), None, 0, P(y), 8, 98, 1e-5, s) != 0
    assert L.mmr_ln_rows_split(P(f), 99, None, None, 0, P(b), P(b), None, 0, P(y), 8, 96, 1e-5, s) != 0
    torch.cuda.synchronize()


def _attn_ref(q, k, v, b, lq, lk, heads, dh, scale, mask=None):
    qh = q.double().view(b, lq, heads, dh).transpose(1, 2)
    kh = k.double().view(b, lk, heads, dh).transpose(1, 2)
    vh = v.double().view(b, lk, heads, dh).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale
    if mask is not None:
        s = s.masked_fill(mask[:, None, None, :] == 0, float("-inf"))
    return (s.softmax(-1) @ vh).transpose(1, 2).reshape(b, lq, heads * dh)


@pytest.mark.parametrize("b,lq,lk,heads,dh,use_mask,mean", [(3, 128, 128, 12, 64, True, False),
                                                          (5, 49, 128, 8, 96, False, True),
                                                          (4, 51, 51, 8, 128, False, True),
                                                          (2, 1, 49, 8, 96, False, True),
                                                          (3, 130, 70, 2, 48, True, True),
                                                          (2, 128, 1, 8, 96, False, True),
                                                          (2, 100, 77, 4, 64, True, True), (3, 65, 128, 2, 32, False, False)])
def test_x3_attention_vs_f64(b, lq, lk, heads, dh, use_mask, mean):
    g = torch.Generator().manual_seed(b * 1000 + lq + lk + dh)
    C = heads * dh
    q = torch.randn(b * lq, 3 * C, generator=g) * 0.7           # strided views of packed rows
    kv = torch.randn(b * lk, 3 * C, generator=g) * 0.7
    mask = None
    if use_mask:
        lens = torch.randint(1, lk + 1, (b,), generator=g)
        mask = (torch.arange(lk)[None, :] < lens[:, None]).to(torch.int64)
    scale = 1.0 / math.sqrt(dh)
    ref = _attn_ref(q[:, :C], kv[:, C:2 * C], kv[:, 2 * C:], b, lq, lk, heads, dh, scale, mask)
    qd, kvd = q.to(DEV), kv.to(DEV)
    out = torch.empty((b * lq, C), dtype=torch.float32, device=DEV)
    m = torch.empty((b, C), dtype=torch.float32, device=DEV) if mean else None
    ops.x3_attention(qd[:, :C], kvd[:, C:2 * C], kvd[:, 2 * C:], b, lq, lk, heads, dh, scale, out=out, mean_out=m,
                     mask=mask.to(DEV) if mask is not None else None)
    assert _rel(out.view(b, lq, C), ref) <= 5e-5
    if mean:
        assert _rel(m, ref.mean(1)) <= 5e-5


@pytest.mark.parametrize("lq,lk,dh", [(40, 40, 64), (128, 128, 64), (7, 70, 96)])
def test_x3_attention_all_masked_row_is_hf_uniform(lq, lk, dh):
    """HF BertSelfAttention adds (1 - mask) * finfo(f32).min to the scaled scores: a sequence whose keys
    are ALL masked gets a uniform softmax (every score rounds to finfo.min), i.e. the mean of V over the lk
    keys — not zeros.  f64 restatement of that additive mask; batch 1 keeps a partial mask, batch 2 none
    (parity unpinned: the reference holds no fixture for an all-zero attention_mask)."""
    b, heads = 3, 2
    g = torch.Generator().manual_seed(lq + lk + dh)
    C = heads * dh
    q = torch.randn(b * lq, C, generator=g) * 0.7
    k = torch.randn(b * lk, C, generator=g) * 0.7
    v = torch.randn(b * lk, C, generator=g) * 0.7
    mask = torch.ones(b, lk, dtype=torch.int64)
    mask[0] = 0
    mask[1, lk // 3:] = 0
    scale = 1.0 / math.sqrt(dh)
    qh = q.double().view(b, lq, heads, dh).transpose(1, 2)
    kh = k.double().view(b, lk, heads, dh).transpose(1, 2)
    vh = v.double().view(b, lk, heads, dh).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale + (1.0 - mask.double())[:, None, None, :] * torch.finfo(torch.float32).min
    ref = (s.softmax(-1) @ vh).transpose(1, 2).reshape(b, lq, C)
    assert torch.allclose(ref[0], vh[0].mean(1).reshape(1, C).expand(lq, C))
    out = torch.empty((b * lq, C), dtype=torch.float32, device=DEV)
    m = torch.empty((b, C), dtype=torch.float32, device=DEV)
    ops.x3_attention(q.to(DEV), k.to(DEV), v.to(DEV), b, lq, lk, heads, dh, scale, out=out, mean_out=m,
                     mask=mask.to(DEV))
    assert _rel(out.view(b, lq, C), ref) <= 5e-5
    assert _rel(m, ref.mean(1)) <= 5e-5


@pytest.mark.parametrize("hw,c,heads,shift", [(56, 96, 3, 0), (56, 96, 3, 3), (14, 384, 12, 3), (7, 768, 24, 0)])
def test_x3_swin_window_attention_vs_f64(hw, c, heads, shift):
    """roll(-shift) / window partition / q*dh^-0.5 k^T + rel-pos bias + shift mask / softmax / v /
    reverse / roll(+shift) (timm WindowAttention, restated with oracle/towers.py's helpers) in f64."""
    B, ws = 2, 7
    g = torch.Generator().manual_seed(hw + c + shift)
    qkv = torch.randn(B, hw, hw, 3 * c, generator=g) * 0.7
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5
    bias = ops.swin_attn_bias(table.to(DEV), heads, ws, hw, shift)
    out = ops.x3_swin_window_attention(qkv.to(DEV).contiguous(), bias, hw, heads, ws, shift)
    dh, N = c // heads, ws * ws
    x = qkv.double()
    if shift:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    win = otw.window_partition(x, ws).view(-1, N, 3, heads, dh).permute(2, 0, 3, 1, 4)
    q, k, v = win[0] * dh ** -0.5, win[1], win[2]
    a = q @ k.transpose(-2, -1)
    a = a + table.double()[otw.relative_position_index(ws).view(-1)].view(N, N, heads).permute(2, 0, 1)[None]
    if shift:
        msk = otw.shift_mask(hw, hw, ws, shift).double()
        nW = msk.shape[0]
        a = (a.view(-1, nW, heads, N, N) + msk[None, :, None]).view(-1, heads, N, N)
    o = (a.softmax(-1) @ v).transpose(1, 2).reshape(-1, ws, ws, c)
    o = otw.window_reverse(o, ws, hw, hw)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    assert _rel(out, o) <= 5e-5


def _swin_attn_half_f64(x, g, b, wqkv, bqkv, wp, bp, table, heads, ws, shift, eps=1e-5):
    """x + proj(W-MSA(LN1(x))) (timm SwinTransformerBlock's attention half) in f64, oracle helpers."""
    x = x.double()
    B, hw, _, c = x.shape
    dh, N = c // heads, ws * ws
    h = F.layer_norm(x, (c,), g.double(), b.double(), eps)
    qkv = h @ wqkv.double().T + bqkv.double()
    if shift:
        qkv = torch.roll(qkv, shifts=(-shift, -shift), dims=(1, 2))
    win = otw.window_partition(qkv, ws).view(-1, N, 3, heads, dh).permute(2, 0, 3, 1, 4)
    q, k, v = win[0] * dh ** -0.5, win[1], win[2]
    a = q @ k.transpose(-2, -1)
    a = a + table.double()[otw.relative_position_index(ws).view(-1)].view(N, N, heads).permute(2, 0, 1)[None]
    if shift:
        msk = otw.shift_mask(hw, hw, ws, shift).double()
        nW = msk.shape[0]
        a = (a.view(-1, nW, heads, N, N) + msk[None, :, None]).view(-1, heads, N, N)
    o = (a.softmax(-1) @ v).transpose(1, 2).reshape(-1, ws, ws, c)
    o = otw.window_reverse(o, ws, hw, hw)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    return x + o @ wp.double().T + bp.double()


@pytest.mark.parametrize("B,shift", [(4, 0), (4, 3), (1, 3), (3, 0)])
def test_x3_swin_attn_block_vs_chain_and_f64(B, shift):
    """The fused stage-1 attention half (mmr_x3_swin_attn_block, C = 96) against the unfused x3 chain it
    replaces (x3_rowlin norm1 + qkv -> window attention -> x3_rowlin proj + residual: same products,
    another kernel's summation order) and against f64 (timm's attention half restated)."""
    c, heads, ws, hw = 96, 3, 7, 56
    gen = torch.Generator().manual_seed(100 + B + shift)
    x = torch.randn(B, hw, hw, c, generator=gen)
    lg, lb = 1 + 0.1 * torch.randn(c, generator=gen), 0.1 * torch.randn(c, generator=gen)
    wqkv, bqkv = torch.randn(3 * c, c, generator=gen) * c ** -0.5, 0.1 * torch.randn(3 * c, generator=gen)
    wp, bp = torch.randn(c, c, generator=gen) * c ** -0.5, 0.1 * torch.randn(c, generator=gen)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=gen) * 0.5
    d = [t.to(DEV) for t in (x, lg, lb, wqkv, bqkv, wp, bp)]
    xd, lgd, lbd, wqd, bqd, wpd, bpd = d
    bias = ops.swin_attn_bias(table.to(DEV), heads, ws, hw, shift)
    pack = ops.x3_swin_attn_block_pack(wqd, bqd, wpd, bpd, lgd, lbd)
    assert pack is not None
    y = ops.x3_swin_attn_block(xd, pack, bias, ws, shift, 1e-5)
    assert y.shape == x.shape and torch.isfinite(y).all()
    ref = _swin_attn_half_f64(x, lg, lb, wqkv, bqkv, wp, bp, table, heads, ws, shift)
    err = _rel(y, ref)
    if B * hw * hw % 256 == 0:
        qkv = ops.x3_rowlin(xd, ops.x3_rowlin_pack(wqd), bqd, 3 * c, ln=(lgd, lbd, 1e-5))
        a = ops.x3_swin_window_attention_split(qkv, bias, hw, heads, ws, shift)
        chain = ops.x3_rowlin(a, ops.x3_rowlin_pack(wpd), bpd, c, residual=xd)
        dc = _rel(y, chain)
        print(json.dumps({"B": B, "shift": shift, "vs_f64": err, "vs_chain": dc, "chain_vs_f64": _rel(chain, ref)}))
        assert dc <= 1e-5  # both ~4e-6 from f64 (the products' 2^-17 bound), in different orders
    assert err <= 1e-5


def test_x3_swin_tower_fused_attn_half_matches_chain():
    """Swin-T x3 forward_features (random init, B = 2) with the fused stage-1 attention half against the same
    tower on the unfused chain (fused_attn = False): same f32 features within the products' error."""
    ssd = init_swin_state(SWIN_T, 11)
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(2, 12))).to(DEV)
    sw = SwinTowerX3(ssd, SWIN_T, DEV)
    assert sw.stages[0]["blocks"][0]["sab_pack"] is not None and sw.stages[1]["blocks"][0]["sab_pack"] is None
    f_fused = sw.forward_features(img)
    sw.fused_attn = False
    f_chain = sw.forward_features(img)
    d = _rel(f_fused, f_chain)
    print(json.dumps({"fused_vs_chain": d}))
    assert d <= 1e-5


def test_x3_swin_attn_block_rejects():
    """Unbuilt widths / windows are refused with MMR_ERR_UNSUPPORTED (pack: 0 bytes, None from ops)."""
    assert _lib.lib().mmr_x3_swin_attn_block_pack_bytes(192) == 0
    w = torch.zeros(3 * 192, 192, device=DEV)
    assert ops.x3_swin_attn_block_pack(w, w[0], w[:192], w[0, :192], w[0, :192], w[0, :192]) is None


def _split_bits(y, kp):
    """[hi | lo] rows (int16 view) of f32 rows y (rows, c), zero columns c..kp: mmr_x3_split_rows' split."""
    c = y.shape[-1]
    hi = y.to(torch.bfloat16)
    lo = (y - hi.float()).to(torch.bfloat16)
    out = torch.zeros(y.shape[0], 2 * kp, dtype=torch.int16, device=y.device)
    out[:, :c] = hi.view(torch.int16)
    out[:, kp:kp + c] = lo.view(torch.int16)
    return out


@pytest.mark.parametrize("hw,c,heads,shift,B", [(56, 96, 3, 3, 4), (28, 192, 6, 0, 16), (14, 384, 12, 3, 64),
                                                (7, 768, 24, 0, 256)])  # B hw^2 = 12544 tokens = 49 x 256
def test_x3_swin_window_attention_split_rows(hw, c, heads, shift, B):
    """The window attention's split-row output (the proj operand) equals the split of its f32 output
    bit for bit, padding columns zero; proj through it equals proj through the f32 rows."""
    ws = 7
    g = torch.Generator().manual_seed(hw + c + shift + 1)
    qkv = (torch.randn(B, hw, hw, 3 * c, generator=g) * 0.7).to(DEV)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5
    bias = ops.swin_attn_bias(table.to(DEV), heads, ws, hw, shift)
    ref = ops.x3_swin_window_attention(qkv, bias, hw, heads, ws, shift)
    xr = ops.x3_swin_window_attention_split(qkv, bias, hw, heads, ws, shift)
    assert isinstance(xr, ops.X3Rows) and xr.lead == (B, hw, hw)
    assert torch.equal(xr.t.view(torch.int16), _split_bits(ref.reshape(-1, c), xr.kp))
    w = ops.X3W((torch.randn(c, c, generator=g) * c ** -0.5).to(DEV))
    b = torch.randn(c, generator=g).to(DEV)
    r = torch.randn(B, hw, hw, c, generator=g).to(DEV)
    torch.cuda.synchronize()
    y_split = ops.x3_linear(xr, w, b, residual=r)
    if c >= 192:  # N = 96 alone runs the 128 x 128 x3 kernel (another summation order)
        assert torch.equal(y_split, ops.x3_linear(ref, w, b, residual=r))
    y64 = ref.double() @ w.w.double().T + b.double() + r.double()
    assert _rel(y_split, y64) < 1e-5


@pytest.mark.parametrize("b,l,heads,dh,use_mask", [(8, 128, 12, 64, True), (4, 64, 8, 96, False)])
def test_x3_attention_split_rows(b, l, heads, dh, use_mask):
    """BERT-shaped x3 attention with split-row output (the O-proj operand) = the split of the f32 output."""
    g = torch.Generator().manual_seed(b * l + dh)
    C = heads * dh
    qkv = (torch.randn(b * l, 3 * C, generator=g) * 0.7).to(DEV)
    mask = torch.ones(b, l, dtype=torch.int64)
    if use_mask:
        for i in range(b):
            mask[i, l - 7 * i:] = 0
    mask = mask.to(DEV)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    out = torch.empty(b * l, C, device=DEV)
    ops.x3_attention(q, k, v, b, l, l, heads, dh, dh ** -0.5, out=out, mask=mask)
    xr = ops.x3_attention_split(q, k, v, b, l, l, heads, dh, dh ** -0.5, mask=mask)
    torch.cuda.synchronize()
    assert isinstance(xr, ops.X3Rows)
    assert torch.equal(xr.t.view(torch.int16), _split_bits(out, xr.kp))


@pytest.mark.parametrize("B,hw,c", [(16, 56, 96), (64, 28, 192), (256, 14, 384), (256, 14, 100), (2, 6, 52),
                                    (2, 6, 50)])  # 12544 merged tokens = 49 x 256; 4c = 400: kp 512; c % 4 != 0
def test_x3_patch_merge_ln(B, hw, c):
    """timm PatchMerging (2x2 gather in x0..x3 order, LayerNorm over 4c) in f32 vs f64; the split-row
    form (the reduction linear's operand) = the split of the f32 rows, and the reduction through it
    equals the reduction through the f32 rows bit for bit (merged token counts of 256-row tiles)."""
    g_ = torch.Generator().manual_seed(B * hw + c)
    x = (torch.randn(B, hw, hw, c, generator=g_) * 2 + 0.5).to(DEV)
    gm = (1 + 0.1 * torch.randn(4 * c, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(4 * c, generator=g_)).to(DEV)
    y = ops.x3_patch_merge_ln(x, gm, bt, 1e-5)
    xd = x.double()
    m = torch.cat([xd[:, 0::2, 0::2], xd[:, 1::2, 0::2], xd[:, 0::2, 1::2], xd[:, 1::2, 1::2]], -1)
    ref = (m - m.mean(-1, keepdim=True)) / torch.sqrt(m.var(-1, unbiased=False, keepdim=True) + 1e-5) * gm.double() + bt.double()
    assert _rel(y, ref) < 2e-6
    xr = ops.x3_patch_merge_ln_split(x, gm, bt, 1e-5)
    if not isinstance(xr, ops.X3Rows):
        assert (B * (hw // 2) ** 2) % 256 or c % 4
        return
    assert torch.equal(xr.t.view(torch.int16), _split_bits(y.reshape(-1, 4 * c), xr.kp))
    w = ops.X3W((torch.randn(2 * c, 4 * c, generator=g_) * (4 * c) ** -0.5).to(DEV))
    assert torch.equal(ops.x3_linear(xr, w), ops.x3_linear(y, w))
    torch.cuda.synchronize()


@pytest.mark.parametrize("B,cin,hw,kp", [(3, 3, 224, 64), (2, 3, 32, 48), (2, 5, 16, 96)])
def test_x3_patch_im2col_exact(B, cin, hw, kp):
    """The patch-embed im2col (k = c p^2 + ky p + kx, zero columns past cin p^2) = torch's unfold, bit for bit."""
    img = torch.randn(B, cin, hw, hw, generator=torch.Generator().manual_seed(hw + cin)).to(DEV)
    cols = ops.x3_patch_im2col(img, 4, kp)
    g = hw // 4
    ref = img.view(B, cin, g, 4, g, 4).permute(0, 2, 4, 1, 3, 5).reshape(B, g * g, cin * 16)
    torch.cuda.synchronize()
    assert torch.equal(cols[..., :cin * 16], ref) and (cols[..., cin * 16:] == 0).all()


@pytest.mark.parametrize("B,hw", [(3, 224), (2, 32), (1, 64)])
def test_x3_patch_embed_ln_vs_f64(B, hw):
    """The fused x3 Swin stem (conv 4x4/s4, 3 -> 96, + its LayerNorm) vs the f64 conv + LayerNorm, and vs the
    unfused x3 route (im2col -> x3_linear -> ln_rows); timm-scale inputs (normalised pixels, fan-in init)."""
    g_ = torch.Generator().manual_seed(hw + B)
    img = (torch.randn(B, 3, hw, hw, generator=g_) * 1.5).to(DEV)
    w = (torch.randn(96, 3, 4, 4, generator=g_) * 48 ** -0.5).to(DEV)
    bias = (torch.randn(96, generator=g_) * 0.1).to(DEV)
    gm = (1 + 0.2 * torch.randn(96, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(96, generator=g_)).to(DEV)
    pack = ops.x3_patch_embed_pack(w)
    y = ops.x3_patch_embed_ln(img, pack, bias, gm, bt, 1e-5)
    ref = torch.nn.functional.conv2d(img.double(), w.double(), bias.double(), stride=4).permute(0, 2, 3, 1)
    ref = torch.nn.functional.layer_norm(ref, (96,), gm.double(), bt.double(), 1e-5)
    assert y.shape == (B, hw // 4, hw // 4, 96)
    assert _rel(y, ref) < 2e-5
    kp = 64
    wp = torch.zeros(96, kp, device=DEV)
    wp[:, :48] = w.reshape(96, 48)
    cols = ops.x3_patch_im2col(img, 4, kp)
    un = ops.x3_linear(cols, ops.X3W(wp), bias)
    un = ops.ln_rows(un.reshape(-1, 96), gm, bt, 1e-5).view(y.shape)
    assert _rel(y, un) < 2e-5
    torch.cuda.synchronize()


@pytest.mark.parametrize("rows,l,c", [(256 * 51, 51, 768), (1000, 7, 6), (4 * 130, 130, 1024)])
def test_x3_add_pos_exact(rows, l, c):
    g = torch.Generator().manual_seed(rows + c)
    x = torch.randn(rows, c, generator=g).to(DEV)
    pos = torch.randn(l, c, generator=g).to(DEV)
    y = ops.x3_add_pos(x, pos, l)
    torch.cuda.synchronize()
    assert torch.equal(y, x + pos.repeat(rows // l + 1, 1)[:rows])


def _assert_split_of(xr, y):
    """X3Rows xr = the split of f32 rows y bit for bit (padding columns zero)."""
    assert isinstance(xr, ops.X3Rows)
    assert torch.equal(xr.t.view(torch.int16), _split_bits(y.reshape(-1, y.shape[-1]), xr.kp))


@pytest.mark.parametrize("rows,l,c", [(256 * 51, 51, 768), (512, 128, 96), (256, 1, 1000)])
def test_x3_add_pos_split_bitwise(rows, l, c):
    """add-pos writing the in_proj operand: f32 rows equal x3_add_pos, split rows = their split."""
    g = torch.Generator().manual_seed(rows + c + 1)
    x = torch.randn(rows, c, generator=g).to(DEV)
    pos = torch.randn(l, c, generator=g).to(DEV)
    y, xr = ops.x3_add_pos_split(x, pos, l)
    ref = ops.x3_add_pos(x, pos, l)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    _assert_split_of(xr, ref)
    _, xr2 = ops.x3_add_pos_split(x, pos, l, keep_f32=False)
    torch.cuda.synchronize()
    assert torch.equal(xr2.t.view(torch.int16), xr.t.view(torch.int16))


def test_x3_assemble_seq_split_bitwise():
    b, np_, c = 256, 49, 768  # 256 * 51 rows
    g = torch.Generator().manual_seed(11)
    x1, x2 = torch.randn(b, c, generator=g).to(DEV), torch.randn(b, c, generator=g).to(DEV)
    pf = torch.randn(b * np_, c, generator=g).to(DEV)
    pe = torch.randn(np_ + 2, c, generator=g).to(DEV)
    xr = ops.x3_assemble_seq_split(x1, pf, x2, pe, np_)
    torch.cuda.synchronize()
    _assert_split_of(xr, ops.x3_assemble_seq(x1, pf, x2, pe, np_))


@pytest.mark.parametrize("rows,c", [(512, 768), (12544, 768), (256, 96)])
def test_ln_rows_split_alpha(rows, c):
    """LN(alpha x + residual) (the PreFusionEnhancer norm) in the split form: within f32 rounding of
    ln_rows(alpha=...) and of f64; split rows = the split of its own f32 output."""
    g_ = torch.Generator().manual_seed(rows + c + 7)
    x = (torch.randn(rows, c, generator=g_) * 2).to(DEV)
    r = torch.randn(rows, c, generator=g_).to(DEV)
    g = (1 + 0.1 * torch.randn(c, generator=g_)).to(DEV)
    b = (0.1 * torch.randn(c, generator=g_)).to(DEV)
    alpha = torch.tensor([0.37], device=DEV)
    y, xr = ops.x3_ln_split(x, g, b, 1e-5, residual=r, keep_f32=True, alpha=alpha)
    ref = ops.ln_rows(x, g, b, 1e-5, alpha=alpha, residual=r)
    torch.cuda.synchronize()
    z = 0.37 * x.double() + r.double()
    z64 = (z - z.mean(-1, keepdim=True)) / torch.sqrt(z.var(-1, unbiased=False, keepdim=True) + 1e-5) * g.double() + b.double()
    assert (y - ref).abs().max().item() <= 2e-6 * ref.abs().max().item()
    assert _rel(y, z64) < 2e-6
    _assert_split_of(xr, y)


def test_x3_attention_split_with_mean():
    """The i2t cross attention's form: split-row output AND the query-row mean in one launch, equal to
    the f32 form's output (split bit for bit) and mean."""
    b, lq, lk, heads, dh = 256, 49, 128, 8, 96
    g = torch.Generator().manual_seed(3)
    C = heads * dh
    q = (torch.randn(b * lq, C, generator=g) * 0.7).to(DEV)
    kv = (torch.randn(b * lk, 2 * C, generator=g) * 0.7).to(DEV)
    out = torch.empty(b * lq, C, device=DEV)
    m_ref = torch.empty(b, C, device=DEV)
    ops.x3_attention(q, kv[:, :C], kv[:, C:], b, lq, lk, heads, dh, dh ** -0.5, out=out, mean_out=m_ref)
    m = torch.empty(b, C, device=DEV)
    xr = ops.x3_attention_split(q, kv[:, :C], kv[:, C:], b, lq, lk, heads, dh, dh ** -0.5, mean_out=m)
    torch.cuda.synchronize()
    _assert_split_of(xr, out)
    assert torch.equal(m, m_ref)


@pytest.mark.parametrize("b,np_,c", [(256, 49, 768), (3, 5, 6)])
def test_x3_assemble_seq_exact(b, np_, c):
    """seq = [x1; patches; x2] + pe (fusion.py:451-468 + model.py:397), bit for bit."""
    g = torch.Generator().manual_seed(b + c)
    x1, x2 = torch.randn(b, c, generator=g).to(DEV), torch.randn(b, c, generator=g).to(DEV)
    pf = torch.randn(b * np_, c, generator=g).to(DEV)
    pe = torch.randn(np_ + 2, c, generator=g).to(DEV)
    seq = ops.x3_assemble_seq(x1, pf, x2, pe, np_)
    ref = torch.cat([x1[:, None], pf.view(b, np_, c), x2[:, None]], 1) + pe[None]
    torch.cuda.synchronize()
    assert torch.equal(seq, ref)


def _double(sd):
    return {k: v.double() for k, v in sd.items()}


def test_x3_towers_vs_f64_oracle():
    """Swin-T + BERT-base (random init, the bench geometry) at B = 2 against the oracle run in f64,
    with the fp32 oracle's own distance from f64 printed beside it."""
    ssd, bsd = init_swin_state(SWIN_T, 5), init_bert_state(BERT_BASE, 6)
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(2, 9)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(2, 128, 10))
    sw = SwinTowerX3(ssd, SWIN_T, DEV)
    bt = BertTowerX3(bsd, BERT_BASE, DEV)
    f_gpu = sw.forward_features(img.to(DEV))
    t_gpu = bt.forward(ids.to(DEV), mask.to(DEV))
    with torch.no_grad():
        f64 = otw.swin_forward_features(img.double(), _double(ssd), SWIN_T["depths"], SWIN_T["num_heads"])
        t64 = otw.bert_forward(ids, mask, _double(bsd), 12, 12)
        f32 = otw.swin_forward_features(img, ssd, SWIN_T["depths"], SWIN_T["num_heads"])
        t32 = otw.bert_forward(ids, mask, bsd, 12, 12)
    rep = {"swin_x3": _rel(f_gpu, f64), "swin_f32_oracle": _rel(f32, f64), "bert_x3": _rel(t_gpu, t64),
           "bert_f32_oracle": _rel(t32, t64)}
    print(json.dumps(rep))
    assert rep["swin_x3"] <= 5e-4 and rep["bert_x3"] <= 5e-4


def test_x3_mini_towers_match_reference_golden():
    """The reference's own fp32 outputs (towers_mini.npz: Backbones.forward + all three heads,
    multimodal with 2 fusion layers) reproduced by the x3 mode to 2e-4 * max|ref| (the bf16 mode: 4e-2)."""
    f = np.load(os.path.join(GOLDEN, "towers_mini.npz"), allow_pickle=False)
    cfg = json.loads(bytes(f["cfg"]).decode())
    w = {k[2:]: torch.from_numpy(synthetic.bf16_bits_to_f32(f[k]).copy()) for k in f.files if k.startswith("w:")}
    swin = {k[5:]: v for k, v in w.items() if k.startswith("swin.")}
    bert = {k[5:]: v for k, v in w.items() if k.startswith("bert.")}
    head = {k[5:]: v for k, v in w.items() if k.startswith("head.")}
    scfg = dict(SWIN_T, embed_dim=cfg["swin"]["embed_dim"], depths=cfg["swin"]["depths"],
                num_heads=cfg["swin"]["num_heads"])
    bcfg = dict(BERT_BASE, **cfg["bert"])
    bb = Backbones(swin_state=swin, bert_state=bert, swin_cfg=scfg, bert_cfg=bcfg, device=DEV, tower_dtype="x3")
    image = torch.from_numpy(synthetic.image_from_u8(f["img_u8"])).to(DEV)
    ids = torch.from_numpy(f["input_ids"]).to(DEV)
    mask = torch.from_numpy(f["attention_mask"]).to(DEV)
    (g, p), t = bb(image, ids, mask)
    errs = {"img_global": _rel(g, torch.from_numpy(f["img_global"])),
            "img_patches": _rel(p, torch.from_numpy(f["img_patches"])),
            "txt_feats": _rel(t, torch.from_numpy(f["txt_feats"]))}
    for mt in ("text", "image", "multimodal"):
        m = MultiModalRetrievalModel(joint_dim=cfg["joint_dim"], num_heads=cfg["num_heads"], model_type=mt,
                                     backbones=bb, head_state=head, device=DEV, use_shared_ffn=False)
        o = m(image, ids, mask)
        for k in ("joint_emb", "img_emb", "txt_emb"):
            errs[f"{mt}_{k}"] = _rel(o[k], torch.from_numpy(f[f"{mt}_{k}"]))
    print(json.dumps(errs))
    assert max(errs.values()) <= 2e-4, errs


def _labels(n, seed):
    rng = np.random.default_rng(seed)
    lab = np.zeros((n, synthetic.NUM_LABELS), np.uint8)
    for i in range(n):
        lab[i, rng.choice(synthetic.NUM_LABELS, size=int(rng.integers(1, 4)), replace=False)] = 1
    return synthetic.labels_to_bits(lab)


def _metrics(idx, qb, gbits, K=10):
    rel = [[str(j) for j in np.nonzero(gbits & qb[q])[0]] for q in range(len(qb))]
    p = np.mean([metrics.precision_at_k([str(j) for j in idx[q]], rel[q], K) for q in range(len(qb))])
    mrr, _, rec = metrics.ranking_metrics(idx, qb, gbits, K)
    return {"P@10": float(p), "R@10": float(rec), "MRR": float(mrr)}


@pytest.mark.parametrize("model_type", ["multimodal", "text"])
def test_e2e_x3_batch_256_identical_topk(model_type):
    """BASELINE.md §3 end to end: the bench model (Swin-T + BERT-base + 5-layer multimodal head, or the
    text head) in the x3 mode at B = 256, every query against the fp32 oracle path (oracle towers +
    head -> sklearn cosine_similarity + argsort, retrieval_overlap.py:84-115) over a 100k x 768
    labelled gallery: topk_equivalent on every query (tie_tol 1e-6, scores within 1e-4) and identical
    P@10 / R@10 / MRR under random query labels."""
    m = build_bench_model(device=DEV, joint_dim=768, model_type=model_type, tower_dtype="x3")
    B = 256
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 71)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(B, 128, 72))
    imgd = img.to(DEV) if model_type == "multimodal" else None
    q_gpu = m.query_embeddings(imgd, ids.to(DEV), mask.to(DEV)).float().cpu().numpy()
    from mmr_amd.model import init_fusion_state, init_head_state
    ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
    hsd = init_head_state(768, 768, 768, 2711)
    with torch.no_grad():
        if model_type == "multimodal":
            hsd.update(init_fusion_state(768, 768, 768, 8, 5, 2712))
            (g, p), t = otw.backbones_forward(img, ids, mask, ssd, bsd, SWIN_T, BERT_BASE)
            q_cpu = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"].numpy()
        else:
            t = otw.bert_forward(ids, mask, bsd, 12, 12)
            q_cpu = otw.heads(None, None, t, hsd, "text")["joint_emb"].numpy()
    G, gl = synthetic.labelled_gallery(100_000, 768, 73)
    gbits = synthetic.labels_to_bits(gl)
    eng = MI355XRetrievalEngine(embs=G, ids=[str(i) for i in range(len(G))], dtype="fp32")
    gi, gs = eng.search(np.ascontiguousarray(q_gpu), K=10)
    eng.close()
    gi = gi.cpu().numpy() if isinstance(gi, torch.Tensor) else np.asarray(gi)
    gs = gs.cpu().numpy() if isinstance(gs, torch.Tensor) else np.asarray(gs)
    ci, cs = oknn.sklearn_topk(q_cpu, G, 10)
    cos = np.sum(q_gpu * q_cpu, 1) / (np.linalg.norm(q_gpu, axis=1) * np.linalg.norm(q_cpu, axis=1))
    ok, msg = oknn.topk_equivalent(ci, cs, gi, gs, tie_tol=1e-6, score_tol=1e-4)
    qb = _labels(B, 74)
    mg, mc = _metrics(gi, qb, gbits), _metrics(ci, qb, gbits)
    print(json.dumps({"model_type": model_type, "topk_equivalent": msg, "min_embedding_cosine": float(cos.min()),
                      "max_rel_emb_err": float(np.abs(q_gpu - q_cpu).max() / np.abs(q_cpu).max()),
                      "exact_list_match": float(np.mean([np.array_equal(gi[i], ci[i]) for i in range(B)])),
                      "gpu": mg, "cpu": mc}))
    assert ok, msg
    assert mg == mc
