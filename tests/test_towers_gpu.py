"""GPU parity of the tower kernels (bf16 compute, f32 accumulation) against plain-torch fp32
references on CPU (oracle/towers.py, pinned to the reference by tests/golden/towers_mini.npz).

Tolerances (bf16 activations/weights, written per test): kernel-level max|err| <= tol * max|ref|;
end-to-end embeddings: cosine(GPU, oracle) >= 0.999 per row and max|err| <= 4e-2 * max|ref|."""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mmr_amd import ops, synthetic
from mmr_amd.model import Backbones, MultiModalRetrievalModel
from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state
from oracle import towers as otw

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(got, ref):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-12)


def bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,act,bias,res", [(1000, 96, 96, 0, True, False), (513, 2304, 768, 0, True, False),
                                                (300, 3072, 768, 1, True, False), (257, 768, 3072, 0, True, True),
                                                (4096, 192, 384, 0, False, False), (77, 288, 64, 1, True, True),
                                                (16461, 3072, 768, 1, True, False),     # 256x256 tiles, M tail
                                                (32768, 768, 768, 0, True, True),       # 256x128 tiles
                                                (32000, 768, 3072, 0, True, True)])
def test_linear_bf16(M, N, K, act, bias, res):
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g) if bias else None
    r = torch.randn(M, N, generator=g) if res else None
    ref = bf(x).float() @ bf(w).float().T
    if b is not None:
        ref = ref + b
    if act == 1:
        ref = F.gelu(ref)
    if r is not None:
        ref = ref + bf(r).float()
    y = ops.linear(bf(x).to(DEV), bf(w).to(DEV), b.to(DEV) if b is not None else None,
                   bf(r).to(DEV) if r is not None else None, act=act)
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("cfg", [7, 8])
@pytest.mark.parametrize("M,N,K,act,bias,res", [(32768, 1152, 128, 0, True, False), (32768, 1152, 384, 0, True, True),
                                                (65536, 768, 768, 0, False, True), (32768, 2304, 256, 0, False, False),
                                                (16384, 768, 3072, 0, True, True), (32768, 1536, 384, 1, True, False),
                                                (32768, 768, 128, 0, True, True), (4096, 1536, 128, 0, False, True)])
def test_linear_bf16_p8_persistent(request, cfg, M, N, K, act, bias, res):
    """The persistent 8-phase GEMM pinned (mmr_pin_variant: variant 9 = 256x256 tiles, 10 = 256x192) on shapes with
    2-4 tiles per workgroup and K = 128 ... 3072 (1 ... 12 K iterations per tile: the K stream runs
    on across tile boundaries; K = 128 with a residual: the one-iteration tile whose residual, loaded at
    the tile start, is counted out of the first wait), every epilogue; vs torch fp32 of the same bf16 operands (tolerance
    1e-2 * max|ref|: bf16 output rounding)."""
    if N % (256 if cfg == 7 else 192):
        pytest.skip("tile width")
    pin = ops.pinned(ops.PIN_GEMM_BF16, {7: 9, 8: 10}[cfg])
    pin.__enter__()
    request.addfinalizer(lambda: pin.__exit__(None, None, None))
    g = torch.Generator(device=DEV).manual_seed(M + N + K + cfg)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=DEV) if bias else None
    r = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16) if res else None
    ref = x.float() @ w.float().T
    if b is not None:
        ref = ref + b
    if act == 1:
        ref = F.gelu(ref)
    if r is not None:
        ref = ref + r.float()
    y = ops.linear(x, w, b, r, act=act)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 1e-2
    # every row block written
    assert ((y.float() - ref).abs().amax(dim=1) <= 2e-2 * ref.abs().max()).all()


@pytest.mark.parametrize("M,N,K,bias,res", [(3136 * 4 + 17, 96, 64, True, False), (784 * 8 + 5, 576, 192, True, False),
                                            (784 * 8 + 5, 192, 192, True, True), (784 * 2, 192, 192, False, False),
                                            (1000, 384, 192, True, True), (31, 576, 192, True, True),
                                            (500, 32, 64, True, False), (300, 160, 192, False, True)])
def test_linear_rw(M, N, K, bias, res):
    """mmr_linear_rw (resident-weight streaming linear: Swin patch embed / stage-2 qkv, proj /
    PatchMerging 1->2 shapes, N split into LDS-sized parts, ragged token counts) vs torch fp32 of the
    same bf16 operands (tolerance 1e-2 * max|ref|) and vs mmr_linear_bf16."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g) if bias else None
    r = torch.randn(M, N, generator=g) if res else None
    ref = bf(x).float() @ bf(w).float().T
    if b is not None:
        ref = ref + b
    if r is not None:
        ref = ref + bf(r).float()
    pk = ops.rw_pack(bf(w).to(DEV))
    assert pk is not None
    args = (b.to(DEV) if b is not None else None, bf(r).to(DEV) if r is not None else None)
    y = ops.linear_rw(bf(x).to(DEV), pk, *args)
    assert rel_err(y, ref) < 1e-2
    y2 = ops.linear(bf(x).to(DEV), bf(w).to(DEV), *args)
    assert rel_err(y, y2) < 1e-2


def test_linear_rw_rejects():
    assert ops.rw_pack(bf(torch.randn(96, 96)).to(DEV)) is None       # K = 96
    assert ops.rw_pack(bf(torch.randn(3072, 768)).to(DEV)) is None    # K = 768
    assert ops.rw_pack(bf(torch.randn(384, 384)).to(DEV)) is None     # K = 384 (dropped: spilled)


@pytest.mark.parametrize("T,C", [(1000, 96), (3136 * 4 + 17, 96), (64, 192), (784 * 8 + 5, 192), (1, 96)])
def test_swin_mlp_fused(T, C):
    """mmr_swin_mlp == x + fc2(GELU(fc1(LN(x)))) (fusion.py:198-199 via timm Mlp), ragged token counts;
    hidden activation rounded to bf16 as in the unfused path.  Tolerance: 2e-2 * max|ref|."""
    g = torch.Generator().manual_seed(T + C)
    x = bf(torch.randn(T, C, generator=g) * 2)
    lg, lb = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    w1, b1 = bf(torch.randn(4 * C, C, generator=g) * C ** -0.5), 0.1 * torch.randn(4 * C, generator=g)
    w2, b2 = bf(torch.randn(C, 4 * C, generator=g) * (4 * C) ** -0.5), 0.1 * torch.randn(C, generator=g)
    h = bf(F.layer_norm(x.float(), (C,), lg, lb, 1e-5)).float()
    h = bf(F.gelu(h @ w1.float().T + b1)).float()
    ref = h @ w2.float().T + b2 + x.float()
    pack = ops.swin_mlp_pack(w1.to(DEV), w2.to(DEV))
    y = ops.swin_mlp(x.to(DEV), lg.to(DEV), lb.to(DEV), pack, b1.to(DEV), b2.to(DEV), 1e-5)
    assert rel_err(y, ref) < 2e-2
    # the unfused kernels agree too (same bf16 rounding points)
    h2 = ops.layernorm(x.to(DEV), lg.to(DEV), lb.to(DEV), 1e-5)
    h2 = ops.linear(h2, w1.to(DEV), b1.to(DEV), act=1)
    y2 = ops.linear(h2, w2.to(DEV), b2.to(DEV), residual=x.to(DEV))
    assert rel_err(y, y2.float().cpu()) < 2e-2


def test_layernorm_bf16():
    x = torch.randn(1000, 768) * 3 + 1
    g, b = torch.randn(768), torch.randn(768)
    ref = F.layer_norm(bf(x).float(), (768,), g, b, 1e-5)
    y = ops.layernorm(bf(x).to(DEV), g.to(DEV), b.to(DEV), 1e-5)
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("rows,c", [(1000, 768), (77, 384), (4096, 96)])
def test_add_layernorm_bf16(rows, c):
    """LN(x + r) as HF BertSelfOutput/BertOutput compute it (sum then LayerNorm), tolerance 1e-2."""
    g = torch.Generator().manual_seed(rows + c)
    x, r = bf(torch.randn(rows, c, generator=g)), bf(torch.randn(rows, c, generator=g) * 2)
    ga, be = 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    ref = F.layer_norm(x.float() + r.float(), (c,), ga, be, 1e-12)
    y = ops.add_layernorm(x.to(DEV), r.to(DEV), ga.to(DEV), be.to(DEV), 1e-12)
    assert rel_err(y, ref) < 1e-2


def test_bert_attention_masked():
    B, L, H, dh = 3, 128, 12, 64
    g = torch.Generator().manual_seed(1)
    qkv = torch.randn(B, L, 3 * H * dh, generator=g)
    ids, mask = synthetic.reports(B, L, 7)
    mask = torch.from_numpy(mask)
    q, k, v = bf(qkv).float().split(H * dh, -1)
    hd = lambda t: t.view(B, L, H, dh).transpose(1, 2)  # noqa: E731
    s = hd(q) @ hd(k).transpose(-1, -2) / 8.0 + (1.0 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    ref = (s.softmax(-1) @ hd(v)).transpose(1, 2).reshape(B, L, H * dh)
    y = ops.bert_attention(bf(qkv).to(DEV), mask.to(DEV), H, dh)
    assert rel_err(y, ref) < 2e-2


@pytest.mark.parametrize("L", [64, 256, 512])
def test_bert_attention_lengths(L):
    B, H, dh = 2, 2, 64
    qkv = torch.randn(B, L, 3 * H * dh)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[1, L // 3:] = 0
    q, k, v = bf(qkv).float().split(H * dh, -1)
    hd = lambda t: t.view(B, L, H, dh).transpose(1, 2)  # noqa: E731
    s = hd(q) @ hd(k).transpose(-1, -2) / 8.0 + (1.0 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    ref = (s.softmax(-1) @ hd(v)).transpose(1, 2).reshape(B, L, H * dh)
    y = ops.bert_attention(bf(qkv).to(DEV), mask.to(DEV), H, dh)
    assert rel_err(y, ref) < 2e-2


def _swin_attn_ref(qkv, table, H, heads, ws, shift):
    """Window attention core (timm WindowAttention + roll/partition) from the oracle's pieces."""
    B = qkv.shape[0]
    C = qkv.shape[-1] // 3
    hd = C // heads
    N = ws * ws
    x = qkv.view(B, H, H, 3 * C)
    if shift:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    win = otw.window_partition(x, ws).view(-1, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = win[0] * hd ** -0.5, win[1], win[2]
    a = q @ k.transpose(-2, -1)
    bias = table[otw.relative_position_index(ws).view(-1)].view(N, N, heads).permute(2, 0, 1)
    a = a + bias[None]
    if shift:
        m = otw.shift_mask(H, H, ws, shift)
        a = (a.view(-1, m.shape[0], heads, N, N) + m[None, :, None]).view(-1, heads, N, N)
    o = (a.softmax(-1) @ v).transpose(1, 2).reshape(-1, ws, ws, C)
    o = otw.window_reverse(o, ws, H, H)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    return o


@pytest.mark.parametrize("H,heads,shift", [(56, 3, 0), (56, 3, 3), (28, 6, 3), (14, 12, 3), (7, 24, 0)])
def test_swin_window_attention(H, heads, shift):
    B, ws = 2, 7
    C = heads * 32
    g = torch.Generator().manual_seed(H + heads + shift)
    qkv = torch.randn(B, H, H, 3 * C, generator=g)
    table = torch.randn(169, heads, generator=g)
    ref = _swin_attn_ref(bf(qkv).float(), table, H, heads, ws, shift)
    y = ops.swin_window_attention(bf(qkv).to(DEV), ops.swin_attn_bias(table.to(DEV), heads, ws, H, shift),
                                  H, heads, ws, shift)
    assert rel_err(y, ref) < 2e-2


@pytest.mark.parametrize("B,H,c,want_y", [(64, 28, 192, True), (256, 28, 192, False), (256, 14, 384, True),
                                          (512, 14, 384, False)])
def test_patch_merge_ln_q8(B, H, c, want_y):
    """PatchMerging gather + LN(4c) emitting the reduction GEMM's MX-fp8 operand (fp8 stages 3-4: 4c =
    768 / 1536): y equal to the bf16 kernel bit for bit, the operand equal to quantize_mxfp8 of it."""
    g = torch.Generator().manual_seed(B + H + c)
    x = bf(torch.randn(B, H, H, c, generator=g)).to(DEV)
    gam, bet = (torch.randn(4 * c, generator=g) * 0.5 + 1).to(DEV), (torch.randn(4 * c, generator=g) * 0.1).to(DEV)
    y, m8 = ops.patch_merge_ln_q8(x, gam, bet, 1e-5, want_y=want_y)
    ref = ops.patch_merge_ln(x, gam, bet, 1e-5)
    ref8 = ops.quantize_mxfp8(ref.reshape(-1, 4 * c), layout=0)
    torch.cuda.synchronize()
    assert (y is None) == (not want_y)
    if want_y:
        assert torch.equal(y, ref)
    assert torch.equal(m8.q, ref8.q)
    assert torch.equal(m8.s, ref8.s)


@pytest.mark.parametrize("B,H,heads,shift,kp", [(128, 14, 12, 3, 512), (128, 14, 12, 0, 512), (256, 7, 24, 0, 768),
                                                (256, 7, 24, 0, 1024)])
def test_swin_window_attention_q8(B, H, heads, shift, kp):
    """The fp8 stages' window attention writing the proj GEMM's MX-fp8 operand (stage 3: C = 384, K
    padded to 512; stage 4: C = 768): bytes and scale bytes equal quantize_mxfp8 of the bf16 kernel's
    output, the padding included."""
    ws, C = 7, heads * 32
    g = torch.Generator().manual_seed(B + H + heads + shift)
    qkv = bf(torch.randn(B, H, H, 3 * C, generator=g)).to(DEV)
    bias = ops.swin_attn_bias(torch.randn(169, heads, generator=g).to(DEV), heads, ws, H, shift)
    a8 = ops.swin_window_attention_q8(qkv, bias, H, heads, ws, shift, kp=kp)
    ref8 = ops.quantize_mxfp8(ops.swin_window_attention(qkv, bias, H, heads, ws, shift), layout=0, kp=kp)
    torch.cuda.synchronize()
    assert a8.kp == kp and a8.k == C
    assert torch.equal(a8.q, ref8.q)
    assert torch.equal(a8.s, ref8.s)


@pytest.mark.parametrize("B,shift", [(2, 0), (2, 3), (5, 3)])
def test_swin_attn_block_fused(B, shift):
    """mmr_swin_attn_block == oracle swin_attn_half (timm: x + proj(W-MSA(norm1(x))) with roll,
    rel-pos bias and shift mask) at stage-1 geometry; tolerance 3e-2 * max|ref| (bf16 Q/K/V/P)."""
    g = torch.Generator().manual_seed(B * 10 + shift)
    C, H, heads, ws = 96, 56, 3, 7
    sd = {"b.norm1.weight": 1 + 0.1 * torch.randn(C, generator=g), "b.norm1.bias": 0.1 * torch.randn(C, generator=g),
          "b.attn.qkv.weight": bf(torch.randn(3 * C, C, generator=g) * C ** -0.5).float(),
          "b.attn.qkv.bias": 0.1 * torch.randn(3 * C, generator=g),
          "b.attn.proj.weight": bf(torch.randn(C, C, generator=g) * C ** -0.5).float(),
          "b.attn.proj.bias": 0.1 * torch.randn(C, generator=g),
          "b.attn.relative_position_bias_table": torch.randn(169, heads, generator=g)}
    x = bf(torch.randn(B, H, H, C, generator=g))
    ref = otw.swin_attn_half(x.float(), sd, "b.", heads, ws, shift)
    d = lambda k: sd["b." + k].to(DEV)
    pack = ops.swin_attn_block_pack(bf(d("attn.qkv.weight")), d("attn.qkv.bias"), bf(d("attn.proj.weight")),
                                    d("attn.proj.bias"), d("norm1.weight"), d("norm1.bias"))
    bias = ops.swin_attn_bias(d("attn.relative_position_bias_table"), heads, ws, H, shift)
    y = ops.swin_attn_block(x.to(DEV), pack, bias, ws, shift, 1e-5)
    assert rel_err(y, ref) < 3e-2
    # and the unfused kernel chain agrees
    h = ops.layernorm(x.to(DEV), d("norm1.weight"), d("norm1.bias"), 1e-5)
    qkv = ops.linear(h, bf(d("attn.qkv.weight")), d("attn.qkv.bias"))
    a = ops.swin_window_attention(qkv, bias, H, heads, ws, shift)
    y2 = ops.linear(a, bf(d("attn.proj.weight")), d("attn.proj.bias"), residual=x.to(DEV))
    assert rel_err(y, y2.float().cpu()) < 3e-2


def test_patch_im2col_and_merge():
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(2, 3)))
    cols = ops.patch_im2col(img.to(DEV)).float().cpu()
    ref = F.unfold(img, 4, stride=4).transpose(1, 2)  # (B, 3136, 48) in (c, ky, kx) order
    assert torch.equal(cols[..., :48], ref.to(torch.bfloat16).float())
    assert (cols[..., 48:] == 0).all()
    x = torch.randn(2, 28, 28, 96)
    g, b = torch.randn(384), torch.randn(384)
    xx = bf(x).float()
    ref = F.layer_norm(xx.reshape(2, 14, 2, 14, 2, 96).permute(0, 1, 3, 4, 2, 5).flatten(3), (384,), g, b, 1e-5)
    y = ops.patch_merge_ln(bf(x).to(DEV), g.to(DEV), b.to(DEV), 1e-5)
    assert rel_err(y, ref) < 1e-2



@pytest.mark.parametrize("B,hw", [(3, 224), (2, 32), (1, 64)])
def test_patch_embed_ln_bf16_fused(B, hw):
    """The bf16 towers' fused stem (mmr_patch_embed_ln_bf16: bf16 pixels x bf16 conv weight, bias + LayerNorm
    on the f32 accumulators, bf16 out) vs the f64 conv + LayerNorm of the same bf16-rounded operands: within
    one bf16 rounding of the output (2^-8 relative + 2e-3 absolute per element); and vs the unfused route
    (im2col -> GEMM -> LayerNorm, which also rounds the conv output to bf16) within 2 output ulps."""
    g_ = torch.Generator().manual_seed(7 * hw + B)
    img = (torch.randn(B, 3, hw, hw, generator=g_) * 1.5).to(DEV)
    w = (torch.randn(96, 3, 4, 4, generator=g_) * 48 ** -0.5).to(DEV)
    bias = (torch.randn(96, generator=g_) * 0.1).to(DEV)
    gm = (1 + 0.2 * torch.randn(96, generator=g_)).to(DEV)
    bt = (0.1 * torch.randn(96, generator=g_)).to(DEV)
    wb = bf(w.reshape(96, 48))
    pack = ops.x3_patch_embed_pack(wb.float().contiguous())
    y = ops.patch_embed_ln_bf16(img, pack, bias, gm, bt, 1e-5)
    assert y.shape == (B, hw // 4, hw // 4, 96) and y.dtype == torch.bfloat16
    ref = F.conv2d(bf(img).double(), wb.double().reshape(96, 3, 4, 4), bias.double(), stride=4).permute(0, 2, 3, 1)
    ref = F.layer_norm(ref, (96,), gm.double(), bt.double(), 1e-5)
    err = (y.double() - ref).abs()
    assert (err <= ref.abs() * 2.0 ** -8 + 2e-3).all(), err.max().item()
    wp = torch.zeros(96, 64, device=DEV)
    wp[:, :48] = wb.float()
    cols = ops.patch_im2col(img, 4)
    x = ops.layernorm(ops.linear(cols, bf(wp), bias), gm, bt, 1e-5).view(B, hw // 4, hw // 4, 96)
    assert ((y.float() - x.float()).abs() <= x.float().abs() * 2.0 ** -7 + 4e-3).all()


@pytest.mark.parametrize("B,H,C", [(2, 28, 96), (3, 14, 192), (1, 14, 384), (1, 2, 96), (5, 6, 192)])
def test_patch_merge_ln_geometries(B, H, C):
    """PatchMerging gather + LN (timm: x0..x3 = x[0::2,0::2], x[1::2,0::2], x[0::2,1::2], x[1::2,1::2]
    concatenated, LayerNorm(4C)) for the grouped-lane forms (4C = 384 / 768) and the generic one,
    incl. output row counts that leave a partial wave."""
    g0 = torch.Generator().manual_seed(B * H + C)
    x = torch.randn(B, H, H, C, generator=g0)
    g, b = torch.randn(4 * C, generator=g0), torch.randn(4 * C, generator=g0)
    xx = bf(x).float()
    h2 = H // 2
    ref = F.layer_norm(xx.reshape(B, h2, 2, h2, 2, C).permute(0, 1, 3, 4, 2, 5).flatten(3), (4 * C,), g, b, 1e-5)
    y = ops.patch_merge_ln(bf(x).to(DEV), g.to(DEV), b.to(DEV), 1e-5)
    assert rel_err(y, ref) < 1e-2


def test_swin_head_and_means():
    x = torch.randn(3, 49, 768) * 2
    g, b = torch.rand(768) + 0.5, torch.randn(768) * 0.1
    xx = bf(x).float()
    y1 = F.layer_norm(xx, (768,), g, b, 1e-5)
    patches, glob, pool = ops.swin_head(bf(x).to(DEV), g.to(DEV), b.to(DEV), 1e-5)
    p_ref = F.layer_norm(y1, (768,), g, b, 1e-5)
    assert rel_err(patches, p_ref) < 1e-4
    assert rel_err(glob, y1.mean(1)) < 1e-4
    assert rel_err(pool, torch.cat([y1.mean(1, keepdim=True), p_ref], 1).mean(1)) < 1e-4
    t = torch.randn(4, 128, 768)
    assert rel_err(ops.mean_tokens(bf(t).to(DEV)), bf(t).float().mean(1)) < 1e-5


def test_proj_head_l2norm():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(300, 768, generator=g)
    wp, bp = torch.randn(512, 768, generator=g) * 0.03, torch.randn(512, generator=g)
    w1, b1 = torch.randn(1024, 512, generator=g) * 0.03, torch.randn(1024, generator=g)
    w2, b2 = torch.randn(512, 1024, generator=g) * 0.03, torch.randn(512, generator=g)
    ref = F.linear(F.gelu(F.linear(F.linear(x, wp, bp), w1, b1)), w2, b2)
    y = ops.proj_head(*(t.to(DEV) for t in (x, wp, bp, w1, b1, w2, b2)), l2norm=False)
    assert rel_err(y, ref) < 1e-5
    yn = ops.proj_head(*(t.to(DEV) for t in (x, wp, bp, w1, b1, w2, b2)), l2norm=True)
    assert rel_err(yn, ref / ref.norm(dim=1, keepdim=True)) < 1e-5


def _check_emb(got, ref, tol=4e-2):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    cos = F.cosine_similarity(got.reshape(got.shape[0], -1), ref.reshape(ref.shape[0], -1), dim=1)
    assert cos.min().item() >= 0.999, cos
    assert rel_err(got, ref) <= tol


def test_mini_towers_match_reference_golden():
    f = np.load(os.path.join(GOLDEN, "towers_mini.npz"), allow_pickle=False)
    cfg = json.loads(bytes(f["cfg"]).decode())
    w = {k[2:]: torch.from_numpy(synthetic.bf16_bits_to_f32(f[k]).copy()) for k in f.files if k.startswith("w:")}
    swin = {k[5:]: v for k, v in w.items() if k.startswith("swin.")}
    bert = {k[5:]: v for k, v in w.items() if k.startswith("bert.")}
    head = {k[5:]: v for k, v in w.items() if k.startswith("head.")}
    scfg = dict(SWIN_T, embed_dim=cfg["swin"]["embed_dim"], depths=cfg["swin"]["depths"],
                num_heads=cfg["swin"]["num_heads"])
    bcfg = dict(BERT_BASE, **cfg["bert"])
    bb = Backbones(swin_state=swin, bert_state=bert, swin_cfg=scfg, bert_cfg=bcfg, device=DEV)
    image = torch.from_numpy(synthetic.image_from_u8(f["img_u8"])).to(DEV)
    ids = torch.from_numpy(f["input_ids"]).to(DEV)
    mask = torch.from_numpy(f["attention_mask"]).to(DEV)
    (g, p), t = bb(image, ids, mask)
    _check_emb(g, torch.from_numpy(f["img_global"]))
    _check_emb(p, torch.from_numpy(f["img_patches"]))
    _check_emb(t, torch.from_numpy(f["txt_feats"]))
    for mt in ("text", "image", "multimodal"):
        m = MultiModalRetrievalModel(joint_dim=cfg["joint_dim"], num_heads=cfg["num_heads"], model_type=mt,
                                     backbones=bb, head_state=head, device=DEV, use_shared_ffn=False)
        o = m(image, ids, mask)
        _check_emb(o["joint_emb"], torch.from_numpy(f[f"{mt}_joint_emb"]))
        _check_emb(o["img_emb"], torch.from_numpy(f[f"{mt}_img_emb"]))
        _check_emb(o["txt_emb"], torch.from_numpy(f[f"{mt}_txt_emb"]))


def test_full_size_towers_vs_oracle():
    """Swin-Tiny + BERT-base geometry (random init) vs the fp32 oracle, B=2."""
    ssd, bsd = init_swin_state(SWIN_T, 5), init_bert_state(BERT_BASE, 6)
    bb = Backbones(swin_state=ssd, bert_state=bsd, device=DEV)
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(2, 9)))
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(2, 128, 10))
    (g, p), t = bb(img.to(DEV), ids.to(DEV), mask.to(DEV))
    with torch.no_grad():
        (rg, rp), rt = otw.backbones_forward(img, ids, mask, ssd, bsd, SWIN_T, BERT_BASE)
    _check_emb(g, rg)
    _check_emb(p, rp)
    _check_emb(t, rt)


def test_checkpoint_path_reference_layout(tmp_path):
    """The reference's inference constructor path (model.py:116-137 arguments; checkpoint loaded as
    model.py:282-287 does, here with torch.load(..., weights_only=True)): the golden mini model's
    weights re-keyed into the reference state-dict layout (backbones.vision.* timm keys,
    backbones.bert.* HF keys, head keys) and saved; MultiModalRetrievalModel(checkpoint_path=...)
    reads the tower geometry off the weights and reproduces the golden outputs of all three heads.
    Without a checkpoint (training=False) it raises like the reference."""
    from test_boundary_cpu import _reference_layout_state
    sd, cfg = _reference_layout_state()
    p = tmp_path / "model_best.pt"
    torch.save(sd, p)
    f = np.load(os.path.join(GOLDEN, "towers_mini.npz"), allow_pickle=False)
    image = torch.from_numpy(synthetic.image_from_u8(f["img_u8"])).to(DEV)
    ids = torch.from_numpy(f["input_ids"]).to(DEV)
    mask = torch.from_numpy(f["attention_mask"]).to(DEV)
    for mt in ("text", "image", "multimodal"):
        m = MultiModalRetrievalModel(joint_dim=cfg["joint_dim"], num_heads=cfg["num_heads"], num_classes=43,
                                     num_fusion_layers=2, checkpoint_path=str(p), device=DEV, use_shared_ffn=False,
                                     model_type=mt)
        o = m(image, ids, mask)
        _check_emb(o["joint_emb"], torch.from_numpy(f[f"{mt}_joint_emb"]))
        _check_emb(o["img_emb"], torch.from_numpy(f[f"{mt}_img_emb"]))
        _check_emb(o["txt_emb"], torch.from_numpy(f[f"{mt}_txt_emb"]))
    with pytest.raises(ValueError, match="checkpoint_path must be provided"):
        MultiModalRetrievalModel(joint_dim=64, device=DEV)


def _ln_ref(y, g, b, eps):
    """LayerNorm over the last dim in f64 (the folded GEMMs' reference)."""
    y = y.double()
    mu = y.mean(-1, keepdim=True)
    var = ((y - mu) ** 2).mean(-1, keepdim=True)
    return (y - mu) / torch.sqrt(var + eps) * g.double() + b.double()


@pytest.mark.parametrize("M", [256, 4096])
def test_linear_ln_modes(M):
    """mmr_linear_bf16_ln, every built combination, vs f64 torch on the same bf16 operands:
    (0) plain residual + row statistics: the pairs sum to (sum y, sum y^2) of the stored bf16 rows;
    (1) LayerNorm folded into the consumer (QKV N=2304; FFN1 N=3072 + GELU): == LN(y) W^T + b;
    (2) normalised residual + statistics (O-proj / FFN2): == ctx W^T + b + LN(r).
    Raw rows carry a per-row mean and scale (the un-normalised BERT residual stream).  Tolerance
    1e-2 * max|ref| (bf16 output rounding + bf16 W diag(gamma))."""
    g = torch.Generator(device=DEV).manual_seed(M)
    C, eps = 768, 1e-12
    rnd = lambda *s: torch.randn(*s, generator=g, device=DEV)  # noqa: E731
    # producer: y = ctx Wo^T + bo + h (plain residual), with statistics
    ctx, h = bf(rnd(M, C)), bf(rnd(M, C) * 3 + rnd(M, 1) * 2)
    wo, bo = bf(rnd(C, C) * C ** -0.5), rnd(C)
    y, st = ops.linear_ln(ctx, wo, bo, residual=h, want_stats=True)
    ref_y = ctx.double() @ wo.double().T + bo.double() + h.double()
    assert rel_err(y, ref_y) < 1e-2
    yd = y.double()
    assert st.shape == (M, ops.linear_ln_parts(M, C, 0), 2)
    s = st.double().sum(1)
    assert torch.allclose(s[:, 0], yd.sum(1), rtol=1e-5, atol=1e-3)
    # second word: each part's centred sum of squares M2_p; Chan's merge gives the row's M2
    npart = st.shape[1]
    pm = st[..., 0].double() / (C // npart)
    m2 = st[..., 1].double().sum(1) + (C // npart) * ((pm - yd.mean(1, keepdim=True)) ** 2).sum(1)
    assert torch.allclose(m2, ((yd - yd.mean(1, keepdim=True)) ** 2).sum(1), rtol=1e-4, atol=1e-3)
    cf = ops.ln_row_coef(st, C, eps)
    yd64 = yd - yd.mean(1, keepdim=True)
    ref_cf = torch.stack([1 / torch.sqrt((yd64 ** 2).mean(1) + eps), -yd.mean(1) / torch.sqrt((yd64 ** 2).mean(1) + eps)], 1)
    assert torch.allclose(cf.double(), ref_cf, rtol=1e-4, atol=1e-5)
    gam, bet = 1 + 0.2 * rnd(C), 0.2 * rnd(C)
    from mmr_amd.towers import _ln_fold
    # fold (1): QKV-like and FFN1-like consumers
    for N, act in ((2304, 0), (3072, 1)):
        w, b = bf(rnd(N, C) * C ** -0.5), rnd(N)
        wf, c, d = _ln_fold(w, b, gam, bet)
        out, none = ops.linear_ln(y, wf, d, act=act, ln_mode=1, coef=cf, v1=c)
        assert none is None
        ref = _ln_ref(yd, gam, bet, eps) @ w.double().T + b.double()
        if act:
            ref = F.gelu(ref)
        assert rel_err(out, ref) < 1e-2, (N, act, rel_err(out, ref))
    # normalised residual (2) + statistics: FFN2-like (K = 3072)
    f1, w2, b2 = bf(rnd(M, 3072)), bf(rnd(C, 3072) * 3072 ** -0.5), rnd(C)
    y2, st2 = ops.linear_ln(f1, w2, b2, residual=y, ln_mode=2, coef=cf, v1=gam, v2=bet, want_stats=True)
    ref2 = f1.double() @ w2.double().T + b2.double() + _ln_ref(yd, gam, bet, eps)
    assert rel_err(y2, ref2) < 1e-2
    s2 = st2.double().sum(1)
    assert torch.allclose(s2[:, 0], y2.double().sum(1), rtol=1e-5, atol=1e-3)


def test_ln_row_coef_large_row_offset():
    """Rows whose |mean| is large against their spread (a residual stream offset by ~1e3): the producer's
    per-part (sum, centred M2) merged by Chan's formula keep the variance that E[y^2] - mean^2 in f32 loses
     — coefficients vs f64 on the stored bf16 rows."""
    g = torch.Generator(device=DEV).manual_seed(9)
    M, C, eps = 512, 768, 1e-12
    ctx = bf(torch.randn(M, C, generator=g, device=DEV))
    wo, bo = bf(torch.randn(C, C, generator=g, device=DEV) * C ** -0.5), torch.zeros(C, device=DEV)
    h = bf(torch.randn(M, C, generator=g, device=DEV) * 4 + 1000.0)
    y, st = ops.linear_ln(ctx, wo, bo, residual=h, want_stats=True)
    cf = ops.ln_row_coef(st, C, eps).double()
    yd = y.double()
    var = ((yd - yd.mean(1, keepdim=True)) ** 2).mean(1)
    rstd = 1 / torch.sqrt(var + eps)
    assert torch.allclose(cf[:, 0], rstd, rtol=2e-4), (cf[:, 0] / rstd - 1).abs().max().item()
    assert torch.allclose(cf[:, 1], -yd.mean(1) * rstd, rtol=2e-4)
    # the parts are n / nparts columns each: a row width they do not divide fails loudly
    with pytest.raises(Exception, match="equal parts"):
        ops.ln_row_coef(st, C + 2, eps)


def test_linear_ln_rejects():
    """Shapes and combinations the LayerNorm-fused GEMM does not build fail loudly."""
    x, w, b = bf(torch.randn(100, 768, device=DEV)), bf(torch.randn(768, 768, device=DEV)), torch.randn(768, device=DEV)
    with pytest.raises(Exception, match="multiple of 256"):
        ops.linear_ln(x, w, b, want_stats=True)
    x = bf(torch.randn(256, 768, device=DEV))
    with pytest.raises(Exception, match="without GELU"):
        ops.linear_ln(x, w, b, act=1, want_stats=True)
    with pytest.raises(Exception, match="not built"):
        ops.linear_ln(x, w, b, residual=x)


def test_bert_ln_fold_matches_unfused():
    """BERT-base tower (random init), B=4 x L=128: the LayerNorm-folded layer stack (towers.py
    _forward_folded) and the unfused one (add_layernorm passes) against the fp32 oracle — both at the
    end-to-end embedding bar (cosine >= 0.999, max|err| <= 4e-2 * max|ref|), and the folded stack's
    error no worse than 1.5x the unfused one's."""
    bsd = init_bert_state(BERT_BASE, 11)
    from mmr_amd.towers import BertTower
    tw = BertTower(bsd, BERT_BASE, device=DEV)
    assert tw.ln_fold
    ids, mask = (torch.from_numpy(a) for a in synthetic.reports(4, 128, 12))
    fold = tw.forward(ids.to(DEV), mask.to(DEV))
    tw.ln_fold = False
    unf = tw.forward(ids.to(DEV), mask.to(DEV))
    with torch.no_grad():
        ref = otw.bert_forward(ids, mask, bsd, BERT_BASE["num_hidden_layers"], BERT_BASE["num_attention_heads"])
    for got in (fold, unf):
        cos = F.cosine_similarity(got.float().cpu().reshape(-1, 768), ref.float().reshape(-1, 768), dim=-1)
        assert cos.min().item() >= 0.999
        assert rel_err(got, ref) <= 4e-2
    assert rel_err(fold, ref) <= 1.5 * rel_err(unf, ref) + 1e-3, (rel_err(fold, ref), rel_err(unf, ref))
