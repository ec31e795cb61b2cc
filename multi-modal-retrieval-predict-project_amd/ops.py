"""Thin torch-facing wrappers over the libmmr tower ops (include/mmr.h).  Every op launches a
hand-written gfx950 kernel on torch's current stream and raises if the library or the GPU is
missing — there is no torch fallback.  bf16 activations travel as torch.bfloat16 tensors (same
bits as the C ABI's uint16)."""
import contextlib

import torch

from . import _lib


def _L():
    return _lib.lib()


def side_stream(cache, main, device, limit=8):
    """The side stream paired with calling stream `main` (towers / fusion overlap): one per calling
    stream so pipelined callers keep their batches independent, held in a small LRU (`cache`, an
    OrderedDict keyed by the raw stream handle) — a caller creating a stream per request reuses at
    most `limit` side streams instead of leaking one per call; a recycled handle value maps to a side
    stream this object owns, which stays valid."""
    key = main.cuda_stream
    side = cache.get(key)
    if side is None:
        if len(cache) >= limit:
            cache.popitem(last=False)
        side = cache[key] = torch.cuda.Stream(device)
    else:
        cache.move_to_end(key)
    return side


def _s(t):
    return _lib.stream_ptr(t.device)


def _chk(status, what):
    _lib.check(status, what)


PIN_GEMM_BF16, PIN_X3_WAVES, PIN_X3_MLP = 0, 1, 2  # mmr.h MMR_PIN_*


@contextlib.contextmanager
def pinned(which, value):
    """Pin a launch variant for the duration (mmr_pin_variant: tests and A/B tools only; the product
    path never pins).  PIN_GEMM_BF16: mmr_linear_bf16 variant index; PIN_X3_WAVES: 4 / 8; PIN_X3_MLP: 0 / 1
    (8-wave / 4-wave workgroups of the x3 Swin MLP at C = 96)."""
    _chk(_L().mmr_pin_variant(which, value), "mmr_pin_variant")
    try:
        yield
    finally:
        _chk(_L().mmr_pin_variant(which, -1), "mmr_pin_variant")


def linear(x, w, bias=None, residual=None, act=0, out=None):
    """act(x @ w.T + bias) (+ residual); x (..., K) bf16, w (N, K) bf16, bias f32."""
    _lib.require_gpu(x)
    K = x.shape[-1]
    N = w.shape[0]
    M = x.numel() // K
    y = out if out is not None else torch.empty(x.shape[:-1] + (N,), dtype=torch.bfloat16, device=x.device)
    _chk(_L().mmr_linear_bf16(_lib.ptr(x), _lib.ptr(w), _lib.ptr(bias), _lib.ptr(residual), _lib.ptr(y),
                              M, N, K, act, _s(x)), "mmr_linear_bf16")
    return y


class RWPack:
    """A weight image for mmr_linear_rw (resident-weight streaming linear): W (N, K) bf16 re-laid for
    LDS; `None` from rw_pack when the shape is not one the kernel takes."""
    __slots__ = ("img", "n", "k")

    def __init__(self, img, n, k):
        self.img, self.n, self.k = img, n, k


def linear_ln_parts(rows, n, ln_mode=0):
    """Row-statistics pairs per row that mmr_linear_bf16_ln writes for an (rows x n) output (0: shape not
    built)."""
    return int(_L().mmr_linear_bf16_ln_parts(rows, n, ln_mode))


def ln_row_coef(stats, n, eps):
    """Row statistics [rows, parts, 2] of a linear_ln producer -> LayerNorm coefficients [rows, 2]
    (rstd, -mean rstd) over a row width n (mmr_ln_row_coef)."""
    rows, parts = stats.shape[0], stats.shape[1]
    coef = torch.empty((rows, 2), dtype=torch.float32, device=stats.device)
    _chk(_L().mmr_ln_row_coef(_lib.ptr(stats), rows, parts, n, float(eps), _lib.ptr(coef), _s(stats)),
         "mmr_ln_row_coef")
    return coef


def linear_ln(x, w, bias, residual=None, act=0, ln_mode=0, coef=None, v1=None, v2=None, want_stats=False):
    """mmr_linear_bf16_ln: the BERT linears with the residual LayerNorm folded in (no LayerNorm pass).
    coef = ln_row_coef of the producer of x (ln_mode 1: x raw, w = W diag(gamma), v1 = row sums of w,
    bias = W beta + b) or of the residual (ln_mode 2: residual raw, v1 / v2 = gamma / beta).
    Returns (y, stats) — stats [rows, parts, 2] f32 when want_stats, else None: per part of N / parts
    columns, (sum, M2 = centred sum of squares) of the bf16 outputs, merged by ln_row_coef (Chan)."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = w.shape[0]
    assert x2.is_contiguous() and w.is_contiguous() and w.shape[1] == K
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    r = residual.reshape(M, N) if residual is not None else None
    st = None
    if want_stats:
        np_ = linear_ln_parts(M, N, ln_mode)
        if np_ == 0:
            raise _lib.MMRError(f"mmr_linear_bf16_ln: no row statistics for {M} x {N}")
        st = torch.empty((M, np_, 2), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_linear_bf16_ln(_lib.ptr(x2), _lib.ptr(w), _lib.ptr(bias), _lib.ptr(r), _lib.ptr(y), M, N, K, act,
                                 ln_mode, _lib.ptr(coef), _lib.ptr(v1), _lib.ptr(v2), _lib.ptr(st), _s(x)),
         "mmr_linear_bf16_ln")
    return y.view(*lead, N), st


def rw_pack(w):
    """bf16 W (N, K) -> RWPack, or None (K not in {64, 192, 384} or W too large for LDS parts)."""
    _lib.require_gpu(w)
    n, k = w.shape
    if _L().mmr_linear_rw_parts(n, k) <= 0:
        return None
    img = torch.empty((n, k), dtype=torch.bfloat16, device=w.device)
    _chk(_L().mmr_linear_rw_pack(_lib.ptr(w.contiguous()), n, k, _lib.ptr(img), _s(w)), "mmr_linear_rw_pack")
    return RWPack(img, n, k)


def linear_rw(x, pack, bias=None, residual=None, out=None):
    """x @ W^T + bias (+ residual) on the resident-weight streaming kernel; x (..., K) bf16."""
    _lib.require_gpu(x)
    K = x.shape[-1]
    assert K == pack.k
    M = x.numel() // K
    y = out if out is not None else torch.empty(x.shape[:-1] + (pack.n,), dtype=torch.bfloat16, device=x.device)
    _chk(_L().mmr_linear_rw(_lib.ptr(x), _lib.ptr(pack.img), _lib.ptr(bias), _lib.ptr(residual), _lib.ptr(y), M,
                            pack.n, K, _s(x)), "mmr_linear_rw")
    return y


class MXFP8:
    """An MX-fp8 operand: e4m3 bytes q [rows][kp] + E8M0 scales in the GEMM's image order (see
    mmr_quantize_mxfp8), k the unpadded inner size, layout 0 (activations) / 1 (weights)."""
    __slots__ = ("q", "s", "k", "layout")

    def __init__(self, q, s, k, layout):
        self.q, self.s, self.k, self.layout = q, s, k, layout

    @property
    def kp(self):
        return self.q.shape[1]


def quantize_mxfp8(x, layout=0, kp=None):
    """bf16 (..., k) -> MXFP8 (rows = prod of leading dims; rows % 256 == 0 for layouts 0 / 2, % 192 for
    layout 1).  Weights: layout 2 (256-row panels, 256 x 256 GEMM tiles) when N % 256 == 0, else 1."""
    _lib.require_gpu(x)
    k = x.shape[-1]
    rows = x.numel() // k
    kp = kp or -(-k // 256) * 256
    q = torch.empty((rows, kp), dtype=torch.uint8, device=x.device)
    pr = 192 if layout == 1 else 256
    nsc = (rows // pr) * (kp // 128) * 1024 if rows % pr == 0 else 0
    s = torch.zeros((max(nsc, 1),), dtype=torch.uint8, device=x.device)
    _chk(_L().mmr_quantize_mxfp8(_lib.ptr(x), rows, k, kp, layout, _lib.ptr(q), _lib.ptr(s), _s(x)),
         "mmr_quantize_mxfp8")
    return MXFP8(q, s, k, layout)


def linear_mxfp8(x8, w8, bias=None, residual=None, act=0, out=None, lead=None):
    """act(deq(x8) @ deq(w8).T + bias) (+ residual) -> bf16 (rows, N) (or lead + (N,))."""
    _lib.require_gpu(x8.q)
    assert x8.layout == 0 and w8.layout in (1, 2) and x8.kp == w8.kp, "operand layouts / padded K disagree"
    M, N = x8.q.shape[0], w8.q.shape[0]
    shape = (lead if lead is not None else (M,)) + (N,)
    y = out if out is not None else torch.empty(shape, dtype=torch.bfloat16, device=x8.q.device)
    _chk(_L().mmr_linear_mxfp8(_lib.ptr(x8.q), _lib.ptr(x8.s), _lib.ptr(w8.q), _lib.ptr(w8.s), w8.layout, _lib.ptr(bias),
                               _lib.ptr(residual), _lib.ptr(y), M, N, x8.kp, act, _s(x8.q)), "mmr_linear_mxfp8")
    return y


def linear_mxfp8_q8(x8, w8, bias=None, act=0):
    """act(deq(x8) @ deq(w8).T + bias) emitted as the next GEMM's MX-fp8 activation operand (== a
    quantize_mxfp8 of the bf16 result, fused into the epilogue); w8 in layout 2, N % 256 == 0."""
    _lib.require_gpu(x8.q)
    assert x8.layout == 0 and w8.layout == 2 and x8.kp == w8.kp, "operand layouts / padded K disagree"
    M, N = x8.q.shape[0], w8.q.shape[0]
    q = torch.empty((M, N), dtype=torch.uint8, device=x8.q.device)
    s = torch.empty(((M // 256) * (N // 128) * 1024,), dtype=torch.uint8, device=x8.q.device)
    _chk(_L().mmr_linear_mxfp8_q8(_lib.ptr(x8.q), _lib.ptr(x8.s), _lib.ptr(w8.q), _lib.ptr(w8.s), _lib.ptr(bias),
                                  _lib.ptr(q), _lib.ptr(s), M, N, x8.kp, act, _s(x8.q)), "mmr_linear_mxfp8_q8")
    return MXFP8(q, s, N, 0)


def layernorm(x, g, b, eps, out=None):
    _lib.require_gpu(x)
    c = x.shape[-1]
    y = out if out is not None else torch.empty_like(x)
    _chk(_L().mmr_layernorm_bf16(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), x.numel() // c, c,
                                 float(eps), _s(x)), "mmr_layernorm_bf16")
    return y


def add_layernorm(x, r, g, b, eps, out=None):
    """LayerNorm(x + r) (post-LN residual block), sum in f32."""
    _lib.require_gpu(x)
    c = x.shape[-1]
    assert r.shape == x.shape
    y = out if out is not None else torch.empty_like(x)
    _chk(_L().mmr_add_layernorm_bf16(_lib.ptr(x), _lib.ptr(r), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y),
                                     x.numel() // c, c, float(eps), _s(x)), "mmr_add_layernorm_bf16")
    return y


def layernorm_q8(x, r, g, b, eps, kp=None, want_y=True):
    """LayerNorm(x (+ r)) -> (y bf16, its MX-fp8 activation operand) in one pass (rows % 256 == 0,
    C % 32 == 0); r may be None.  kp: the operand's padded K (a multiple of 256 >= C; default C, which
    must then be a multiple of 256) — the padding is written as quantize_mxfp8 writes it.  want_y=False
    skips the bf16 output (y is None) when only the operand is consumed."""
    _lib.require_gpu(x)
    c = x.shape[-1]
    rows = x.numel() // c
    kp = kp or c
    y = torch.empty_like(x) if want_y else None
    q = torch.empty((rows, kp), dtype=torch.uint8, device=x.device)
    s = torch.empty(((rows // 256) * (kp // 128) * 1024,), dtype=torch.uint8, device=x.device)
    if kp == c and want_y:
        _chk(_L().mmr_layernorm_bf16_q8(_lib.ptr(x), _lib.ptr(r), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), _lib.ptr(q),
                                        _lib.ptr(s), rows, c, float(eps), _s(x)), "mmr_layernorm_bf16_q8")
    else:
        _chk(_L().mmr_layernorm_bf16_q8p(_lib.ptr(x), _lib.ptr(r), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), _lib.ptr(q),
                                         _lib.ptr(s), rows, c, kp, float(eps), _s(x)), "mmr_layernorm_bf16_q8p")
    return y, MXFP8(q, s, c, 0)


def _q8_out(rows, c, dev):
    return (torch.empty((rows, c), dtype=torch.uint8, device=dev),
            torch.empty(((rows // 256) * (c // 128) * 1024,), dtype=torch.uint8, device=dev))


def scaled_add_layernorm(x, alpha, r, g, b, eps, out=None, q8=False):
    """LayerNorm(alpha * x + r), alpha a device scalar tensor (vectorised row kernel, bf16).  q8: also
    the result's MX-fp8 activation operand, returned as (y, MXFP8) (rows % 256 == 0, C % 256 == 0)."""
    _lib.require_gpu(x)
    c = x.shape[-1]
    if r is not None:
        assert r.shape == x.shape
    y = out if out is not None else torch.empty_like(x)
    rows = x.numel() // c
    if q8:
        q, s = _q8_out(rows, c, x.device)
        _chk(_L().mmr_scaled_add_layernorm_bf16_q8(_lib.ptr(x), _lib.ptr(alpha), _lib.ptr(r), _lib.ptr(g),
                                                   _lib.ptr(b), _lib.ptr(y), _lib.ptr(q), _lib.ptr(s), rows, c,
                                                   float(eps), _s(x)), "mmr_scaled_add_layernorm_bf16_q8")
        return y, MXFP8(q, s, c, 0)
    _chk(_L().mmr_scaled_add_layernorm_bf16(_lib.ptr(x), _lib.ptr(alpha), _lib.ptr(r), _lib.ptr(g), _lib.ptr(b),
                                            _lib.ptr(y), rows, c, float(eps), _s(x)),
         "mmr_scaled_add_layernorm_bf16")
    return y


def bert_embed(ids, word, pos, type0, g, b, eps):
    _lib.require_gpu(ids)
    B, L = ids.shape
    C = word.shape[1]
    y = torch.empty((B, L, C), dtype=torch.bfloat16, device=ids.device)
    _chk(_L().mmr_bert_embed(_lib.ptr(ids), _lib.ptr(word), _lib.ptr(pos), _lib.ptr(type0), _lib.ptr(g),
                             _lib.ptr(b), _lib.ptr(y), B, L, C, float(eps), _s(ids)), "mmr_bert_embed")
    return y


def bert_embed_q8(ids, word, pos, type0, g, b, eps):
    """bert_embed also emitting the first QKV GEMM's MX-fp8 operand: (y, MXFP8) with the operand ==
    quantize_mxfp8(y); B * L % 256 == 0, C % 256 == 0."""
    _lib.require_gpu(ids)
    B, L = ids.shape
    C = word.shape[1]
    y = torch.empty((B, L, C), dtype=torch.bfloat16, device=ids.device)
    q, s = _q8_out(B * L, C, ids.device)
    _chk(_L().mmr_bert_embed_q8(_lib.ptr(ids), _lib.ptr(word), _lib.ptr(pos), _lib.ptr(type0), _lib.ptr(g),
                                _lib.ptr(b), _lib.ptr(y), _lib.ptr(q), _lib.ptr(s), B, L, C, float(eps), _s(ids)),
         "mmr_bert_embed_q8")
    return y, MXFP8(q, s, C, 0)


def bert_attention(qkv, mask, heads, dh=64, q8=False, bf16=True):
    """ctx (B, L, C) bf16; q8: the context as an MX-fp8 activation operand too, returned as
    (ctx or None, MXFP8) — bf16=False skips the bf16 copy ((B*L) % 256 == 0, C % 256 == 0)."""
    B, L, C3 = qkv.shape
    ctx = torch.empty((B, L, C3 // 3), dtype=torch.bfloat16, device=qkv.device) if (bf16 or not q8) else None
    if q8:
        C = C3 // 3
        q, s = _q8_out(B * L, C, qkv.device)
        _chk(_L().mmr_bert_attention_q8(_lib.ptr(qkv), _lib.ptr(mask), _lib.ptr(ctx), _lib.ptr(q), _lib.ptr(s), B, L,
                                        heads, dh, _s(qkv)), "mmr_bert_attention_q8")
        return ctx, MXFP8(q, s, C, 0)
    _chk(_L().mmr_bert_attention(_lib.ptr(qkv), _lib.ptr(mask), _lib.ptr(ctx), B, L, heads, dh, _s(qkv)),
         "mmr_bert_attention")
    return ctx


def swin_attn_bias(table, heads, ws, hw, shift):
    """Dense [types][heads][64][64] f32 bias (rel-pos + shift mask + padded keys) for one block."""
    nt = 4 if shift > 0 else 1
    bias = torch.empty((nt, heads, 64, 64), dtype=torch.float32, device=table.device)
    _chk(_L().mmr_swin_attn_bias(_lib.ptr(table), _lib.ptr(bias), heads, ws, hw, shift, _s(table)),
         "mmr_swin_attn_bias")
    return bias


def swin_window_attention(qkv, bias, hw, heads, ws, shift):
    B = qkv.shape[0]
    C = qkv.shape[-1] // 3
    out = torch.empty(qkv.shape[:-1] + (C,), dtype=torch.bfloat16, device=qkv.device)
    _chk(_L().mmr_swin_window_attention(_lib.ptr(qkv), _lib.ptr(bias), _lib.ptr(out), B, hw, C, heads, ws,
                                        shift, _s(qkv)), "mmr_swin_window_attention")
    return out


def swin_window_attention_q8(qkv, bias, hw, heads, ws, shift, kp=None):
    """swin_window_attention emitting the proj GEMM's MX-fp8 operand (K padded to kp) instead of bf16
    rows: == quantize_mxfp8(swin_window_attention(...), kp=kp), rows % 256 == 0."""
    B = qkv.shape[0]
    C = qkv.shape[-1] // 3
    kp = kp or -(-C // 256) * 256
    rows = qkv.numel() // qkv.shape[-1]
    q = torch.empty((rows, kp), dtype=torch.uint8, device=qkv.device)
    s = torch.empty(((rows // 256) * (kp // 128) * 1024,), dtype=torch.uint8, device=qkv.device)
    _chk(_L().mmr_swin_window_attention_q8(_lib.ptr(qkv), _lib.ptr(bias), _lib.ptr(q), _lib.ptr(s), B, hw, C, kp,
                                           heads, ws, shift, _s(qkv)), "mmr_swin_window_attention_q8")
    return MXFP8(q, s, C, 0)


def patch_im2col(img, patch=4):
    B, Cin, H, W = img.shape
    g = H // patch
    cols = torch.empty((B, g * g, 64), dtype=torch.bfloat16, device=img.device)
    _chk(_L().mmr_patch_im2col(_lib.ptr(img), _lib.ptr(cols), B, Cin, H, patch, _s(img)), "mmr_patch_im2col")
    return cols


def patch_merge_ln(x, g, b, eps):
    B, H, W, C = x.shape
    y = torch.empty((B, H // 2, W // 2, 4 * C), dtype=torch.bfloat16, device=x.device)
    _chk(_L().mmr_patch_merge_ln(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), B, H, C, float(eps),
                                 _s(x)), "mmr_patch_merge_ln")
    return y


def patch_merge_ln_q8(x, g, b, eps, want_y=False):
    """patch_merge_ln emitting the reduction GEMM's MX-fp8 operand: (y or None, MXFP8) with the operand
    == quantize_mxfp8(patch_merge_ln(...)); merged rows % 256 == 0, 4C % 256 == 0."""
    B, H, W, C = x.shape
    rows = B * (H // 2) * (W // 2)
    y = torch.empty((B, H // 2, W // 2, 4 * C), dtype=torch.bfloat16, device=x.device) if want_y else None
    q = torch.empty((rows, 4 * C), dtype=torch.uint8, device=x.device)
    s = torch.empty(((rows // 256) * (4 * C // 128) * 1024,), dtype=torch.uint8, device=x.device)
    _chk(_L().mmr_patch_merge_ln_q8(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), _lib.ptr(q), _lib.ptr(s), B, H,
                                    C, float(eps), _s(x)), "mmr_patch_merge_ln_q8")
    return y, MXFP8(q, s, 4 * C, 0)


def swin_head(x, g, b, eps, want_patches=True):
    """x (B, T, C) bf16 pre-final-norm tokens -> (patches f32 (B,T,C) | None, global f32, pool f32)."""
    B, T, C = x.shape
    dev = x.device
    patches = torch.empty((B, T, C), dtype=torch.float32, device=dev) if want_patches else None
    glob = torch.empty((B, C), dtype=torch.float32, device=dev)
    pool = torch.empty((B, C), dtype=torch.float32, device=dev)
    _chk(_L().mmr_swin_head(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(patches), _lib.ptr(glob),
                            _lib.ptr(pool), B, T, C, float(eps), _s(x)), "mmr_swin_head")
    return patches, glob, pool


def mean_tokens(x):
    B, L, C = x.shape
    y = torch.empty((B, C), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_mean_tokens(_lib.ptr(x), _lib.ptr(y), B, L, C, _s(x)), "mmr_mean_tokens")
    return y


def proj_head(x, wp, bp, w1=None, b1=None, w2=None, b2=None, l2norm=False):
    B, Cin = x.shape
    D = wp.shape[0]
    y = torch.empty((B, D), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_proj_head(_lib.ptr(x), _lib.ptr(wp), _lib.ptr(bp), _lib.ptr(w1), _lib.ptr(b1), _lib.ptr(w2),
                            _lib.ptr(b2), _lib.ptr(y), B, Cin, D, int(bool(l2norm)), _s(x)), "mmr_proj_head")
    return y


def linear_f32(x, w, bias=None, residual=None, act=0, out=None):
    """act(x @ w.T + bias) (+ residual) in exact f32; x (B, cin) f32 rows (may be a strided view with
    unit column stride), residual may be `out` (in-place accumulate)."""
    _lib.require_gpu(x)
    assert x.dim() == 2 and x.stride(1) == 1
    B, cin = x.shape
    cout = w.shape[0]
    y = out if out is not None else torch.empty((B, cout), dtype=torch.float32, device=x.device)
    ldr = residual.stride(0) if residual is not None else 0
    _chk(_L().mmr_linear_f32(_lib.ptr(x), x.stride(0), _lib.ptr(w), _lib.ptr(bias), _lib.ptr(residual), ldr,
                             _lib.ptr(y), y.stride(0), B, cin, cout, act, _s(x)), "mmr_linear_f32")
    return y


class X3W:
    """A per-query linear weight for linear_x3: the f32 weight (kept for the exact-f32 fallback) and its
    bf16 split hi = bf16(w), lo = bf16(w - hi); (..., cout, cin).  `w2()`: the split GEMM's weight image
    [hi | lo] (each segment kp = mmr_x3_p8_kpad(cin) wide, zero-padded) of a 2-D weight, built on first use
    (x3_linear)."""
    __slots__ = ("w", "hi", "lo", "_w2", "_bpad")

    def __init__(self, w):
        self.w = w.contiguous()
        self.hi = self.w.to(torch.bfloat16)
        self.lo = (self.w - self.hi.float()).to(torch.bfloat16)
        self._w2 = None
        self._bpad = None

    def w2(self, kp, npad):
        """[npad][2 kp] bf16: rows n.. npad - 1 and each segment's columns k.. kp - 1 zero."""
        if self._w2 is None:
            n, k = self.w.shape
            img = torch.zeros((npad, 2 * kp), dtype=torch.bfloat16, device=self.w.device)
            img[:n, :k] = self.hi
            img[:n, kp:kp + k] = self.lo
            self._w2 = img
        return self._w2

    def bias_padded(self, bias, npad):
        """bias zero-padded to npad entries (cached for the last bias seen)."""
        if bias is None or bias.shape[0] == npad:
            return bias
        if self._bpad is None or self._bpad[0] is not bias:
            bp = torch.zeros(npad, dtype=torch.float32, device=bias.device)
            bp[:bias.shape[0]] = bias
            self._bpad = (bias, bp)
        return self._bpad[1]


def _x3_ok(cin, cout):
    return cin % 128 == 0 and cout % 32 == 0


def linear_x3(x, wx, bias=None, residual=None, act=0, out=None):
    """act(x @ w.T + bias) (+ residual) on bf16x3 MFMA (mmr_linear_x3; ~2^-17 relative per product);
    x (B, cin) f32 rows (unit column stride), residual may be `out`.  Shapes the kernel does not take
    (cin % 128, cout % 32) run linear_f32."""
    cout, cin = wx.w.shape
    if not _x3_ok(cin, cout):
        return linear_f32(x, wx.w, bias, residual=residual, act=act, out=out)
    _lib.require_gpu(x)
    assert x.dim() == 2 and x.stride(1) == 1
    B = x.shape[0]
    y = out if out is not None else torch.empty((B, cout), dtype=torch.float32, device=x.device)
    ldr = residual.stride(0) if residual is not None else 0
    _chk(_L().mmr_linear_x3(_lib.ptr(x), x.stride(0), 0, _lib.ptr(wx.hi), _lib.ptr(wx.lo), 0, _lib.ptr(bias), 0,
                            _lib.ptr(residual), ldr, 0, _lib.ptr(y), y.stride(0), 0, 1, B, cin, cout, act, _s(x)),
         "mmr_linear_x3")
    return y


def linear_x3_batched(x, wx, bias, nbatch, b, residual=None, act=0, out=None, ldx=None, bsx=None, ldy=None,
                      bsy=None, ldr=None, bsr=None):
    """linear_f32_batched on bf16x3 MFMA: wx.w (nbatch, cout, cin); same stride conventions."""
    cout, cin = wx.w.shape[1], wx.w.shape[2]
    if not _x3_ok(cin, cout):
        return linear_f32_batched(x, wx.w, bias, nbatch, b, residual=residual, act=act, out=out, ldx=ldx, bsx=bsx,
                                  ldy=ldy, bsy=bsy, ldr=ldr, bsr=bsr)
    _lib.require_gpu(x)
    ldx = cin if ldx is None else ldx
    bsx = b * ldx if bsx is None else bsx
    y = out if out is not None else torch.empty((nbatch, b, cout), dtype=torch.float32, device=x.device)
    ldy = cout if ldy is None else ldy
    bsy = b * ldy if bsy is None else bsy
    if residual is not None:
        ldr = cout if ldr is None else ldr
        bsr = b * ldr if bsr is None else bsr
    _chk(_L().mmr_linear_x3(_lib.ptr(x), ldx, bsx, _lib.ptr(wx.hi), _lib.ptr(wx.lo), cout * cin, _lib.ptr(bias),
                            cout if bias is not None else 0, _lib.ptr(residual), ldr or 0, bsr or 0, _lib.ptr(y), ldy,
                            bsy, nbatch, b, cin, cout, act, _s(x)), "mmr_linear_x3")
    return y


def mha(q, k, v, b, lq, lk, heads, dh, scale, out=None, mean_out=None, q8=False):
    """Attention core over strided row views: q (b*lq, >=heads*dh) etc. (unit column stride).  q8: the
    output also as an MX-fp8 activation operand, returned as (out, mean_out, MXFP8)."""
    _lib.require_gpu(q)
    if q8:
        c = heads * dh
        q8t, s8 = _q8_out(b * lq, c, q.device)
        _chk(_L().mmr_mha_q8(_lib.ptr(q), q.stride(0), _lib.ptr(k), k.stride(0), _lib.ptr(v), v.stride(0),
                             _lib.ptr(out), out.stride(0) if out is not None else 0, _lib.ptr(mean_out),
                             _lib.ptr(q8t), _lib.ptr(s8), b, lq, lk, heads, dh, float(scale), _s(q)), "mmr_mha_q8")
        return out, mean_out, MXFP8(q8t, s8, c, 0)
    _chk(_L().mmr_mha(_lib.ptr(q), q.stride(0), _lib.ptr(k), k.stride(0), _lib.ptr(v), v.stride(0),
                      _lib.ptr(out), out.stride(0) if out is not None else 0, _lib.ptr(mean_out), b, lq, lk,
                      heads, dh, float(scale), _s(q)), "mmr_mha")
    return out, mean_out


def add_pos(x, pos, l, q8=False):
    """bf16 (rows, c) = x + pos[row % l] for x (..., c) f32 or bf16 contiguous, pos f32 [>= l][c].
    q8: also its MX-fp8 activation operand, returned as (y, MXFP8) (rows % 256 == 0, C % 256 == 0)."""
    _lib.require_gpu(x)
    c = x.shape[-1]
    rows = x.numel() // c
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    if q8:
        q, s = _q8_out(rows, c, x.device)
        _chk(_L().mmr_add_pos_bf16_q8(_lib.ptr(x), int(x.dtype == torch.float32), _lib.ptr(pos), _lib.ptr(y),
                                      _lib.ptr(q), _lib.ptr(s), rows, l, c, _s(x)), "mmr_add_pos_bf16_q8")
        return y, MXFP8(q, s, c, 0)
    _chk(_L().mmr_add_pos_bf16(_lib.ptr(x), int(x.dtype == torch.float32), _lib.ptr(pos), _lib.ptr(y),
                               rows, l, c, _s(x)), "mmr_add_pos_bf16")
    return y


def ln_rows(x, g, b, eps, alpha=None, residual=None, post=None, post_scale=None, out=None, groups=1, group_div=1):
    """LN(alpha*x + residual) * g + b (+ post_scale*post) over 2-D row views (f32 or bf16 in/out);
    with groups > 1, row r uses parameter set (r // group_div) % groups of g/b [groups][c] and
    alpha/post_scale [groups]."""
    _lib.require_gpu(x)
    assert x.dim() == 2 and x.stride(1) == 1
    rows, c = x.shape
    y = out if out is not None else torch.empty((rows, c), dtype=x.dtype, device=x.device)
    _chk(_L().mmr_ln_rows(_lib.ptr(x), x.stride(0), _lib.ptr(alpha), _lib.ptr(residual),
                          residual.stride(0) if residual is not None else 0, _lib.ptr(g), _lib.ptr(b),
                          _lib.ptr(post), post.stride(0) if post is not None else 0, _lib.ptr(post_scale),
                          _lib.ptr(y), y.stride(0), rows, c, float(eps), int(x.dtype == torch.bfloat16), groups,
                          group_div, _s(x)), "mmr_ln_rows")
    return y


def linear_f32_batched(x, w, bias, nbatch, b, residual=None, act=0, out=None, ldx=None, bsx=None, ldy=None,
                       bsy=None, ldr=None, bsr=None):
    """nbatch independent f32 linears: problem i reads rows of x at x + i*bsx (row stride ldx), weights
    w[i] (w (nbatch, cout, cin)), bias[i], residual + i*bsr and writes out + i*bsy (row stride ldy).
    Defaults: contiguous (nbatch, b, cin) -> (nbatch, b, cout)."""
    _lib.require_gpu(x)
    cout, cin = w.shape[1], w.shape[2]
    ldx = cin if ldx is None else ldx
    bsx = b * ldx if bsx is None else bsx
    y = out if out is not None else torch.empty((nbatch, b, cout), dtype=torch.float32, device=x.device)
    ldy = cout if ldy is None else ldy
    bsy = b * ldy if bsy is None else bsy
    if residual is not None:
        ldr = cout if ldr is None else ldr
        bsr = b * ldr if bsr is None else bsr
    _chk(_L().mmr_linear_f32_batched(_lib.ptr(x), ldx, bsx, _lib.ptr(w), cout * cin, _lib.ptr(bias),
                                     cout if bias is not None else 0, _lib.ptr(residual), ldr or 0, bsr or 0,
                                     _lib.ptr(y), ldy, bsy, nbatch, b, cin, cout, act, _s(x)),
         "mmr_linear_f32_batched")
    return y


def assemble_seq(x1, pf, x2, pe, np_, q8=False):
    """bf16 (B, np_+2, c) = [x1; pf; x2] + pe; q8: only its MX-fp8 operand (MXFP8 of B*(np_+2) rows)."""
    B, c = x1.shape
    if q8:
        q, s = _q8_out(B * (np_ + 2), c, x1.device)
        _chk(_L().mmr_assemble_seq_q8(_lib.ptr(x1), _lib.ptr(pf), _lib.ptr(x2), _lib.ptr(pe), _lib.ptr(q), _lib.ptr(s),
                                      B, np_, c, _s(x1)), "mmr_assemble_seq_q8")
        return MXFP8(q, s, c, 0)
    seq = torch.empty((B, np_ + 2, c), dtype=torch.bfloat16, device=x1.device)
    _chk(_L().mmr_assemble_seq(_lib.ptr(x1), _lib.ptr(pf), _lib.ptr(x2), _lib.ptr(pe), _lib.ptr(seq), B, np_, c,
                               _s(x1)), "mmr_assemble_seq")
    return seq


def rows_to_f32(x, b, c, ldx, out=None):
    y = out if out is not None else torch.empty((b, c), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_rows_to_f32(_lib.ptr(x), ldx, _lib.ptr(y), b, c, _s(x)), "mmr_rows_to_f32")
    return y


def swin_mlp_pack(w1, w2):
    """fc1.weight [4C][C], fc2.weight [C][4C] (bf16, device) -> packed chunks for swin_mlp, or None if
    C is not one of the fused widths."""
    C = w1.shape[1]
    n = _L().mmr_swin_mlp_pack_elems(C)
    if n <= 0:
        return None
    pack = torch.empty((n,), dtype=torch.bfloat16, device=w1.device)
    _chk(_L().mmr_swin_mlp_pack(_lib.ptr(w1.contiguous()), _lib.ptr(w2.contiguous()), _lib.ptr(pack), C, _s(w1)),
         "mmr_swin_mlp_pack")
    return pack


def swin_mlp(x, g, b, pack, b1, b2, eps):
    """x + fc2(GELU(fc1(LN(x)))) fused (C in {96, 192})."""
    C = x.shape[-1]
    y = torch.empty_like(x)
    _chk(_L().mmr_swin_mlp(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(pack), _lib.ptr(b1), _lib.ptr(b2),
                           _lib.ptr(y), x.numel() // C, C, float(eps), _s(x)), "mmr_swin_mlp")
    return y


def swin_attn_block_pack(qkv_w, qkv_b, proj_w, proj_b, ln_g, ln_b):
    """Weights of one Swin block's attention half -> packed LDS image for swin_attn_block, or None
    if C is not a fused width."""
    C = qkv_w.shape[1]
    n = _L().mmr_swin_attn_block_pack_bytes(C)
    if n <= 0:
        return None
    pack = torch.empty((n,), dtype=torch.uint8, device=qkv_w.device)
    _chk(_L().mmr_swin_attn_block_pack(_lib.ptr(qkv_w), _lib.ptr(qkv_b), _lib.ptr(proj_w), _lib.ptr(proj_b),
                                       _lib.ptr(ln_g), _lib.ptr(ln_b), _lib.ptr(pack), C, _s(qkv_w)),
         "mmr_swin_attn_block_pack")
    return pack


def swin_attn_block(x, pack, bias, ws, shift, eps):
    """x + proj(W-MSA(LN1(x))) for x (B, H, H, C), fused (C = 96)."""
    B, H, _, C = x.shape
    y = torch.empty_like(x)
    _chk(_L().mmr_swin_attn_block(_lib.ptr(x), _lib.ptr(pack), _lib.ptr(bias), _lib.ptr(y), B, H, C, ws, shift,
                                  float(eps), _s(x)), "mmr_swin_attn_block")
    return y


# ---------------------------------------------------------------- fp32-faithful tower mode ("x3")
# f32 activations, every contraction on bf16x3 MFMA (csrc/x3.hip); weights as X3W (hi / lo splits).
class X3Rows:
    """An x3 GEMM operand already split: t = [hi | lo] bf16 rows (rows, 2 kp), kp = mmr_x3_p8_kpad(k),
    standing for f32 rows of width k with leading shape `lead` (mmr_ln_rows_split's output)."""
    __slots__ = ("t", "k", "kp", "lead")

    def __init__(self, t, k, kp, lead):
        self.t, self.k, self.kp, self.lead = t, k, kp, lead

    @property
    def rows(self):
        return self.t.shape[0]


def x3_ln_split(x, g, b, eps, residual=None, keep_f32=False, alpha=None):
    """LayerNorm(alpha * x + residual) over the last dim of f32 rows for an x3 linear (alpha: a device f32
    scalar or None): rows filling 256-row tiles come back as X3Rows (mmr_ln_rows_split: the next GEMM
    skips its split pass), with the f32 output too when keep_f32 (-> (y, X3Rows)); other row counts as
    plain f32 rows (ln_rows)."""
    _lib.require_gpu(x)
    c = x.shape[-1]
    x2 = x.reshape(-1, c)
    r2 = residual.reshape(-1, c) if residual is not None else None
    M = x2.shape[0]
    kp = _L().mmr_x3_p8_kpad(c)
    if not (M > 0 and M % 256 == 0 and kp > 0 and c % 4 == 0 and c <= 1024 and x2.stride(1) == 1
            and (r2 is None or r2.stride(1) == 1)):
        y = ln_rows(x2, g, b, eps, alpha=alpha, residual=r2).view(x.shape)
        return (y, y) if keep_f32 else y
    xs = torch.empty((M, 2 * kp), dtype=torch.bfloat16, device=x.device)
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device) if keep_f32 else None
    _chk(_L().mmr_ln_rows_split(_lib.ptr(x2), x2.stride(0), _lib.ptr(alpha), _lib.ptr(r2),
                                r2.stride(0) if r2 is not None else 0,
                                _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), c, _lib.ptr(xs), M, c, float(eps), _s(x)),
         "mmr_ln_rows_split")
    xr = X3Rows(xs, c, kp, tuple(x.shape[:-1]))
    return (y, xr) if keep_f32 else xr


def _x3_linear_split_in(xr, wx, bias, residual, act, out):
    """x3_linear of an X3Rows operand (mmr_x3_linear_p8 on the rows as they are)."""
    N, Kw = wx.w.shape
    assert xr.k == Kw, f"x3_linear: K {xr.k} != weight K {Kw}"
    M = xr.rows
    npad = _L().mmr_x3_p8_npad(N)
    if npad <= 0:
        # N not a split-GEMM width (N % 4 != 0 or > 16384): the f32 rows back — hi + lo is exact in f32;
        # its re-split can differ from (hi, lo) where lo rounded to half an ulp of hi (same value)
        x = (xr.t[:, :xr.k].float() + xr.t[:, xr.kp:xr.kp + xr.k].float()).view(xr.lead + (xr.k,))
        return x3_linear(x, wx, bias, residual=residual, act=act, out=out)
    if out is not None and not out.is_contiguous():
        out.copy_(_x3_linear_split_in(xr, wx, bias, residual, act, None))
        return out
    if residual is not None and not residual.is_contiguous():
        residual = residual.contiguous()
    r2 = residual.reshape(-1, N) if residual is not None else None
    y = out if out is not None else torch.empty(xr.lead + (N,), dtype=torch.float32, device=xr.t.device)
    _chk(_L().mmr_x3_linear_p8(_lib.ptr(xr.t), _lib.ptr(wx.w2(xr.kp, npad)), _lib.ptr(wx.bias_padded(bias, npad)),
                               _lib.ptr(r2), _lib.ptr(y), M, N, xr.k, act, 0, _s(xr.t)), "mmr_x3_linear_p8")
    return y


def x3_linear(x, wx, bias=None, residual=None, act=0, out=None):
    """act(x @ w.T + bias) (+ residual) for any number of rows: x (..., K) f32 (last-dim contiguous rows),
    wx an X3W of w (N, K), K % 32 == 0; residual may be `out`.  Row counts that fill 256-row tiles with
    N >= 192 run as one three-product split GEMM on the 8-phase kernel (mmr_x3_split_rows +
    mmr_x3_linear_p8, N padded to whole tiles); the rest on mmr_x3_linear (128 x 128 tiles).  x may be
    an X3Rows (x3_ln_split), read as is."""
    if isinstance(x, X3Rows):
        return _x3_linear_split_in(x, wx, bias, residual, act, out)
    _lib.require_gpu(x)
    K = x.shape[-1]
    N, Kw = wx.w.shape
    assert K == Kw, f"x3_linear: K {K} != weight K {Kw}"
    x2 = x.reshape(-1, K)
    assert x2.stride(1) == 1
    M = x2.shape[0]
    y = out if out is not None else torch.empty(x.shape[:-1] + (N,), dtype=torch.float32, device=x.device)
    r2 = residual.reshape(-1, N) if residual is not None else None
    kp, npad = _L().mmr_x3_p8_kpad(K), _L().mmr_x3_p8_npad(N)
    # (N < 192: the split pass costs more than the GEMM saves — Swin stage-1 fc2, N = 96 K = 384: 0.96 ->
    # 1.11 ms per call with the earlier 6-byte split)
    if (M > 0 and M % 256 == 0 and N >= 192 and kp > 0 and npad > 0 and y.is_contiguous()
            and (r2 is None or r2.is_contiguous())):
        xs = torch.empty((M, 2 * kp), dtype=torch.bfloat16, device=x.device)
        _chk(_L().mmr_x3_split_rows(_lib.ptr(x2), x2.stride(0), M, K, _lib.ptr(xs), _s(x)), "mmr_x3_split_rows")
        _chk(_L().mmr_x3_linear_p8(_lib.ptr(xs), _lib.ptr(wx.w2(kp, npad)), _lib.ptr(wx.bias_padded(bias, npad)),
                                   _lib.ptr(r2), _lib.ptr(y), M, N, K, act, 0, _s(x)), "mmr_x3_linear_p8")
        return y
    _chk(_L().mmr_x3_linear(_lib.ptr(x2), x2.stride(0), _lib.ptr(wx.hi), _lib.ptr(wx.lo), _lib.ptr(bias), _lib.ptr(r2),
                            r2.stride(0) if r2 is not None else 0, _lib.ptr(y), N, M, N, K, act, _s(x)),
         "mmr_x3_linear")
    return y


def x3_linear_split_out(xr, wx, bias, act=0):
    """x3_linear of an X3Rows operand with its output written as the NEXT x3 GEMM's operand: X3Rows of
    [hi | lo] bf16 rows 2 N wide (mmr_x3_linear_p8 out_hilo; the split of the f32 output, bit for bit).
    N % 384 == 0, rows % 256 == 0, no residual."""
    N, K = wx.w.shape
    assert isinstance(xr, X3Rows) and xr.k == K and N % 384 == 0 and xr.rows % 256 == 0
    hl = torch.empty((xr.rows, 2 * N), dtype=torch.bfloat16, device=xr.t.device)
    _chk(_L().mmr_x3_linear_p8(_lib.ptr(xr.t), _lib.ptr(wx.w2(xr.kp, N)), _lib.ptr(wx.bias_padded(bias, N)), None,
                               _lib.ptr(hl), xr.rows, N, K, act, 1, _s(xr.t)), "mmr_x3_linear_p8")
    return X3Rows(hl, N, N, xr.lead)


def x3_ffn(x, w1, b1, w2, b2, residual=None):
    """fc2(GELU(fc1(x))) (+ residual), f32 in and out (the BERT / Swin MLP in the x3 mode).  When both
    rows fill 256-row tiles and fc1's width is a multiple of 384, fc1 writes its output straight as
    fc2's [hi | lo] bf16 operand rows (mmr_x3_linear_p8 out_hilo): the f32 round trip and the
    split pass drop out; bit-identical to the two x3_linear calls where those take the 8-phase route
    (fc2 N >= 192), within the split's rounding of them otherwise.  x may be an X3Rows."""
    L = _L()
    N1, N2 = w1.w.shape[0], w2.w.shape[0]
    kp2, np1, np2 = L.mmr_x3_p8_kpad(N1), L.mmr_x3_p8_npad(N1), L.mmr_x3_p8_npad(N2)
    r2 = residual.reshape(-1, N2) if residual is not None else None
    if isinstance(x, X3Rows):
        M = x.rows
        if not (N1 % 384 == 0 and kp2 == N1 and np1 == N1 and np2 > 0 and b1 is not None and b2 is not None
                and (r2 is None or r2.is_contiguous())):
            return x3_linear(x3_linear(x, w1, b1, act=1), w2, b2, residual=residual)
        hl = x3_linear_split_out(x, w1, b1, act=1).t
        y = torch.empty(x.lead + (N2,), dtype=torch.float32, device=x.t.device)
        _chk(L.mmr_x3_linear_p8(_lib.ptr(hl), _lib.ptr(w2.w2(kp2, np2)), _lib.ptr(w2.bias_padded(b2, np2)),
                                _lib.ptr(r2), _lib.ptr(y), M, N2, N1, 0, 0, _s(x.t)), "mmr_x3_linear_p8")
        return y
    _lib.require_gpu(x)
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    kp1 = L.mmr_x3_p8_kpad(K)
    # (fc2 with N2 < 192 — Swin stage 1, N2 = 96 — included: its weight rows pad to one 192 tile, which
    # the MFMA has room for, while the unfused route's split pass is what made it slower there)
    if not (M > 0 and M % 256 == 0 and N1 % 384 == 0 and kp1 > 0 and kp2 == N1 and np1 == N1
            and np2 > 0 and b1 is not None and b2 is not None and x2.stride(1) == 1
            and (r2 is None or r2.is_contiguous())):
        return x3_linear(x3_linear(x, w1, b1, act=1), w2, b2, residual=residual)
    xs = torch.empty((M, 2 * kp1), dtype=torch.bfloat16, device=x.device)
    _chk(L.mmr_x3_split_rows(_lib.ptr(x2), x2.stride(0), M, K, _lib.ptr(xs), _s(x)), "mmr_x3_split_rows")
    hl = torch.empty((M, 2 * N1), dtype=torch.bfloat16, device=x.device)  # [h_hi | h_lo] rows
    _chk(L.mmr_x3_linear_p8(_lib.ptr(xs), _lib.ptr(w1.w2(kp1, N1)), _lib.ptr(w1.bias_padded(b1, N1)), None,
                            _lib.ptr(hl), M, N1, K, 1, 1, _s(x)), "mmr_x3_linear_p8")
    y = torch.empty(x.shape[:-1] + (N2,), dtype=torch.float32, device=x.device)
    _chk(L.mmr_x3_linear_p8(_lib.ptr(hl), _lib.ptr(w2.w2(kp2, np2)), _lib.ptr(w2.bias_padded(b2, np2)),
                            _lib.ptr(r2), _lib.ptr(y), M, N2, N1, 0, 0, _s(x)), "mmr_x3_linear_p8")
    return y


def x3_swin_mlp_pack(w1, w2):
    """fc1.weight [4C][C], fc2.weight [C][4C] (f32, device) -> the split chunk images of x3_swin_mlp, or None
    if C is not a fused width (96, 192)."""
    C = w1.shape[1]
    n = _L().mmr_x3_swin_mlp_pack_elems(C)
    if n <= 0:
        return None
    pack = torch.empty((n,), dtype=torch.bfloat16, device=w1.device)
    _chk(_L().mmr_x3_swin_mlp_pack(_lib.ptr(w1.contiguous()), _lib.ptr(w2.contiguous()), _lib.ptr(pack), C, _s(w1)),
         "mmr_x3_swin_mlp_pack")
    return pack


def x3_swin_mlp(x, g, b, pack, b1, b2, eps):
    """x + fc2(GELU(fc1(LN(x)))) in the x3 mode, fused (f32 tokens (..., C), C in {96, 192})."""
    _lib.require_gpu(x)
    C = x.shape[-1]
    y = torch.empty_like(x)
    _chk(_L().mmr_x3_swin_mlp(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(pack), _lib.ptr(b1), _lib.ptr(b2),
                              _lib.ptr(y), x.numel() // C, C, float(eps), _s(x)), "mmr_x3_swin_mlp")
    return y


def x3_rowlin_pack(w):
    """f32 weight [n][c] (device) -> the streamed W^T chunks of x3_rowlin, or None if (n, c) is not built."""
    n, c = w.shape
    e = _L().mmr_x3_rowlin_pack_elems(n, c)
    if e <= 0 or (c == 96 and n <= 64):
        return None
    pack = torch.empty((e,), dtype=torch.bfloat16, device=w.device)
    _chk(_L().mmr_x3_rowlin_pack(_lib.ptr(w.contiguous()), _lib.ptr(pack), n, c, _s(w)), "mmr_x3_rowlin_pack")
    return pack


def x3_rowlin(x, pack, bias, n, ln=None, residual=None):
    """y = LN(x) W^T + b (+ residual) for f32 token rows x (..., c) with ln = (gamma, beta, eps), or
    xs W^T + b (+ residual) for an X3Rows x (the window attention's split rows); y f32 (..., n)."""
    if isinstance(x, X3Rows):
        c, lead, xf, xs = x.k, x.lead, None, x.t
    else:
        c, lead, xf, xs = x.shape[-1], tuple(x.shape[:-1]), x.contiguous(), None
        assert ln is not None, "f32 rows are taken with their LayerNorm"
    _lib.require_gpu(x.t if xs is not None else xf)
    rows = 1
    for d in lead:
        rows *= d
    y = torch.empty(lead + (n,), dtype=torch.float32, device=(xs if xs is not None else xf).device)
    r = residual.contiguous() if residual is not None else None
    g, b, eps = ln if ln is not None else (None, None, 0.0)
    _chk(_L().mmr_x3_rowlin(_lib.ptr(xf), _lib.ptr(xs), _lib.ptr(g), _lib.ptr(b), _lib.ptr(pack), _lib.ptr(bias),
                            _lib.ptr(r), _lib.ptr(y), rows, n, c, float(eps), _s(y)), "mmr_x3_rowlin")
    return y


def x3_swin_attn_block_pack(qkv_w, qkv_b, proj_w, proj_b, ln_g, ln_b):
    """f32 weights of one Swin block's attention half (attn.qkv [3C][C] / .bias, attn.proj [C][C] / .bias,
    norm1) -> the LDS image of mmr_x3_swin_attn_block, or None if C is not a fused width (96)."""
    C = qkv_w.shape[1]
    n = _L().mmr_x3_swin_attn_block_pack_bytes(C)
    if n <= 0:
        return None
    pack = torch.empty((n,), dtype=torch.uint8, device=qkv_w.device)
    args = [t.contiguous().float() for t in (qkv_w, qkv_b, proj_w, proj_b, ln_g, ln_b)]
    _chk(_L().mmr_x3_swin_attn_block_pack(*(_lib.ptr(t) for t in args), _lib.ptr(pack), C, _s(qkv_w)),
         "mmr_x3_swin_attn_block_pack")
    return pack


def x3_swin_attn_block(x, pack, bias, ws, shift, eps):
    """x + proj(W-MSA(LN1(x))) for f32 x (B, H, H, C), fused in one pass (C = 96): the x3_rowlin (norm1 +
    qkv) -> x3 window attention -> x3_rowlin (proj + residual) chain."""
    _lib.require_gpu(x)
    B, H, _, C = x.shape
    x = x.contiguous()
    y = torch.empty_like(x)
    _chk(_L().mmr_x3_swin_attn_block(_lib.ptr(x), _lib.ptr(pack), _lib.ptr(bias), _lib.ptr(y), B, H, C, ws, shift,
                                     float(eps), _s(x)), "mmr_x3_swin_attn_block")
    return y


def x3_attention(q, k, v, b, lq, lk, heads, dh, scale, out=None, mean_out=None, mask=None):
    """f32 attention core over strided row views (mmr_x3_attention); mask (b, lk) int64 or None."""
    _lib.require_gpu(q)
    _chk(_L().mmr_x3_attention(_lib.ptr(q), q.stride(0), _lib.ptr(k), k.stride(0), _lib.ptr(v), v.stride(0),
                               _lib.ptr(out), out.stride(0) if out is not None else 0, _lib.ptr(mean_out),
                               _lib.ptr(mask), b, lq, lk, heads, dh, float(scale), _s(q)), "mmr_x3_attention")
    return out, mean_out


def x3_swin_window_attention(qkv, bias, hw, heads, ws, shift):
    B = qkv.shape[0]
    C = qkv.shape[-1] // 3
    out = torch.empty(qkv.shape[:-1] + (C,), dtype=torch.float32, device=qkv.device)
    _chk(_L().mmr_x3_swin_window_attention(_lib.ptr(qkv), _lib.ptr(bias), _lib.ptr(out), B, hw, C, heads, ws, shift,
                                           _s(qkv)), "mmr_x3_swin_window_attention")
    return out


def x3_swin_window_attention_split(qkv, bias, hw, heads, ws, shift):
    """x3_swin_window_attention with its output as X3Rows (the proj GEMM's split operand), for token
    counts filling 256-row tiles; plain f32 rows otherwise."""
    C = qkv.shape[-1] // 3
    M = qkv.numel() // (3 * C)
    kp = _L().mmr_x3_p8_kpad(C)
    if not (M > 0 and M % 256 == 0 and kp > 0):
        return x3_swin_window_attention(qkv, bias, hw, heads, ws, shift)
    xs = torch.empty((M, 2 * kp), dtype=torch.bfloat16, device=qkv.device)
    _chk(_L().mmr_x3_swin_window_attention_xs(_lib.ptr(qkv), _lib.ptr(bias), _lib.ptr(xs), qkv.shape[0], hw, C, heads,
                                              ws, shift, _s(qkv)), "mmr_x3_swin_window_attention_xs")
    return X3Rows(xs, C, kp, tuple(qkv.shape[:-1]))


def x3_attention_split(q, k, v, b, lq, lk, heads, dh, scale, mask=None, mean_out=None):
    """x3_attention's output rows (b*lq, heads*dh) as X3Rows when b*lq fills 256-row tiles, else f32;
    mean_out (b, heads*dh) f32 or None: also the mean over the query rows."""
    C = heads * dh
    kp = _L().mmr_x3_p8_kpad(C)
    if not (b * lq > 0 and (b * lq) % 256 == 0 and kp > 0):
        out = torch.empty((b * lq, C), dtype=torch.float32, device=q.device)
        x3_attention(q, k, v, b, lq, lk, heads, dh, scale, out=out, mask=mask, mean_out=mean_out)
        return out.view(b, lq, C)
    _lib.require_gpu(q)
    xs = torch.empty((b * lq, 2 * kp), dtype=torch.bfloat16, device=q.device)
    _chk(_L().mmr_x3_attention_xs(_lib.ptr(q), q.stride(0), _lib.ptr(k), k.stride(0), _lib.ptr(v), v.stride(0),
                                  _lib.ptr(xs), _lib.ptr(mean_out), _lib.ptr(mask), b, lq, lk, heads, dh, float(scale),
                                  _s(q)),
         "mmr_x3_attention_xs")
    return X3Rows(xs, C, kp, (b, lq))


def x3_patch_im2col(img, patch=4, kp=64):
    B, Cin, H, W = img.shape
    g = H // patch
    cols = torch.empty((B, g * g, kp), dtype=torch.float32, device=img.device)
    _chk(_L().mmr_x3_patch_im2col(_lib.ptr(img), _lib.ptr(cols), B, Cin, H, patch, kp, _s(img)), "mmr_x3_patch_im2col")
    return cols


def x3_patch_embed_pack(w):
    """f32 conv weight (96, 3, 4, 4) or (96, 48) (device) -> the fused x3 stem's weight image, or None when
    the shape is not Swin-T's stem."""
    w2 = w.reshape(w.shape[0], -1)
    if tuple(w2.shape) != (96, 48):
        return None
    pack = torch.empty((_L().mmr_x3_patch_embed_pack_elems(),), dtype=torch.bfloat16, device=w.device)
    _chk(_L().mmr_x3_patch_embed_pack(_lib.ptr(w2.float().contiguous()), _lib.ptr(pack), _s(w)), "mmr_x3_patch_embed_pack")
    return pack


def x3_patch_embed_ln(img, pack, bias, g, b, eps):
    """(B, 3, H, W) f32 -> (B, H/4, W/4, 96) f32 = LayerNorm(conv4x4/s4(img) + bias) (timm PatchEmbed with its
    norm), the conv on bf16x3 MFMA, one pass."""
    _lib.require_gpu(img)
    B, _, H, _ = img.shape
    y = torch.empty((B, H // 4, H // 4, 96), dtype=torch.float32, device=img.device)
    _chk(_L().mmr_x3_patch_embed_ln(_lib.ptr(img), B, H, _lib.ptr(pack), _lib.ptr(bias), _lib.ptr(g), _lib.ptr(b),
                                    float(eps), _lib.ptr(y), _s(img)), "mmr_x3_patch_embed_ln")
    return y


def patch_embed_ln_bf16(img, pack, bias, g, b, eps):
    """(B, 3, H, W) f32 -> (B, H/4, W/4, 96) bf16 = LayerNorm(conv4x4/s4(img) + bias) for the bf16 towers: bf16
    pixels x the bf16 weight (the x3 pack's hi image), bias + LayerNorm in f32, one pass."""
    _lib.require_gpu(img)
    B, _, H, _ = img.shape
    y = torch.empty((B, H // 4, H // 4, 96), dtype=torch.bfloat16, device=img.device)
    _chk(_L().mmr_patch_embed_ln_bf16(_lib.ptr(img), B, H, _lib.ptr(pack), _lib.ptr(bias), _lib.ptr(g), _lib.ptr(b),
                                      float(eps), _lib.ptr(y), _s(img)), "mmr_patch_embed_ln_bf16")
    return y


def x3_patch_merge_ln_split(x, g, b, eps):
    """x3_patch_merge_ln as X3Rows (the reduction linear's split operand) when the merged token count
    fills 256-row tiles, else f32 rows."""
    B, H, W, C = x.shape
    nout = B * (H // 2) * (W // 2)
    kp = _L().mmr_x3_p8_kpad(4 * C)
    if not (nout > 0 and nout % 256 == 0 and kp > 0 and C % 4 == 0):
        return x3_patch_merge_ln(x, g, b, eps)
    xs = torch.empty((nout, 2 * kp), dtype=torch.bfloat16, device=x.device)
    _chk(_L().mmr_x3_patch_merge_ln_xs(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(xs), B, H, C, float(eps), _s(x)),
         "mmr_x3_patch_merge_ln_xs")
    return X3Rows(xs, 4 * C, kp, (B, H // 2, W // 2))


def x3_patch_merge_ln(x, g, b, eps):
    B, H, W, C = x.shape
    y = torch.empty((B, H // 2, W // 2, 4 * C), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_x3_patch_merge_ln(_lib.ptr(x), _lib.ptr(g), _lib.ptr(b), _lib.ptr(y), B, H, C, float(eps), _s(x)),
         "mmr_x3_patch_merge_ln")
    return y


def x3_bert_embed(ids, word, pos, type0, g, b, eps):
    B, L = ids.shape
    C = word.shape[1]
    y = torch.empty((B, L, C), dtype=torch.float32, device=ids.device)
    _chk(_L().mmr_x3_bert_embed(_lib.ptr(ids), _lib.ptr(word), _lib.ptr(pos), _lib.ptr(type0), _lib.ptr(g), _lib.ptr(b),
                                _lib.ptr(y), B, L, C, float(eps), _s(ids)), "mmr_x3_bert_embed")
    return y


def x3_add_pos(x, pos, l):
    c = x.shape[-1]
    rows = x.numel() // c
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    _chk(_L().mmr_x3_add_pos(_lib.ptr(x), _lib.ptr(pos), _lib.ptr(y), rows, l, c, _s(x)), "mmr_x3_add_pos")
    return y


def x3_add_pos_split(x, pos, l, keep_f32=True):
    """x3_add_pos for an x3 linear: rows filling 256-row tiles come back as (y f32 or None, X3Rows)
    (mmr_x3_add_pos_split), other row counts as (y, y)."""
    c = x.shape[-1]
    rows = x.numel() // c
    kp = _L().mmr_x3_p8_kpad(c)
    if not (rows > 0 and rows % 256 == 0 and kp > 0 and c % 4 == 0 and x.is_contiguous()):
        y = x3_add_pos(x, pos, l)
        return y, y
    _lib.require_gpu(x)
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device) if keep_f32 else None
    xs = torch.empty((rows, 2 * kp), dtype=torch.bfloat16, device=x.device)
    _chk(_L().mmr_x3_add_pos_split(_lib.ptr(x), _lib.ptr(pos), _lib.ptr(y), _lib.ptr(xs), rows, l, c, _s(x)),
         "mmr_x3_add_pos_split")
    return y, X3Rows(xs, c, kp, tuple(x.shape[:-1]))


def x3_assemble_seq_split(x1, pf, x2, pe, np_):
    """x3_assemble_seq as X3Rows (the combiner QKV operand) when its rows fill 256-row tiles, else f32."""
    B, c = x1.shape
    rows = B * (np_ + 2)
    kp = _L().mmr_x3_p8_kpad(c)
    if not (rows % 256 == 0 and kp > 0 and c % 4 == 0):
        return x3_assemble_seq(x1, pf, x2, pe, np_)
    xs = torch.empty((rows, 2 * kp), dtype=torch.bfloat16, device=x1.device)
    _chk(_L().mmr_x3_assemble_seq_split(_lib.ptr(x1), _lib.ptr(pf), _lib.ptr(x2), _lib.ptr(pe), _lib.ptr(xs), B, np_, c,
                                        _s(x1)), "mmr_x3_assemble_seq_split")
    return X3Rows(xs, c, kp, (rows,))


def x3_assemble_seq(x1, pf, x2, pe, np_):
    B, c = x1.shape
    seq = torch.empty((B, np_ + 2, c), dtype=torch.float32, device=x1.device)
    _chk(_L().mmr_x3_assemble_seq(_lib.ptr(x1), _lib.ptr(pf), _lib.ptr(x2), _lib.ptr(pe), _lib.ptr(seq), B, np_, c,
                                  _s(x1)), "mmr_x3_assemble_seq")
    return seq


def x3_mean_rows(x, extra=None):
    """(B, L, C) f32 -> (B, C): sum_t x / L, or (extra + sum_t x) / (L + 1)."""
    B, L, C = x.shape
    y = torch.empty((B, C), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_x3_mean_rows(_lib.ptr(x), _lib.ptr(extra), _lib.ptr(y), B, L, C, _s(x)), "mmr_x3_mean_rows")
    return y


def x3_gather_rows(x, b, c, ldx, out=None):
    y = out if out is not None else torch.empty((b, c), dtype=torch.float32, device=x.device)
    _chk(_L().mmr_x3_gather_rows(_lib.ptr(x), ldx, _lib.ptr(y), b, c, _s(x)), "mmr_x3_gather_rows")
    return y
