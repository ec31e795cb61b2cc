"""ORACLE (test infrastructure): MX-fp8 (OCP e4m3 elements, one E8M0 scale per 32 consecutive k)
quantisation restated in numpy, the checker of mmr_quantize_mxfp8 / mmr_linear_mxfp8 (the fp8 tower
path of BASELINE.json config 5; the reference itself runs the towers in fp32, fusion.py:198-199,
322-325, so there is no reference fp8 output to pin against — the restatement is pinned instead to
torch's own float8_e4m3fn conversion in tests/test_oracle_golden.py).

quantize(x)      -> (q values as f32 on the e4m3 grid, scale exponents e) per row / 32-block:
                    e = the smallest integer with amax <= 448 * 2^e (clamped to [-127, 126]),
                    q = round-to-nearest-even(x * 2^-e) onto e4m3 (normal step 2^(E-3), subnormal
                    step 2^-9; |x * 2^-e| <= 448 so nothing saturates).
dequantize       q * 2^e.
scale_offsets    (row, block) -> byte offset of the scale in the GEMM's LDS-image order (layout 0:
                 activations, panels of 256 rows; layouts 1 / 2: weights, panels of 192 / 256 rows)."""
import numpy as np


def e4m3_round(v):
    """f32 -> nearest (ties to even) OCP e4m3fn value, |v| <= 448."""
    v = np.asarray(v, np.float32)
    a = np.abs(v)
    ex = ((a.view(np.uint32) >> 23) & 255).astype(np.int32) - 127  # binade of |v|, exact from the bits
    step = np.where(ex >= -6, np.ldexp(np.float32(1.0), ex - 3), np.float32(2.0 ** -9)).astype(np.float32)
    return (np.rint(v / step) * step).astype(np.float32)


def block_exponents(x):
    """x [rows][k] f32 (k % 32 == 0) -> e [rows][k/32] int32."""
    x = np.asarray(x, np.float32)
    amax = np.abs(x.reshape(x.shape[0], -1, 32)).max(-1).astype(np.float32)
    ab = amax.view(np.uint32)
    e = ((ab >> 23) & 255).astype(np.int32) - 127 - 8 + ((ab & 0x7FFFFF) > 0x600000).astype(np.int32)
    return np.clip(e, -127, 126)


def quantize(x, kp=None):
    """x [rows][k] (bf16 values as f32) -> (q [rows][kp] f32 on the e4m3 grid, e [rows][kp/32])."""
    x = np.asarray(x, np.float32)
    rows, k = x.shape
    kp = kp or -(-k // 256) * 256
    xp = np.zeros((rows, kp), np.float32)
    xp[:, :k] = x
    e = block_exponents(xp)
    inv = np.ldexp(np.float32(1.0), -np.repeat(e, 32, axis=1)).astype(np.float32)
    return e4m3_round(xp * inv), e


def dequantize(q, e):
    return (np.asarray(q, np.float64) * np.ldexp(1.0, np.repeat(np.asarray(e), 32, axis=1))).astype(np.float64)


def scale_offsets(rows, kp, layout):
    """[rows][kp/32] int64 byte offsets of each (row, block) scale in the image order."""
    r = np.arange(rows)[:, None]
    blk = np.arange(kp // 32)[None, :]
    kt, fq = blk // 4, blk % 4
    if layout == 0:
        P, rr = r // 256, r % 256
        wr, i, fr = rr // 128, (rr % 128) // 16, rr % 16
        return (P * (kp // 128) + kt) * 1024 + ((wr * 4 + fq) * 16 + fr) * 8 + i
    pr = 192 if layout == 1 else 256          # weight panels: 256 x 192 (1) or 256 x 256 (2) GEMM tiles
    wt = pr // 4
    P, rr = r // pr, r % pr
    wc, j, fr = rr // wt, (rr % wt) // 16, rr % 16
    return (P * (kp // 128) + kt) * 1024 + ((wc * 4 + fq) * 16 + fr) * 4 + j


def e4m3_decode(b):
    """OCP e4m3fn bytes -> f32 (NaN for 0x7F / 0xFF)."""
    b = np.asarray(b, np.uint8).astype(np.int32)
    s = np.where(b & 0x80, -1.0, 1.0)
    E = (b >> 3) & 15
    m = b & 7
    v = np.where(E == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * np.ldexp(1.0, E - 7))
    v = np.where((b & 0x7F) == 0x7F, np.nan, v)
    return (s * v).astype(np.float32)


GELU_Q8_A, GELU_Q8_B = np.float32(1.60031416), np.float32(0.06940179)


def gelu_q8(x):
    """The GELU the MX-fp8 output epilogue computes (csrc/common.h gelu_q8x2: x sigmoid(x (a + b x^2)), (a, b)
    minimax-fitted to the erf form), restated in f32 numpy (the device's v_exp / v_rcp differ by ~1 ulp)."""
    x = np.asarray(x, np.float32)
    p = (GELU_Q8_B * (x * x) + GELU_Q8_A).astype(np.float32)
    return (x / (np.float32(1) + np.exp(-(x * p)).astype(np.float32))).astype(np.float32)

