"""The cheap GELU of the MX-fp8 output epilogue (csrc/common.h gelu_q8x2: x sigmoid(x (a + b x^2)), used where
the GELU's output is quantised to e4m3 — the fused FFN1 -> FFN2 operand, BERT / Swin stages 3-4 at config 5)
against the erf form the reference's nn.GELU computes (HF BertIntermediate / timm Mlp, reached through
src/Model/fusion.py:198-199, 322-325), restated in f32 numpy on 1M values: its error stays under half an
e4m3 ulp (3 mantissa bits: 2^-5 relative at the least) wherever the value is not negligible against a block's
amax, and under 2.8e-4 absolute everywhere."""
import numpy as np
from scipy.special import erf

from oracle.mxfp8 import gelu_q8


def test_gelu_q8_under_half_e4m3_ulp():
    rng = np.random.default_rng(8)
    x = np.concatenate([np.linspace(-12, 12, 500_001), rng.normal(0, 3, 500_000)]).astype(np.float32)
    g = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    y = gelu_q8(x).astype(np.float64)
    err = np.abs(y - g)
    assert err.max() <= 2.75e-4, err.max()
    big = np.abs(g) >= 1e-2
    rel = err[big] / np.abs(g[big])
    assert rel.max() < 2.0 ** -5, rel.max()           # under the smallest e4m3 half-ulp (relative)
    assert rel.max() <= 0.0235, rel.max()
    # against a block's quantisation: e4m3 of a 32-block with amax >= 0.5 rounds to steps >= amax 2^-11
    # below its subnormal range, 2^-4 amax at the top; the approximation error is 2^-11 of amax = 0.5
    assert err.max() <= 0.5 * 2.0 ** -10
