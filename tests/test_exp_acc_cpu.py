"""The x3 softmax's exp (common.h mmr::exp_acc) restated in f32 numpy: 2^t with t = RN(x log2 e) and t's
rounding error carried to first order, checked against f64 exp on 2M arguments in [-40, 0] (the softmax's
x = s - max range) and at the clamp (a masked score, HF's -FLT_MAX, gives 0, not NaN).  The device's
v_exp_f32 (exp2) is modelled as correctly rounded here; it adds <= 1 ulp on the hardware
(tests/test_x3_gpu.py holds the kernels to the f64 oracle)."""
import numpy as np

F = np.float32
L2E, L2E_LO, LN2 = F(1.44269504088896341), F(1.925962991e-08), F(0.69314718055994531)


def exp_acc(x):
    """Elementwise restatement (fma as an exact f64 product-sum rounded once to f32)."""
    x = np.maximum(x.astype(F), F(-104.0))
    t = (x * L2E).astype(F)
    inner = (x.astype(np.float64) * np.float64(L2E) - t.astype(np.float64)).astype(F)
    c = (x.astype(np.float64) * np.float64(L2E_LO) + inner.astype(np.float64)).astype(F)
    e = np.exp2(t.astype(np.float64)).astype(F)
    return (e.astype(np.float64) * (c * LN2).astype(np.float64) + e.astype(np.float64)).astype(F)


def test_exp_acc_within_one_ulp():
    x = -np.random.default_rng(0).uniform(0, 40, 2_000_000).astype(F)
    ref = np.exp(x.astype(np.float64))
    got = exp_acc(x).astype(np.float64)
    ulp = np.spacing(ref.astype(F)).astype(np.float64)
    assert (np.abs(got - ref) / ulp).max() <= 1.0
    naive = np.exp2((x * L2E).astype(F).astype(np.float64)).astype(F).astype(np.float64)
    assert (np.abs(naive - ref) / ulp).max() > 8.0  # what the carried rounding error fixes


def test_exp_acc_masked_scores_and_zero():
    x = np.array([-3.4028235e38, -1e30, -104.0, -200.0, 0.0], dtype=F)
    got = exp_acc(x)
    assert np.isfinite(got).all()
    assert got[0] == 0.0 and got[1] == 0.0 and got[3] == 0.0 and got[4] == 1.0
