"""Fit of GELU(x) = x * Phi(x) by x * sigmoid(x * P(x^2)), P of degree 4 (mmr::gelu_fast in
csrc/common.h).  Prints the coefficients and the max |error| against the exact erf form."""
import numpy as np
from scipy.optimize import least_squares
from scipy.special import ndtr

x = np.linspace(-7, 7, 200001)
ref = x * ndtr(x)


def model(c, v):
    return v / (1 + np.exp(-v * np.polyval(c[::-1], v * v)))


c = least_squares(lambda cc: model(cc, x) - ref, np.array([1.5957691, 0.0713548, 0.0, 0.0, 0.0])).x
for _ in range(30):  # iteratively reweighted least squares towards minimax
    e = model(c, x) - ref
    w = 1 + 50 * (np.abs(e) / np.abs(e).max()) ** 2
    c = least_squares(lambda cc: (model(cc, x) - ref) * w, c).x
print("coefficients (x^0 .. x^8):", c.tolist())
print("max |err| on [-7, 7]:", np.abs(model(c, x) - ref).max())
xx = np.linspace(-40, 40, 100001)
with np.errstate(over="ignore"):
    print("max |err| on [-40, 40]:", np.abs(model(c, xx) - xx * ndtr(xx)).max())
