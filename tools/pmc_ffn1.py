"""The BERT FFN1 kernel the timed cfg2 / cfg5 steps run, launched N times for rocprofv3 --pmc passes:
  fold: mmr_linear_bf16_ln ln_mode 1 + GELU (bf16, LayerNorm folded; gemm_bf16_tn_p8<4, 1, LNM=1>)
  mx8:  mmr_linear_mxfp8_q8 + GELU (MX-fp8 in, fp8 operand of FFN2 out; gemm_bf16_tn_p8<4, 1, FP8, OUT8>)
usage: python tools/pmc_ffn1.py fold|mx8 [M] [launches] [tag: also time the launches with HIP events]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402
from mmr_amd.towers import _ln_fold, _w8  # noqa: E402

mode = sys.argv[1]
M = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
n_launch = int(sys.argv[3]) if len(sys.argv) > 3 else 5
C, N = 768, 3072
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: torch.randn(*s, generator=g, device="cuda")  # noqa: E731
w, b = (rnd(N, C) * C ** -0.5).to(torch.bfloat16), rnd(N)
y = (rnd(M, C) * 2).to(torch.bfloat16)
if mode == "fold":
    gam, bet = 1 + 0.1 * rnd(C), 0.1 * rnd(C)
    wf, c, d = _ln_fold(w, b, gam, bet)
    ctx, wo = rnd(M, C).to(torch.bfloat16), (rnd(C, C) * C ** -0.5).to(torch.bfloat16)
    _, st = ops.linear_ln(ctx, wo, rnd(C), residual=y, want_stats=True)
    cf = ops.ln_row_coef(st, C, 1e-12)
    run = lambda: ops.linear_ln(y, wf, d, act=1, ln_mode=1, coef=cf, v1=c)  # noqa: E731
elif mode == "mx8":
    w8 = _w8(w, plain=True)
    x8 = ops.quantize_mxfp8(y, layout=0, kp=w8.kp)
    run = lambda: ops.linear_mxfp8_q8(x8, w8, b, act=1)  # noqa: E731
else:
    raise SystemExit(f"unknown mode {mode}")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
run()
e0.record()
for _ in range(n_launch):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / n_launch * 1e3
fl = 2.0 * M * N * C
tag = sys.argv[4] if len(sys.argv) > 4 else ""
print(f"{tag} {mode} M={M} N={N} K={C}: {n_launch} launches, {us:.1f} us each = {fl / us / 1e6:.0f} TF "
      f"({fl / us / 1e6 / (5000 if mode == 'mx8' else 2500):.3f} of the dtype's dense peak)")
