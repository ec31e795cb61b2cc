"""Resident-weight streaming linear (mmr_linear_rw) vs the tuned bf16 GEMM (mmr_linear_bf16) on the
Swin short-K shapes of the cfg2 step (B = 256); HIP events, random operands, max |difference| of
the two outputs.  Diagnostic only.  usage: python tools/rw_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

SHAPES = [(802816, 96, 64, True, False), (200704, 576, 192, True, False), (200704, 192, 192, True, True),
          (200704, 192, 384, False, False), (50176, 384, 384, True, True), (50176, 1152, 384, True, False)]


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for M, N, K, bias, res in SHAPES:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") if bias else None
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16) if res else None
    pk = ops.rw_pack(w)
    if pk is None:
        print(f"M={M} N={N} K={K}: not taken")
        continue
    y1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    t_g = timeit(lambda: ops.linear(x, w, b, r, out=y1))
    t_r = timeit(lambda: ops.linear_rw(x, pk, b, r, out=y2))
    by = M * K * 2 + M * N * 2 * (2 if res else 1)
    d = (y1.float() - y2.float()).abs().max().item()
    print(f"M={M:6d} N={N:4d} K={K:3d} b={int(bias)} r={int(res)} | gemm {t_g:6.1f}us | rw {t_r:6.1f}us "
          f"{by / t_r / 1e3:5.0f}GB/s (min bytes) | max|diff| {d:.3g}", flush=True)
