"""Throughput of the MX-fp8 GEMM (mmr_linear_mxfp8) vs the bf16 GEMM (tuned) on the config-5 tower
shapes (B = 2048), and of the activation quantiser; HIP events, random operands.  Diagnostic only.
usage: python tools/gemm_mx.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

SHAPES = [(262144, 2304, 768, 0), (262144, 768, 768, 0), (262144, 3072, 768, 1), (262144, 768, 3072, 0),
          (401408, 1152, 384, 0), (401408, 1536, 384, 1), (401408, 384, 1536, 0), (100352, 2304, 768, 0)]


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for M, N, K, act in SHAPES:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    w8 = ops.quantize_mxfp8(w, layout=2 if (N % 256 == 0 and not act) else 1)
    x8 = ops.quantize_mxfp8(x, layout=0)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    t_bf = timeit(lambda: ops.linear(x, w, b, act=act, out=y))
    t_mx = timeit(lambda: ops.linear_mxfp8(x8, w8, b, act=act, out=y))
    t_q = timeit(lambda: ops.quantize_mxfp8(x, layout=0))
    t_q8 = None
    if N % 256 == 0:
        w8b = ops.quantize_mxfp8(w, layout=2)
        t_q8 = timeit(lambda: ops.linear_mxfp8_q8(x8, w8b, b, act=act))
    fl = 2.0 * M * N * K
    print(f"M={M:6d} N={N:5d} K={K:5d} act={act} | bf16 {t_bf:7.1f}us {fl / t_bf / 1e6:5.0f}TF | mxfp8 {t_mx:7.1f}us "
          f"{fl / t_mx / 1e6:5.0f}TF | quantise x {t_q:6.1f}us ({M * K * 3 / t_q / 1e6:5.2f} TB/s)"
          + (f" | q8-out {t_q8:7.1f}us {fl / t_q8 / 1e6:5.0f}TF" if t_q8 else ""), flush=True)
    del x, w, x8, w8, y
