"""K sweep of the 8-phase GEMM (bf16 and MX-fp8, plain bias epilogue) at M = 262144, N = 2304:
time per 256x256 tile = a + b*K, so a = the per-tile fixed cost (epilogue, tile switch) and b the
steady-state K-loop rate.  HIP events, random operands, 10 launches each.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import _lib, ops  # noqa: E402


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


M, N = int(os.environ.get("KS_M", 262144)), int(os.environ.get("KS_N", 2304))
tiles = (M // 256) * (N // 256)
rounds = tiles / 256
res = {"bf16": [], "fp8": []}
for K in [256, 512, 768, 1024, 1536, 2048, 3072]:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    t_bf = timeit(lambda: ops.linear(x, w, b, out=y))
    v = _lib.lib().mmr_linear_bf16_variant(M, N, K, 0, 1, 0)
    w8 = ops.quantize_mxfp8(w, layout=2)
    x8 = ops.quantize_mxfp8(x, layout=0)
    t_mx = timeit(lambda: ops.linear_mxfp8(x8, w8, b, out=y))
    fl = 2.0 * M * N * K
    res["bf16"].append((K, t_bf / rounds))
    res["fp8"].append((K, t_mx / rounds))
    print(f"K={K:5d} bf16 {t_bf:8.1f}us {fl / t_bf / 1e6:5.0f}TF (variant {v}) {t_bf / rounds:6.2f}us/tile-round | "
          f"fp8 {t_mx:8.1f}us {fl / t_mx / 1e6:5.0f}TF {t_mx / rounds:6.2f}us/tile-round", flush=True)
    del x, w, x8, w8, y
for k, v in res.items():
    K = np.array([a for a, _ in v], float)
    T = np.array([b for _, b in v], float)
    sel = K >= 512
    bb, aa = np.polyfit(K[sel], T[sel], 1)
    print(f"{k}: per tile-round {aa:.2f} us fixed + {bb * 1e3:.2f} ns per k (fit over K >= 512); "
          f"K=768: fixed share {aa / (aa + bb * 768):.2f}")
