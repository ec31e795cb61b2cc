"""Times the tuned bf16 GEMM (ops.linear) on the cfg2 tower shapes with whichever libmmr MMR_LIBMMR
selects (HIP events, random operands; the variant the tuner picked is printed).  Run it once per
library, interleaved, for a same-box A/B.  Diagnostic only.
usage: [MMR_LIBMMR=...] python tools/lib_ab.py [tag]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import _lib, ops  # noqa: E402

SHAPES = [(32768, 2304, 768, 0, 0), (32768, 3072, 768, 1, 0), (32768, 768, 3072, 0, 0), (32768, 768, 768, 0, 0),
          (50176, 1152, 384, 0, 0), (50176, 1536, 384, 1, 0), (50176, 384, 1536, 0, 1), (50176, 384, 384, 0, 1),
          (12544, 2304, 768, 0, 0), (12544, 768, 768, 0, 0), (12544, 768, 768, 0, 1)]


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


tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(_lib.LIB_PATH)
L = _lib.lib()
row = []
for M, N, K, act, res in SHAPES:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16) if res else None
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    us = timeit(lambda: ops.linear(x, w, b, residual=r, act=act, out=y))
    v = -1
    if hasattr(L, "mmr_linear_bf16_variant"):
        v = L.mmr_linear_bf16_variant(ctypes.c_int64(M), N, K, act, 1, 1 if res else 0)
    row.append(f"{M}x{N}x{K}{'g' if act else ''}{'r' if res else ''} {us:7.1f}us {2 * M * N * K / us / 1e6:5.0f}TF v{v}")
print(tag, " | ".join(row), flush=True)
