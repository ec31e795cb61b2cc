"""One GEMM shape under a pinned launch variant, for rocprofv3 --pmc traffic passes (the bench's
roofline kernel is whichever variant the per-shape tuner picked on that box; this measures each
candidate the same way).  usage: python tools/pmc_gemm.py M N K act variant [launches]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# variant index -> (w4, cfg) of the launcher's kVarW4 / kVarCfg tables (gemm.hip), for the log line
VARIANTS = [(1, 1), (2, 1), (0, 1), (0, 2), (0, 3), (0, 4), (0, 5), (0, 6), (0, 0), (0, 7), (0, 8)]
M, N, K, act, v = (int(x) for x in sys.argv[1:6])
n_launch = int(sys.argv[6]) if len(sys.argv) > 6 else 5
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402

x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
b = torch.randn(N, device="cuda")
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
with ops.pinned(ops.PIN_GEMM_BF16, v):
    for _ in range(n_launch):
        ops.linear(x, w, b, act=act, out=y)
torch.cuda.synchronize()
print(f"M={M} N={N} K={K} act={act} variant={v} {VARIANTS[v]}: {n_launch} launches")
