"""Effective clock of the bf16 vs MX-fp8 8-phase GEMM (run under rocprofv3 --pmc GRBM_GUI_ACTIVE
--kernel-trace): clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md, DVFS).
Random operands, the cfg5 QKV / FFN1 / FFN2 shapes, 6 launches each.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

for M, N, K, act in [(262144, 2304, 768, 0), (262144, 3072, 768, 1), (262144, 768, 3072, 0)]:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    w8 = ops.quantize_mxfp8(w, layout=2 if (N % 256 == 0 and not act) else 1)
    x8 = ops.quantize_mxfp8(x, layout=0)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(6):
        ops.linear(x, w, b, act=act, out=y)
    for _ in range(6):
        ops.linear_mxfp8(x8, w8, b, act=act, out=y)
    torch.cuda.synchronize()
    del x, w, x8, w8, y
print("done")
