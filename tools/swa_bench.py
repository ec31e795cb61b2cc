"""Times mmr_swin_window_attention at the Swin-T stage 2-4 geometries (B = 256, as in the cfg2
step) with whichever libmmr MMR_LIBMMR selects; HIP events, random operands.  Diagnostic only.
usage: [MMR_LIBMMR=...] python tools/swa_bench.py [tag]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

B = int(os.environ.get("SWA_B", "256"))
row = []
for H, heads, shift in [(28, 6, 0), (28, 6, 3), (14, 12, 3), (7, 24, 0)]:
    C = heads * 32
    qkv = torch.randn(B, H, H, 3 * C, device="cuda").to(torch.bfloat16)
    bias = ops.swin_attn_bias(torch.randn(169, heads, device="cuda"), heads, 7, H, shift)
    if os.environ.get("SWA_Q8") == "1":  # the MX-fp8-emitting form (fp8 stages)
        f = lambda: ops.swin_window_attention_q8(qkv, bias, H, heads, 7, shift)  # noqa: E731
    else:
        f = lambda: ops.swin_window_attention(qkv, bias, H, heads, 7, shift)  # noqa: E731
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    gb = B * H * H * 4 * C * 2 / us / 1e3
    row.append(f"H{H}s{shift} {us:6.1f}us {gb:5.0f}GB/s")
print(sys.argv[1] if len(sys.argv) > 1 else "", " | ".join(row), flush=True)
