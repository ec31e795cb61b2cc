"""Isolate the epilogue cost of mmr_linear_bf16 on one shape (diagnostic).
usage: python tools/gemm_epi.py [M N K]   (env MMR_GEMM_BIG selects the tile config)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from mmr_amd import ops

M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (32768, 3072, 768)
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


fl = 2.0 * M * N * K
out = [f"M={M} N={N} K={K} cfg={os.environ.get('MMR_GEMM_BIG', 'default')}:"]
for name, kw in [("plain", {}), ("bias", dict(bias=b)), ("bias+gelu", dict(bias=b, act=1)),
                 ("bias+res", dict(bias=b, residual=r))]:
    us = t(lambda: ops.linear(x, w, **kw))
    out.append(f"{name} {us:.1f}us/{fl / us / 1e6:.0f}TF")
ref = (x.float() @ w.float().T + b + r.float())
err = (ops.linear(x, w, bias=b, residual=r).float() - ref).abs().max().item() / ref.abs().max().item()
us = t(lambda: F.linear(x, w))
out.append(f"| hipBLASLt {us:.1f}us/{fl / us / 1e6:.0f}TF | relerr {err:.1e}")
print("  ".join(out))
