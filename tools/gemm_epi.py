"""Isolate epilogue cost of mmr_linear_bf16 (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mmr_amd import ops
M, N, K = 32768, 3072, 768
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3
fl = 2.0 * M * N * K
for name, kw in [("plain", {}), ("bias+gelu", dict(bias=b, act=1)),
                 ("bias+res", dict(bias=b, residual=r))]:
    us = t(lambda: ops.linear(x, w, **kw))
    print(f"{name:<10} {us:8.1f} us {fl/us/1e6:7.0f} TF/s")
x2 = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
us = t(lambda: ops.linear(x2 * 0, w, b, act=1))
print(f"zeros-in bias+gelu {us:8.1f} us")
