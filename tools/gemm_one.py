"""Run one tower GEMM shape repeatedly (for rocprofv3 counter collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mmr_amd import ops
M, N, K, act = (int(x) for x in sys.argv[1:5])
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
for _ in range(int(sys.argv[5]) if len(sys.argv) > 5 else 10):
    ops.linear(x, w, b, act=act)
torch.cuda.synchronize()
