"""Square-ish GEMM rates (diagnostic): mine vs torch for large K to isolate main-loop efficiency."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from mmr_amd import ops
for (M, N, K) in [(8192, 8192, 8192), (32768, 3072, 768), (32768, 3072, 3072), (16384, 4096, 4096)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    def t(fn, it=10):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it): fn()
        e1.record(); torch.cuda.synchronize()
        return e0.elapsed_time(e1) / it
    tm = t(lambda: ops.linear(x, w))
    tt = t(lambda: F.linear(x, w))
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K}: mine {fl/tm/1e9:.0f} TF/s, hipblaslt {fl/tt/1e9:.0f} TF/s")
