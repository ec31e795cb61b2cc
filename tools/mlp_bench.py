"""Timing of the fused Swin MLP (mmr_swin_mlp) vs the unfused LN -> fc1(GELU) -> fc2(+res) chain on
the Swin-T stage-1/2 shapes (B=256).  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mmr_amd import ops


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
only = sys.argv[2] if len(sys.argv) > 2 else ""   # "96" / "192": fused kernel only (for PMC runs)
for C, T in ((96, B * 3136), (192, B * 784)):
    if only and str(C) != only:
        continue
    g = torch.Generator(device="cuda").manual_seed(C)
    x = (torch.randn(T, C, device="cuda", generator=g) * 2).bfloat16()
    lg, lb = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    w1 = (torch.randn(4 * C, C, device="cuda", generator=g) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device="cuda", generator=g) * (2 * C) ** -0.5).bfloat16()
    b1, b2 = torch.zeros(4 * C, device="cuda"), torch.zeros(C, device="cuda")
    pack = ops.swin_mlp_pack(w1, w2)
    fused = timeit(lambda: ops.swin_mlp(x, lg, lb, pack, b1, b2, 1e-5), 5 if only else 20)
    if only:
        print(f"C={C}: fused {fused:.1f} us")
        continue

    def chain():
        h = ops.layernorm(x, lg, lb, 1e-5)
        h = ops.linear(h, w1, b1, act=1)
        return ops.linear(h, w2, b2, residual=x)
    unf = timeit(chain)
    fl = 2 * T * C * 4 * C * 2
    print(f"C={C} T={T}: fused {fused:8.1f} us ({fl / fused / 1e6:6.1f} TF/s, {4 * T * C / fused / 1e3:6.0f} GB/s)"
          f"   unfused {unf:8.1f} us   max|diff| {(ops.swin_mlp(x, lg, lb, pack, b1, b2, 1e-5).float() - chain().float()).abs().max().item():.3e}")
