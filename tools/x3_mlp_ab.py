"""(Round-5 record profiles/r05_x3_mlp_ab.txt; its erff arm used a pin that is gone.)
x3 Swin MLP A/B at B = 256: the fused kernel (mmr_x3_swin_mlp) vs the unfused x3 chain (LayerNorm split
-> fc1 GEMM writing split rows -> fc2 GEMM + residual) for stages 1-4 geometry, time per call (HIP events,
min of 3 x 10) and max |fused - chain| / max|chain|.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import _lib, ops  # noqa: E402

L = _lib.lib()


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


g = torch.Generator().manual_seed(1)
for hw, C in ((56, 96), (28, 192)):
    T = 256 * hw * hw
    x = (torch.randn(T, C, generator=g) * 1.5).cuda()
    gm, bt = (1 + 0.1 * torch.randn(C, generator=g)).cuda(), (0.1 * torch.randn(C, generator=g)).cuda()
    w1, b1 = (torch.randn(4 * C, C, generator=g) * C ** -0.5).cuda(), (0.1 * torch.randn(4 * C, generator=g)).cuda()
    w2, b2 = (torch.randn(C, 4 * C, generator=g) * (4 * C) ** -0.5).cuda(), (0.1 * torch.randn(C, generator=g)).cuda()
    W1, W2 = ops.X3W(w1), ops.X3W(w2)
    pack = ops.x3_swin_mlp_pack(w1, w2)
    fused = lambda: ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)  # noqa: E731
    chain = lambda: ops.x3_ffn(ops.x3_ln_split(x, gm, bt, 1e-5), W1, b1, W2, b2, residual=x)  # noqa: E731
    tc = min(timeit(chain) for _ in range(3))
    yc = chain()
    gf = 48.0 * T * C * C / 1e9
    for name in ("fused",):
        tf = min(timeit(fused) for _ in range(3))
        yf = fused()
        torch.cuda.synchronize()
        err = (yf - yc).abs().max().item() / yc.abs().max().item()
        print(f"C={C:4d} T={T:7d}: chain {tc:8.1f} us  {name} {tf:8.1f} us  x{tc / tf:5.2f}  ({gf / tf:.2f} PF bf16 "
              f"MFMA work)  rel diff vs chain {err:.2e}", flush=True)
    del x
