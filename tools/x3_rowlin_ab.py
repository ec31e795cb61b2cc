"""x3 Swin stage-1/2 linears at B = 256: the streamed row-linear (mmr_x3_rowlin: norm1 + qkv from f32 rows,
proj + residual from the window attention's split rows) vs the x3 GEMM route (LayerNorm split pass + the
K' = 3 kp split GEMM), time per call (HIP events, min of 3 x 10) and max rel diff.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import _lib, ops  # noqa: E402


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


g = torch.Generator().manual_seed(2)
for hw, C in ((56, 96), (28, 192)):
    T = 256 * hw * hw
    x = (torch.randn(T, C, generator=g) * 1.5).cuda()
    gm, bt = (1 + 0.1 * torch.randn(C, generator=g)).cuda(), (0.1 * torch.randn(C, generator=g)).cuda()
    for N, kind in ((3 * C, "qkv"), (C, "proj")):
        w, b = (torch.randn(N, C, generator=g) * C ** -0.5).cuda(), (0.1 * torch.randn(N, generator=g)).cuda()
        W, pack = ops.X3W(w), ops.x3_rowlin_pack(w)
        if kind == "qkv":
            new = lambda: ops.x3_rowlin(x, pack, b, N, ln=(gm, bt, 1e-5))  # noqa: E731
            old = lambda: ops.x3_linear(ops.x3_ln_split(x, gm, bt, 1e-5), W, b)  # noqa: E731
        else:
            kp = _lib.lib().mmr_x3_p8_kpad(C)
            xs = torch.zeros(T, 2 * kp, dtype=torch.bfloat16, device="cuda")
            xs[:, :C] = x.to(torch.bfloat16)
            xs[:, kp:kp + C] = (x - xs[:, :C].float()).to(torch.bfloat16)
            xr = ops.X3Rows(xs, C, kp, (T,))
            r = torch.randn(T, C, generator=g).cuda()
            new = lambda: ops.x3_rowlin(xr, pack, b, N, residual=r)  # noqa: E731
            old = lambda: ops.x3_linear(xr, W, b, residual=r)  # noqa: E731
        tn = min(timeit(new) for _ in range(3))
        to = min(timeit(old) for _ in range(3))
        yn, yo = new(), old()
        torch.cuda.synchronize()
        err = (yn - yo).abs().max().item() / yo.abs().max().item()
        print(f"C={C:4d} {kind:4s} N={N:4d} T={T}: gemm route {to:8.1f} us  rowlin {tn:8.1f} us  x{to / tn:5.2f}  "
              f"rel diff {err:.2e}", flush=True)
    del x
