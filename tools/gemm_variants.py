"""Time one GEMM shape under the launcher's diagnostic variants (env MMR_GEMM_W4 / MMR_GEMM_BIG are
read per launch) plus torch F.linear (hipBLASLt) for the plain GEMM.
usage: python tools/gemm_variants.py M N K act [res]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mmr_amd import ops  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


M, N, K, act = (int(v) for v in sys.argv[1:5])
res = len(sys.argv) > 5 and sys.argv[5] == "1"
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if res else None
fl = 2.0 * M * N * K
out = [f"M={M} N={N} K={K} act={act} res={int(res)}"]
ref = x.float() @ w.float().t() + b
if act == 1:
    ref = F.gelu(ref)
if res:
    ref = ref + r.float()
for v in range(ops._L().mmr_linear_bf16_n_variants()):
    with ops.pinned(ops.PIN_GEMM_BF16, v):
        t = timeit(lambda: ops.linear(x, w, b, r, act=act))
        err = (ops.linear(x, w, b, r, act=act).float() - ref).abs().max().item()
    out.append(f"  variant {v:2d}: {t:8.1f} us  {fl / t / 1e6:7.0f} TF/s  max|err| {err:.3g}")
t = timeit(lambda: F.linear(x, w, b.to(torch.bfloat16)))
out.append(f"  hipBLASLt plain: {t:8.1f} us  {fl / t / 1e6:7.0f} TF/s")
print("\n".join(out), flush=True)
