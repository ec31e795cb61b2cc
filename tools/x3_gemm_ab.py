"""x3 split GEMMs for whichever libmmr MMR_LIBMMR selects: the BERT FFN (fc1 + GELU writing split rows ->
fc2, M = 32768, 768 -> 3072 -> 768), BERT QKV (N = 2304) and the Swin stage-3 fc1 + GELU (M = 50176,
384 -> 1536), time per call (HIP events, min of 3 x 10) and a checksum.  Run once per library,
interleaved, for a same-box A/B.  Diagnostic only.  usage: python tools/x3_gemm_ab.py <tag> [M]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402


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


tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("MMR_LIBMMR", "libmmr.so"))
g = torch.Generator().manual_seed(4)
M, C, F4 = (int(sys.argv[2]) if len(sys.argv) > 2 else 32768), 768, 3072
x = torch.randn(M, C, generator=g).cuda()
gm, bt = torch.ones(C).cuda(), torch.zeros(C).cuda()
w1, b1 = ops.X3W((torch.randn(F4, C, generator=g) * C ** -0.5).cuda()), (0.1 * torch.randn(F4, generator=g)).cuda()
w2, b2 = ops.X3W((torch.randn(C, F4, generator=g) * F4 ** -0.5).cuda()), (0.1 * torch.randn(C, generator=g)).cuda()
wq, bq = ops.X3W((torch.randn(3 * C, C, generator=g) * C ** -0.5).cuda()), (0.1 * torch.randn(3 * C, generator=g)).cuda()
xs = ops.x3_ln_split(x, gm, bt, 1e-5)
for name, fn, gf in (("bert ffn (fc1+gelu, fc2)", lambda: ops.x3_ffn(xs, w1, b1, w2, b2), 6.0 * 2 * M * C * F4),
                     ("bert qkv", lambda: ops.x3_linear(xs, wq, bq), 6.0 * M * C * 3 * C)):
    t = min(timeit(fn) for _ in range(3))
    y = fn()
    torch.cuda.synchronize()
    print(f"{tag:8s} {name:28s} {t:8.1f} us  {gf / t / 1e9:.2f} PF bf16 MFMA work  checksum {float(y.double().sum()):.6e}",
          flush=True)
M3, C3 = 50176, 384
x3 = torch.randn(M3, C3, generator=g).cuda()
w3, b3 = ops.X3W((torch.randn(4 * C3, C3, generator=g) * C3 ** -0.5).cuda()), (0.1 * torch.randn(4 * C3, generator=g)).cuda()
t = min(timeit(lambda: ops.x3_linear(x3, w3, b3, act=1)) for _ in range(3))
y = ops.x3_linear(x3, w3, b3, act=1)
torch.cuda.synchronize()
print(f"{tag:8s} {'swin s3 fc1+gelu (f32 in)':28s} {t:8.1f} us  {6.0 * M3 * C3 * 4 * C3 / t / 1e9:.2f} PF  "
      f"checksum {float(y.double().sum()):.6e}", flush=True)
