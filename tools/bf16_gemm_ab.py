"""The four BERT bf16 GEMMs of the cfg2 step as the LayerNorm-folded layer launches them (mmr_linear_bf16_ln:
QKV ln_mode 1, O-proj ln_mode 2 + statistics, FFN1 ln_mode 1 + GELU, FFN2 ln_mode 2 + statistics), M = 32768,
for whichever libmmr MMR_LIBMMR selects: time per launch (HIP events, min of 3 x 10) and the fraction of 2.5 PF.
usage: python tools/bf16_gemm_ab.py <tag>"""
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


tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
g = torch.Generator(device="cuda").manual_seed(5)
M, C, F4 = 32768, 768, 3072


def bf(*shape, s=1.0):
    return (torch.randn(*shape, device="cuda", generator=g) * s).to(torch.bfloat16)


x, r = bf(M, C), bf(M, C)
f1 = bf(M, F4)
wq, wo, wi, wf = bf(3 * C, C, s=0.02), bf(C, C, s=0.02), bf(F4, C, s=0.02), bf(C, F4, s=0.02)
bq, bo, bi, bff = (torch.randn(n, device="cuda", generator=g) * 0.02 for n in (3 * C, C, F4, C))
coef = torch.stack([torch.rand(M, device="cuda", generator=g) + 0.5, torch.randn(M, device="cuda", generator=g)], 1)
vq, vi = torch.randn(3 * C, device="cuda", generator=g), torch.randn(F4, device="cuda", generator=g)
gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
cases = [("qkv", lambda: ops.linear_ln(x, wq, bq, ln_mode=1, coef=coef, v1=vq), 2 * M * 3 * C * C),
         ("o", lambda: ops.linear_ln(x, wo, bo, residual=r, ln_mode=2, coef=coef, v1=gam, v2=bet, want_stats=True),
          2 * M * C * C),
         ("ffn1", lambda: ops.linear_ln(x, wi, bi, act=1, ln_mode=1, coef=coef, v1=vi), 2 * M * F4 * C),
         ("ffn2", lambda: ops.linear_ln(f1, wf, bff, residual=r, ln_mode=2, coef=coef, v1=gam, v2=bet, want_stats=True),
          2 * M * C * F4)]
for name, fn, fl in cases:
    t = min(timeit(fn) for _ in range(3))
    print(f"{tag:8s} {name:6s} {t:8.1f} us  {fl / t / 1e6:7.1f} TF  {fl / t / 1e6 / 2500:.3f} of 2.5 PF", flush=True)
