"""LayerNorm-fused BERT GEMMs (ops.linear_ln) vs the plain GEMMs they replace, per feature, at the
cfg2 shapes (M = 32768): HIP-event time per launch, best of 3 x 20.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402
from mmr_amd.towers import _ln_fold  # noqa: E402


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it * 1e3)
    return best


M, C = 32768, 768
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: torch.randn(*s, generator=g, device="cuda")  # noqa: E731
bf = lambda t: t.to(torch.bfloat16)  # noqa: E731
ctx, h = bf(rnd(M, C)), bf(rnd(M, C) * 3)
wo, bo = bf(rnd(C, C) * C ** -0.5), rnd(C)
_, st = ops.linear_ln(ctx, wo, bo, residual=h, want_stats=True)
cf = ops.ln_row_coef(st, C, 1e-12)
gam, bet = 1 + 0.1 * rnd(C), 0.1 * rnd(C)
rows = []
# O-proj family (N = 768, K = 768) and FFN2 family (K = 3072)
for name, K in (("o", 768), ("ffn2", 3072)):
    x = bf(rnd(M, K))
    w, b = bf(rnd(C, K) * K ** -0.5), rnd(C)
    rows.append((f"{name} plain tuned (+res)", timeit(lambda: ops.linear(x, w, b, residual=h))))
    with ops.pinned(ops.PIN_GEMM_BF16, 10):
        rows.append((f"{name} plain p8 256x192 (no res)", timeit(lambda: ops.linear(x, w, b))))
        rows.append((f"{name} plain p8 256x192 (+res)", timeit(lambda: ops.linear(x, w, b, residual=h))))
    rows.append((f"{name} mode0 +res +stats", timeit(lambda: ops.linear_ln(x, w, b, residual=h, want_stats=True))))
    rows.append((f"{name} mode2 (LN res)", timeit(lambda: ops.linear_ln(x, w, b, residual=h, ln_mode=2, coef=cf,
                                                                          v1=gam, v2=bet))))
    rows.append((f"{name} mode2 +stats", timeit(lambda: ops.linear_ln(x, w, b, residual=h, ln_mode=2, coef=cf, v1=gam,
                                                                        v2=bet, want_stats=True))))
rows.append(("add_layernorm 768", timeit(lambda: ops.add_layernorm(ctx, h, gam, bet, 1e-12))))
rows.append(("ln_row_coef", timeit(lambda: ops.ln_row_coef(st, C, 1e-12))))
# fold consumers: QKV (2304), FFN1 (3072 + GELU)
for name, N, act in (("qkv", 2304, 0), ("ffn1", 3072, 1)):
    w, b = bf(rnd(N, C) * C ** -0.5), rnd(N)
    wf, c, d = _ln_fold(w, b, gam, bet)
    rows.append((f"{name} plain tuned", timeit(lambda: ops.linear(h, w, b, act=act))))
    rows.append((f"{name} mode1 fold", timeit(lambda: ops.linear_ln(h, wf, d, act=act, ln_mode=1, coef=cf, v1=c))))
for k, v in rows:
    print(f"{k:32s} {v:8.1f} us", flush=True)
