"""LayerNorm kernels on the tower shapes under lanes-per-row overrides (MMR_LN_LPR; diagnostic).
usage: python tools/ln_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402


def timeit(fn, iters=30):
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


for rows, c, add in ((32768, 768, True), (200704, 192, False), (50176, 384, False), (12544, 768, False),
                     (32768, 768, False)):
    x = torch.randn(rows, c, device="cuda").to(torch.bfloat16)
    r = torch.randn(rows, c, device="cuda").to(torch.bfloat16)
    g, b = torch.randn(c, device="cuda"), torch.randn(c, device="cuda")
    byts = rows * c * 2 * (3 if add else 2)
    out = []
    for lpr in (None, 8, 16, 32, 64):
        if lpr is None:
            os.environ.pop("MMR_LN_LPR", None)
        else:
            if (c // 8) % lpr:
                continue
            os.environ["MMR_LN_LPR"] = str(lpr)
        f = (lambda: ops.add_layernorm(x, r, g, b, 1e-12)) if add else (lambda: ops.layernorm(x, g, b, 1e-5))
        t = timeit(f)
        out.append(f"lpr={lpr or 'rule'}: {t:6.1f} us {byts / t / 1e6:5.2f} TB/s")
    print(f"rows={rows} c={c} add={int(add)}: " + " | ".join(out), flush=True)
