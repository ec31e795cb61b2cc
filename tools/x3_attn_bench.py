"""x3 attention (x3_mha) on the cfg2 step's shapes: BERT B=256 x 128 with report-length masks, Swin stages
1-4 windows at B=256, the fusion stack's 8-head dh-96 calls; time per call (HIP events, min of 3 x 20).
Also the driver of tools/gpu_pmc_swin.sh (PMC_PY) for the attention counters.  Diagnostic only.
(The round-4 vs round-5 A/B it once ran is profiles/r05_x3_attn_ab.txt.)"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import _lib, ops  # noqa: E402

DEV = "cuda"
L = _lib.lib()


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def ab(name, fn):
    t = min(timeit(fn) for _ in range(3))
    print(f"{name:34s} {t:8.1f} us", flush=True)
    return t, t


g = torch.Generator().manual_seed(5)
tot_old = tot_new = 0.0
# BERT: B = 256, L = 128, 12 x 64, report-length masks (~40 % padding)
B, Lb, H, dh = 256, 128, 12, 64
qkv = (torch.randn(B * Lb, 3 * H * dh, generator=g) * 0.7).to(DEV)
lens = torch.randint(40, Lb + 1, (B,), generator=g)
mask = (torch.arange(Lb)[None, :] < lens[:, None]).to(torch.int64).to(DEV)
C = H * dh
out = torch.empty(B * Lb, C, device=DEV)
o, n = ab("bert 256x128x128 12x64 mask", lambda: (ops.x3_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, Lb, Lb,
                                                                    H, dh, dh ** -0.5, out=out, mask=mask)[0],))
tot_old += 12 * o
tot_new += 12 * n
# Swin windows, B = 256
for hw, c, heads, shift, nblk in ((56, 96, 3, 3, 2), (28, 192, 6, 3, 2), (14, 384, 12, 3, 6), (7, 768, 24, 0, 2)):
    x = (torch.randn(256, hw, hw, 3 * c, generator=g) * 0.7).to(DEV)
    table = torch.randn(169, heads, generator=g) * 0.5
    bias = ops.swin_attn_bias(table.to(DEV), heads, 7, hw, shift)
    o, n = ab(f"swin hw{hw} c{c} shift{shift}", lambda: (ops.x3_swin_window_attention(x, bias, hw, heads, 7, shift),))
    tot_old += nblk * o
    tot_new += nblk * n
    del x
# fusion stack (8 heads x 96, B = 256): enhancers 128x128 / 49x49, cross 128 q x 49 k (mean), 49 q x 128 k (out +
# mean), combiner 51 x 51 over 5 * 256 sequences (mean)
D, h, dhf = 768, 8, 96
for name, b, lq, lk, want_out, per in (("fusion txt self 128x128", 256, 128, 128, True, 5),
                                       ("fusion patch self 49x49", 256, 49, 49, True, 5),
                                       ("fusion t2i 128x49 mean", 256, 128, 49, False, 5),
                                       ("fusion i2t 49x128 out+mean", 256, 49, 128, True, 5),
                                       ("fusion combiner 51x51 mean", 1280, 51, 51, False, 1)):
    q = (torch.randn(b * lq, 3 * D, generator=g) * 0.7).to(DEV)
    kv = (torch.randn(b * lk, 3 * D, generator=g) * 0.7).to(DEV)
    out = torch.empty(b * lq, D, device=DEV) if want_out else None
    m = torch.empty(b, D, device=DEV)

    def run():
        ops.x3_attention(q[:, :D], kv[:, D:2 * D], kv[:, 2 * D:], b, lq, lk, h, dhf, 1 / math.sqrt(dhf), out=out,
                         mean_out=m)
        return (out, m) if out is not None else (m,)
    o, n = ab(name, run)
    tot_old += per * o
    tot_new += per * n
print(f"per cfg2 x3 step (weighted by call counts): {tot_new / 1e3:.2f} ms", flush=True)
