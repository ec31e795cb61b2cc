"""Timing of the x3 Swin row-linears at the Swin-T stage-2 shapes (B = 256: 200704 tokens, C = 192): norm1 + qkv
(N = 576, f32 out) and proj + residual (N = 192) from split rows, HIP events over several launches.  Diagnostic
only (an A/B of builds goes through tools/ab_variants.sh).
usage: python tools/x3_rowlin_ab.py [B]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402


def timeit(fn, iters=10):
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


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    c, hw = 192, 28
    g = torch.Generator().manual_seed(3)
    dev = "cuda"
    x = torch.randn(B, hw, hw, c, generator=g).to(dev)
    lg, lb = (1 + 0.1 * torch.randn(c, generator=g)).to(dev), (0.1 * torch.randn(c, generator=g)).to(dev)
    wq, bq = (torch.randn(3 * c, c, generator=g) * c ** -0.5).to(dev), (0.1 * torch.randn(3 * c, generator=g)).to(dev)
    wp, bp = (torch.randn(c, c, generator=g) * c ** -0.5).to(dev), (0.1 * torch.randn(c, generator=g)).to(dev)
    qp, pp = ops.x3_rowlin_pack(wq), ops.x3_rowlin_pack(wp)
    xr = ops.x3_ln_split(x, lg, lb, 1e-5)
    yq = ops.x3_rowlin(x, qp, bq, 3 * c, ln=(lg, lb, 1e-5))
    yp = ops.x3_rowlin(xr, pp, bp, c, residual=x)
    res = {"qkv_us": [], "proj_us": []}
    for _ in range(3):
        res["qkv_us"].append(round(timeit(lambda: ops.x3_rowlin(x, qp, bq, 3 * c, ln=(lg, lb, 1e-5))), 1))
        res["proj_us"].append(round(timeit(lambda: ops.x3_rowlin(xr, pp, bp, c, residual=x)), 1))
    res["qkv_sum"] = float(yq.double().abs().sum())
    res["proj_sum"] = float(yp.double().abs().sum())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
