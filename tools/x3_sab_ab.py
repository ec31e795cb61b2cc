"""A/B timing of the fused x3 Swin stage-1 attention half (mmr_x3_swin_attn_block, C = 96) against the unfused
x3 chain it replaces (x3_rowlin norm1 + qkv -> x3 window attention, split rows -> x3_rowlin proj + residual) at
the Swin-T stage-1 shape (B = 256, 56 x 56 x 96), shift 0 and 3, HIP events over several launches, alternated
over rounds on one box; prints the max relative difference of the two outputs.  Diagnostic only.
usage: python tools/x3_sab_ab.py [B] [rounds] [fused]  (fused: time the fused block only)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
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
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    fused_only = len(sys.argv) > 3 and sys.argv[3] == "fused"
    c, heads, ws, hw = 96, 3, 7, 56
    g = torch.Generator().manual_seed(7)
    dev = "cuda"
    x = (torch.randn(B, hw, hw, c, generator=g)).to(dev)
    lg, lb = (1 + 0.1 * torch.randn(c, generator=g)).to(dev), (0.1 * torch.randn(c, generator=g)).to(dev)
    wq, bq = (torch.randn(3 * c, c, generator=g) * c ** -0.5).to(dev), (0.1 * torch.randn(3 * c, generator=g)).to(dev)
    wp, bp = (torch.randn(c, c, generator=g) * c ** -0.5).to(dev), (0.1 * torch.randn(c, generator=g)).to(dev)
    table = (torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5).to(dev)
    pack = ops.x3_swin_attn_block_pack(wq, bq, wp, bp, lg, lb)
    qp, pp = ops.x3_rowlin_pack(wq), ops.x3_rowlin_pack(wp)
    for shift in (0, 3):
        bias = ops.swin_attn_bias(table, heads, ws, hw, shift)

        def chain():
            qkv = ops.x3_rowlin(x, qp, bq, 3 * c, ln=(lg, lb, 1e-5))
            a = ops.x3_swin_window_attention_split(qkv, bias, hw, heads, ws, shift)
            return ops.x3_rowlin(a, pp, bp, c, residual=x)

        def fused():
            return ops.x3_swin_attn_block(x, pack, bias, ws, shift, 1e-5)

        yc, yf = chain(), fused()
        diff = ((yc - yf).abs().max() / yc.abs().max()).item()
        tc, tf = [], []
        for _ in range(rounds):
            if not fused_only:
                tc.append(timeit(chain))
            tf.append(timeit(fused))
        print(json.dumps({"B": B, "shift": shift, "chain_us": [round(t, 1) for t in tc],
                          "fused_us": [round(t, 1) for t in tf], "max_rel_diff": diff}), flush=True)


if __name__ == "__main__":
    main()
