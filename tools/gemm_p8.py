"""A/B of the 8-phase GEMM (pinned variants 9 / 10) against the tuned production variant and torch
F.linear (hipBLASLt) on the tower shapes, interleaved rounds in one process, random operands; each
variant's output is checked against an fp32 torch reference of the same bf16 operands.
Diagnostic only.  usage: python tools/gemm_p8.py [--rounds 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

SHAPES = [(32768, 2304, 768, "b"), (32768, 3072, 768, "bg"), (32768, 768, 3072, "b"), (32768, 768, 768, "b"),
          (12544, 2304, 768, "b"), (50176, 1536, 384, "bg"), (50176, 384, 1536, "br"), (50176, 1152, 384, "b"),
          (12544, 768, 3072, "br"), (12544, 3072, 768, "bg"), (65280, 2304, 768, "b"), (32768, 768, 3072, "br")]
VARIANTS = [("tuned", -1), ("p8_256", 9), ("p8_192", 10)]  # mmr_pin_variant indices


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


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--rounds", type=int, default=3)
    args = a.parse_args()
    torch.manual_seed(0)
    for M, N, K, epi in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device="cuda") if "b" in epi else None
        r = torch.randn(M, N, device="cuda").to(torch.bfloat16) if "r" in epi else None
        act = 1 if "g" in epi else 0
        ref = F.linear(x.float(), w.float(), b)
        if act:
            ref = F.gelu(ref)
        if r is not None:
            ref = ref + r.float()
        res = {}
        for _ in range(args.rounds):
            for name, v in VARIANTS:
                if name != "tuned" and (N % (256 if name == "p8_256" else 192) or K % 128):
                    continue
                with ops.pinned(ops.PIN_GEMM_BF16, v):
                    us = timeit(lambda: ops.linear(x, w, b, r, act=act))
                res.setdefault(name, []).append(us)
            res.setdefault("blas", []).append(timeit(lambda: F.linear(x, w)))
        errs = {}
        for name, v in VARIANTS:
            if name not in res:
                continue
            with ops.pinned(ops.PIN_GEMM_BF16, v):
                y = ops.linear(x, w, b, r, act=act).float()
            errs[name] = ((y - ref).abs() / (ref.abs() + 1.0)).max().item()
        fl = 2.0 * M * N * K
        line = f"{M:6d} {N:5d} {K:5d} {epi:3s}"
        for name in ["tuned", "p8_256", "p8_192", "blas"]:
            if name in res:
                us = sorted(res[name])[len(res[name]) // 2]
                line += f" | {name} {us:7.1f}us {fl / us / 1e6:5.0f}TF" + (f" e={errs[name]:.1e}" if name in errs else "")
        print(line, flush=True)
        del x, w, b, r, ref


if __name__ == "__main__":
    main()
