"""Where the 8-phase GEMM's time goes: the BERT shapes (M = 32768) on the pinned p8 variants, timed
with HIP events, for whichever libmmr is loaded — run once per diagnostic build (MMR_LIBMMR):
  libmmr.so                     production
  -DMMR_P8_SAMEPANEL            every tile stages the first X / W panels (an L2-resident operand stream)
  -DMMR_P8_NOSTORE              outputs computed, not stored
  both                          the schedule's own bound (no memory-system cost beyond L2 hits)
Results of the diagnostic builds are wrong by construction.  Diagnostic only.
usage: MMR_LIBMMR=... python tools/p8_bound.py --tag NAME"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

SHAPES = [("qkv", 2304, 768, 0), ("o", 768, 768, 0), ("ffn1", 3072, 768, 1), ("ffn2", 768, 3072, 0)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it * 1e3)
    return best


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--tag", default="prod")
    a.add_argument("--m", type=int, default=32768)
    args = a.parse_args()
    torch.manual_seed(0)
    M = args.m
    for name, N, K, act in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        line = f"{args.tag:10s} {name:5s} M={M} N={N} K={K}"
        for vname, v, tbn in (("256x256", 9, 256), ("256x192", 10, 192)):
            if N % tbn:
                continue
            with ops.pinned(ops.PIN_GEMM_BF16, v):
                us = timeit(lambda: ops.linear(x, w, b, None, act=act))
            line += f" | {vname} {us:7.1f} us {2.0 * M * N * K / us / 1e6:5.0f} TF"
        print(line, flush=True)
        del x, w, b


if __name__ == "__main__":
    main()
