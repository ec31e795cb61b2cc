"""A/B of an env-selected variant of the 8-phase GEMM (e.g. MMR_P8_EPI=0/1) on the tower shapes:
interleaved rounds in one process, random operands, every output checked against torch fp32
(bias / GELU / residual epilogues).  Diagnostic.
usage: python tools/gemm_ab.py --env MMR_P8_EPI --values 0,1 [--big 7,8] [--fp8]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

SHAPES = [(32768, 3072, 768, "bg"), (32768, 2304, 768, "b"), (32768, 768, 3072, "b"), (32768, 768, 768, "b"),
          (32768, 768, 768, "br"), (50176, 1536, 384, "bg"), (50176, 384, 1536, "br"), (12544, 3072, 768, "bg")]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="MMR_P8_EPI")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--big", default="7,8")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    torch.manual_seed(0)
    os.environ["MMR_GEMM_W4"] = "0"
    for M, N, K, epi in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device="cuda") if "b" in epi else None
        r = torch.randn(M, N, device="cuda").to(torch.bfloat16) if "r" in epi else None
        act = 1 if "g" in epi else 0
        ref = F.linear(x[:2048].float(), w.float(), b)
        if act:
            ref = F.gelu(ref)
        if r is not None:
            ref = ref + r[:2048].float()
        res = {}
        for big in a.big.split(","):
            if N % (256 if big == "7" else 192) or K % 128 or M % 256:
                continue
            os.environ["MMR_GEMM_BIG"] = big
            for _ in range(a.rounds):
                for v in a.values.split(","):
                    os.environ[a.env] = v
                    y = ops.linear(x, w, b, r, act=act)
                    err = (y[:2048].float() - ref).abs().max().item() / ref.abs().max().item()
                    assert err < 1.5e-2, (M, N, K, epi, big, v, err)
                    res.setdefault((big, v), []).append(timeit(lambda: ops.linear(x, w, b, r, act=act)))
        fl = 2.0 * M * N * K
        print(f"M={M} N={N} K={K} {epi}: " + "  ".join(
            f"p8_{'256' if k[0] == '7' else '192'}/{a.env}={k[1]} {min(v):.1f}us {fl / min(v) / 1e6:.0f}TF"
            for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
