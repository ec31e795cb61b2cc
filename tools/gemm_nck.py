"""A/B of the 8-phase GEMM's tile order (MMR_P8_NCK: 0 = row-major, c = n-chunks of c W panels per
XCD, unset = the launcher's model) on the BERT shapes, interleaved rounds in one process, random
operands, each output checked against torch fp32.  Diagnostic.  usage: python tools/gemm_nck.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops  # noqa: E402

SHAPES = [(32768, 3072, 768, 1), (32768, 2304, 768, 0), (32768, 768, 3072, 0), (32768, 768, 768, 0),
          (262144, 3072, 768, 1), (131072, 2304, 768, 0)]
NCKS = ["0", "auto", "2", "3", "4", "6"]


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
    torch.manual_seed(0)
    os.environ["MMR_GEMM_W4"] = "0"
    for M, N, K, act in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        ref = F.linear(x[:4096].float(), w.float(), b)
        if act:
            ref = F.gelu(ref)
        res = {}
        for big in ("7", "8"):
            if N % (256 if big == "7" else 192):
                continue
            os.environ["MMR_GEMM_BIG"] = big
            for _ in range(3):
                for c in NCKS:
                    if c == "auto":
                        os.environ.pop("MMR_P8_NCK", None)
                    else:
                        os.environ["MMR_P8_NCK"] = c
                    y = ops.linear(x, w, b, act=act)
                    err = (y[:4096].float() - ref).abs().max().item() / ref.abs().max().item()
                    assert err < 2e-2, (M, N, K, big, c, err)
                    res.setdefault((big, c), []).append(timeit(lambda: ops.linear(x, w, b, act=act)))
        fl = 2.0 * M * N * K
        print(f"M={M} N={N} K={K} act={act}: " + "  ".join(
            f"p8_{'256' if k[0] == '7' else '192'}/nck={k[1]} {min(v):.1f}us {fl / min(v) / 1e6:.0f}TF"
            for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
