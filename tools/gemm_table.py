"""All-shape GEMM table: every distinct linear of one bench step (shapes captured from the model's
own ops.linear calls), mine (tuned variant, the production epilogue) vs torch F.linear (hipBLASLt,
plain GEMM without bias/act/residual — a lower bound on what the library needs for the same op),
timed in one process with HIP events.  Diagnostic only.
usage: python tools/gemm_table.py [--model-type multimodal|text] [--batch 256] [--out file]"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import _lib, ops, synthetic  # noqa: E402
from mmr_amd.model import build_bench_model  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
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
    p = argparse.ArgumentParser()
    p.add_argument("--model-type", default="multimodal")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    model = build_bench_model(device=dev, joint_dim=768, model_type=a.model_type)
    B = a.batch
    imgs = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, synthetic.SEED))).to(dev)
    ids_np, mask_np = synthetic.reports(B, 128, synthetic.SEED + 100)
    ids, mask = torch.from_numpy(ids_np).to(dev), torch.from_numpy(mask_np).to(dev)
    shapes = collections.Counter()
    orig = ops.linear

    def rec(x, w, bias=None, residual=None, act=0, *args, **kw):
        K = x.shape[-1]
        shapes[(x.numel() // K, w.shape[0], K, int(act), bias is not None, residual is not None)] += 1
        return orig(x, w, bias, residual, act, *args, **kw)
    ops.linear = rec
    model.query_embeddings(imgs if a.model_type != "text" else None, ids, mask)
    torch.cuda.synchronize()
    ops.linear = orig
    lines = [f"{'M':>7s} {'N':>5s} {'K':>5s} epi   calls  mine_us   TF/s  blas_us   TF/s  mine/blas  variant"]
    tm = tb = 0.0
    for (M, N, K, act, hb, hr), c in sorted(shapes.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1]):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        b = torch.randn(N, device=dev) if hb else None
        r = torch.randn(M, N, device=dev, dtype=torch.bfloat16) if hr else None
        us = timeit(lambda: ops.linear(x, w, b, r, act=act))
        ub = timeit(lambda: F.linear(x, w))
        v = _lib.lib().mmr_linear_bf16_variant(M, N, K, act, int(hb), int(hr))
        fl = 2.0 * M * N * K
        epi = ("b" if hb else "") + ("g" if act else "") + ("r" if hr else "")
        lines.append(f"{M:7d} {N:5d} {K:5d} {epi:4s} {c:6d} {us:8.1f} {fl / us / 1e6:6.0f} {ub:8.1f} {fl / ub / 1e6:6.0f}"
                     f"  {us / ub:8.2f}  {v}")
        tm += us * c
        tb += ub * c
        print(lines[-1], flush=True)
        del x, w, b, r
    lines.append(f"per step: mine {tm / 1e3:.3f} ms, hipBLASLt plain {tb / 1e3:.3f} ms ({tm / tb:.2f}x)")
    print(lines[-1])
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
