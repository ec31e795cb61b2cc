"""Same-process comparison of GEMM kernel variants (env switches re-read per call) on the tower
shapes, with the epilogues the towers use.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from mmr_amd import ops

SHAPES = [("bert_qkv", 32768, 2304, 768, "b"), ("bert_o", 32768, 768, 768, "br"),
          ("bert_ffn1", 32768, 3072, 768, "bg"), ("bert_ffn2", 32768, 768, 3072, "br"),
          ("swin3_qkv", 50176, 1152, 384, "b"), ("swin3_proj", 50176, 384, 384, "br"),
          ("swin3_fc1", 50176, 1536, 384, "bg"), ("swin3_fc2", 50176, 384, 1536, "br"),
          ("swin2_qkv", 200704, 576, 192, "b"), ("swin2_proj", 200704, 192, 192, "br")]
VARIANTS = [("old", {"MMR_GEMM_W4": "0"}), ("w4", {"MMR_GEMM_W4": "1"}), ("w4_192", {"MMR_GEMM_W4": "2"})]


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


for name, M, N, K, epi in SHAPES:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if "r" in epi else None
    act = 1 if "g" in epi else 0
    ref = None
    out = []
    for vname, env in VARIANTS:
        os.environ.update(env)
        us = timeit(lambda: ops.linear(x, w, b, r, act=act))
        y = ops.linear(x, w, b, r, act=act).float()
        if ref is None:
            ref = y
        d = (y - ref).abs().max().item()
        out.append(f"{vname} {us:7.1f}us {2 * M * N * K / us / 1e6:5.0f}TF d={d:.1e}")
    us = timeit(lambda: F.linear(x, w))
    print(f"{name:11s} " + " | ".join(out) + f" | blas-plain {us:7.1f}us", flush=True)
