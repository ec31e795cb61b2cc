"""Per-shape timing of mmr_linear_bf16 vs torch F.linear (hipBLASLt) on the tower GEMM shapes.
Diagnostic only (the known-good library number is the ceiling reference, guide rule 10)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from mmr_amd import ops

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
shapes = [  # (name, M, N, K, act, residual)
    ("bert_qkv", B * 128, 2304, 768, 0, False), ("bert_o", B * 128, 768, 768, 0, False),
    ("bert_ffn1", B * 128, 3072, 768, 1, False), ("bert_ffn2", B * 128, 768, 3072, 0, False),
    ("fus_txt_qkv", B * 128, 2304, 768, 0, False), ("fus_pat_qkv", B * 49, 2304, 768, 0, False),
    ("fus_pat_o", B * 49, 768, 768, 0, False), ("fus_pf_o_res", B * 49, 768, 768, 0, True),
    ("fus_seq_qkv", B * 51, 2304, 768, 0, False),
    ("swin1_qkv", B * 3136, 288, 96, 0, False), ("swin1_fc1", B * 3136, 384, 96, 1, False),
    ("swin1_fc2", B * 3136, 96, 384, 0, True), ("swin1_proj", B * 3136, 96, 96, 0, True),
    ("swin2_qkv", B * 784, 576, 192, 0, False), ("swin2_fc1", B * 784, 768, 192, 1, False),
    ("swin2_fc2", B * 784, 192, 768, 0, True), ("swin3_qkv", B * 196, 1152, 384, 0, False),
    ("swin3_fc1", B * 196, 1536, 384, 1, False), ("swin3_fc2", B * 196, 384, 1536, 0, True),
    ("swin4_fc1", B * 49, 3072, 768, 1, False), ("patch_embed", B * 3136, 96, 64, 0, False),
    ("merge1", B * 784, 192, 384, 0, False),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


print(f"{'shape':<12} {'M':>8} {'N':>5} {'K':>5} {'mine_us':>9} {'TF/s':>7} {'hipblaslt_us':>12} {'TF/s':>7} {'ratio':>6}")
tot_m = tot_t = 0.0
for name, M, N, K, act, res in shapes:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.float32)
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if res else None
    bb = b.to(torch.bfloat16)
    tm = timeit(lambda: ops.linear(x, w, b, r, act=act))
    def tl():  # the library GEMM alone (no fused epilogue): a lower bound for hipBLASLt's time
        return F.linear(x, w, bb)
    tt = timeit(tl)
    fl = 2.0 * M * N * K
    tot_m += tm; tot_t += tt
    print(f"{name:<12} {M:>8} {N:>5} {K:>5} {tm*1e3:>9.1f} {fl/tm/1e9:>7.0f} {tt*1e3:>12.1f} {fl/tt/1e9:>7.0f} {tt/tm:>6.2f}")
print(f"total mine {tot_m:.3f} ms, torch/hipblaslt {tot_t:.3f} ms")
