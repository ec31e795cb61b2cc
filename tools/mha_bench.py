"""Time mmr_mha on the fusion-stack shapes (diagnostic): out + mean vs mean only, and the BERT
attention kernel on its shape for comparison."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops, synthetic  # noqa: E402


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
    return e0.elapsed_time(e1) / iters * 1e3


B, h, D = int(os.environ.get("MHA_B", "256")), 8, int(os.environ.get("MHA_D", "768"))  # cfg5: MHA_D=1024 (dh 128)
dh = D // h
shapes = ((128, 128), (49, 49), (128, 49), (49, 128), (51, 51))
if len(sys.argv) > 2:  # one shape: python tools/mha_bench.py LQ LK
    shapes = ((int(sys.argv[1]), int(sys.argv[2])),)
for lq, lk in shapes:
    q = torch.randn(B * lq, 3 * D, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(B * lk, 3 * D, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(B * lq, D, device="cuda", dtype=torch.bfloat16)
    mean = torch.empty(B, D, device="cuda")
    t1 = timeit(lambda: ops.mha(q[:, :D], kv[:, D:2 * D], kv[:, 2 * D:], B, lq, lk, h, dh, 1 / math.sqrt(dh), out=out))
    t2 = timeit(lambda: ops.mha(q[:, :D], kv[:, D:2 * D], kv[:, 2 * D:], B, lq, lk, h, dh, 1 / math.sqrt(dh),
                                mean_out=mean))
    byts = (B * lq * D + 2 * B * lk * D) * 2
    print(f"lq={lq:3d} lk={lk:3d}: out {t1:7.1f} us  mean-only {t2:7.1f} us   in-bytes {byts / 1e6:.0f} MB "
          f"-> {byts / t2 / 1e6:.2f} TB/s (mean-only)", flush=True)
if len(sys.argv) > 2:
    sys.exit(0)
qkv = torch.randn(B, 128, 3 * D, device="cuda", dtype=torch.bfloat16)
for name, mask in (("all keys", torch.ones(B, 128, dtype=torch.int64, device="cuda")),
                   ("synthetic report lengths", torch.from_numpy(synthetic.reports(B, 128, synthetic.SEED + 100)[1]).cuda())):
    t = timeit(lambda: ops.bert_attention(qkv, mask, 12, 64))
    print(f"bert_attention B={B} L=128 12x64 ({name}): {t:7.1f} us")
