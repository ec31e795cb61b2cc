"""Config 5's Swin tower with MX-fp8 linears in stages 3-4 only (the cfg5 default) vs stages 2-4 (stage 2's
qkv / proj / fc1 / fc2 and its PatchMerging reduction on the unfused fp8 GEMM path instead of the fused
bf16 kernels), at B = 2048 (cfg5's batch) and B = 256: tower time per call (HIP events, 10 calls after 3
warm-ups) and the embedding cosine of each variant against the f64-checked bf16 tower.  Stage 1
(C = 96: N = 96 / 288 / 384) does not tile into the fp8 GEMM's 192 / 256-wide weight panels.
Diagnostic only: python tools/swin_fp8_stage_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.towers import SWIN_T, SwinTower, init_swin_state  # noqa: E402

dev = torch.device("cuda:0")
sd = init_swin_state(SWIN_T, 2709)
towers = {name: SwinTower(sd, SWIN_T, dev, fp8_stages=st)
          for name, st in (("bf16", ()), ("fp8 stages 3-4", (2, 3)), ("fp8 stages 2-4", (1, 2, 3)))}


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
    return e0.elapsed_time(e1) / iters


for B in (256, 2048):
    img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 71))).to(dev)
    with torch.no_grad():
        ref = towers["bf16"].forward_features(img).float().reshape(B, -1)
        for name, tw in towers.items():
            ms = timeit(lambda: tw.forward_features(img))
            y = tw.forward_features(img).float().reshape(B, -1)
            cos = torch.nn.functional.cosine_similarity(y, ref, dim=1).min().item()
            print(f"B={B:5d} {name:16s} {ms:8.3f} ms per tower call   min cosine vs bf16 tower {cos:.5f}", flush=True)
