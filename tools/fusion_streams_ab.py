"""Whole cfg2 step (B = 256, bf16 and x3 towers) with the fusion stack's patch-side layer work on a side
stream or not (FusionStack.side_streams), interleaved on one box: ms per step over 10 steps after warm-up.
Diagnostic only: python tools/fusion_streams_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.model import build_bench_model  # noqa: E402

dev = torch.device("cuda:0")
B = 256
img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 71))).to(dev)
ids, mask = (torch.from_numpy(a).to(dev) for a in synthetic.reports(B, 128, 72))
for dt in ("bf16", "x3"):
    m = build_bench_model(device=dev, joint_dim=768, model_type="multimodal", tower_dtype=dt)
    for _ in range(3):
        m.query_embeddings(img, ids, mask)
    torch.cuda.synchronize()
    res = {False: [], True: []}
    for rep in range(3):
        for ns in (False, True):
            m.fusion.side_streams = ns
            m.query_embeddings(img, ids, mask)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                m.query_embeddings(img, ids, mask)
            torch.cuda.synchronize()
            res[ns].append((time.perf_counter() - t0) / 10 * 1e3)
    print(dt, "one stream:", " ".join(f"{v:.3f}" for v in res[False]), " | patch side stream:",
          " ".join(f"{v:.3f}" for v in res[True]), "ms per step", flush=True)
    del m
    torch.cuda.empty_cache()
