"""Batch pipelining probe: the cfg2 serving step (query_embeddings + exact top-10 search, B = 256) issued
on one stream vs alternating over two streams (consecutive batches independent: one batch's fusion
tail / search beside the next batch's towers), bf16 and x3 towers, interleaved on one box; every
batch's results are checked against the one-stream ones.  Diagnostic only: python tools/pipeline_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.model import build_bench_model  # noqa: E402
from mmr_amd.retrieval import GalleryIndex  # noqa: E402

dev = torch.device("cuda:0")
B, K, steps = 256, 10, 12
img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 71))).to(dev)
ids, mask = (torch.from_numpy(a).to(dev) for a in synthetic.reports(B, 128, 72))
index = GalleryIndex(synthetic.gauss_gallery(100_000, 768, synthetic.SEED), device=0, mode="f16")
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]


def run(m, ns):
    outs = []
    main = torch.cuda.current_stream(dev)
    for s in streams[1:ns]:
        s.wait_stream(main)
    for i in range(steps):
        st = streams[i % ns]
        with torch.cuda.stream(st):
            q = m.query_embeddings(img, ids, mask)
            outs.append(index.search(q, K)[0])
    for s in streams[1:ns]:
        main.wait_stream(s)
    return outs


for dt in ("bf16", "x3"):
    m = build_bench_model(device=dev, joint_dim=768, model_type="multimodal", tower_dtype=dt)
    for ns in (1, 2):
        run(m, ns)
    torch.cuda.synchronize()
    ref = run(m, 1)[-1].clone()
    res = {1: [], 2: []}
    ok = True
    for rep in range(3):
        for ns in (1, 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            outs = run(m, ns)
            torch.cuda.synchronize()
            res[ns].append((time.perf_counter() - t0) / steps * 1e3)
            ok = ok and all(torch.equal(o, ref) for o in outs)
    print(f"{dt:4s} one stream " + " ".join(f"{v:.3f}" for v in res[1]) + " | two streams " +
          " ".join(f"{v:.3f}" for v in res[2]) + f" ms per step   identical top-10 every batch: {ok}", flush=True)
    del m
    torch.cuda.empty_cache()
