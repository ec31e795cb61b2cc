"""The x3 (parity) cfg2 step's query embeddings (B = 256, Swin-T + BERT-base + the fusion head) with the Swin tower
and the fusion stack's patch-side work on side streams (the default) vs in sequence, alternated over rounds on one
box, host-timed like bench.py's x3 line.  Diagnostic only.
usage: python tools/x3_overlap_ab.py [B] [rounds]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.model import build_bench_model  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = "cuda"
    m = build_bench_model(device=dev, joint_dim=768, model_type="multimodal", tower_dtype="x3")
    imgs = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 1))).to(dev)
    ids, mask = (torch.from_numpy(a).to(dev) for a in synthetic.reports(B, 128, 2))
    out = {}
    for _ in range(rounds):
        for on in (True, False):
            m.concurrent_towers = on
            if getattr(m, "fusion", None) is not None:
                m.fusion.side_streams = on
            m.query_embeddings(imgs, ids, mask)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                q = m.query_embeddings(imgs, ids, mask)
            torch.cuda.synchronize()
            out.setdefault("overlap" if on else "sequential", []).append(round((time.perf_counter() - t0) / 5 * 1e3, 2))
            out.setdefault("sum_" + ("overlap" if on else "sequential"), float(q.double().abs().sum()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
