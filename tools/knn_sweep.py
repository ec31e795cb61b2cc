"""In-process kNN search timing sweep (one process, interleaved variants, HIP events on the launch
stream).  usage: python tools/knn_sweep.py [--n 100000] [--d 768] [--k 10] [--qs 1,16,64,128,256,1024]
Variants: f16 (the fp16 scan the index dispatches for each Q), x3.  Prints one JSON line per (variant, Q) with the median us per search and the fraction of
the search's HBM / MFMA bound; checks that every variant returns the same lists."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import synthetic  # noqa: E402
from mmr_amd.retrieval import GalleryIndex, check_status  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--qs", default="1,16,64,128,256,1024")
    p.add_argument("--reps", type=int, default=30)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--variants", default="f16,x3")
    a = p.parse_args()
    G = synthetic.gauss_gallery(a.n, a.d, synthetic.SEED)
    ix = GalleryIndex(G, mode="f16")
    ix.reserve(max(int(q) for q in a.qs.split(",")))
    st = torch.cuda.current_stream()
    res = {}
    for q in [int(x) for x in a.qs.split(",")]:
        Q = torch.from_numpy(synthetic.gauss_gallery(q, a.d, synthetic.SEED + 1)).cuda()
        ref = None
        times = {v: [] for v in a.variants.split(",")}
        for _ in range(a.rounds):
            for v in times:
                ix.set_mode("x3" if v.startswith("x3") else "f16")
                for _ in range(3):
                    i, s, stt = ix.search(Q, a.k, want_status=True)
                torch.cuda.synchronize()
                check_status(stt)
                if ref is None:
                    ref = i.clone()
                elif not torch.equal(ref, i):
                    raise SystemExit(f"variant {v} Q={q}: lists differ from the first variant")
                evs = []
                for _ in range(a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    ix.search(Q, a.k)
                    e1.record(st)
                    evs.append((e0, e1))
                torch.cuda.synchronize()
                times[v] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
        for v, ts in times.items():
            ts.sort()
            us = ts[len(ts) // 2]
            gb = 4 if v.startswith("x3") else 2
            byts = a.n * a.d * gb + a.n * 4 + q * a.d * 4 + q * a.k * 12
            fl = 2.0 * q * a.n * a.d * (3 if v.startswith("x3") else 1)
            bound = max(byts / 8e12, fl / 2.5e15 if not (v.startswith("x3") and q <= 32) else 0.0)
            res[(v, q)] = us
            print(json.dumps({"variant": v, "q": q, "n": a.n, "d": a.d, "k": a.k, "us_median": round(us, 2),
                              "us_min": round(ts[0], 2), "bound_us": round(bound * 1e6, 2),
                              "frac_of_bound": round(bound * 1e6 / us, 3),
                              "gpairs_s": round(q * a.n / (us * 1e-6) / 1e9, 1)}), flush=True)
    ix.close()


if __name__ == "__main__":
    main()
