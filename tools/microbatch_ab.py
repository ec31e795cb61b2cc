"""Micro-batch tower pipelining probe: the cfg2 step (B = 256) with each tower's batch split into two
halves on two streams (the halves' kernels interleave: one half's HBM-bound attention / LayerNorm
beside the other's MFMA-bound GEMMs), vs the whole batch per tower.  bf16 and x3 towers, interleaved on
one box; also checks the split embeddings are bitwise equal to the unsplit ones.
Diagnostic only: python tools/microbatch_ab.py"""
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
streams = {}


def stream2(key):
    if key not in streams:
        streams[key] = torch.cuda.Stream(dev)
    return streams[key]


def split2(fn, key):
    def run(*args, **kw):
        h = args[0].shape[0] // 2
        main = torch.cuda.current_stream(dev)
        s2 = stream2(key)
        s2.wait_stream(main)
        a = fn(*(x[:h] if torch.is_tensor(x) else x for x in args), **kw)
        with torch.cuda.stream(s2):
            b = fn(*(x[h:] if torch.is_tensor(x) else x for x in args), **kw)
        main.wait_stream(s2)
        if torch.is_tensor(a):
            b.record_stream(main)
            return torch.cat([a, b], 0)
        out = []
        for u, v in zip(a, b):
            if u is None:
                out.append(None)
            else:
                v.record_stream(main)
                out.append(torch.cat([u, v], 0))
        return tuple(out)
    return run


for dt in ("bf16", "x3"):
    m = build_bench_model(device=dev, joint_dim=768, model_type="multimodal", tower_dtype=dt)
    bb = m.backbones
    enc_t, enc_i = bb.encode_text, bb.encode_image
    variants = {"whole": (enc_t, enc_i), "text split": (split2(enc_t, "t"), enc_i),
                "image split": (enc_t, split2(enc_i, "i")), "both split": (split2(enc_t, "t"), split2(enc_i, "i"))}
    for _ in range(3):
        ref = m.query_embeddings(img, ids, mask).clone()
    res = {k: [] for k in variants}
    same = {}
    for rep in range(3):
        for name, (ft, fi) in variants.items():
            bb.encode_text, bb.encode_image = ft, fi
            q = m.query_embeddings(img, ids, mask)
            torch.cuda.synchronize()
            same[name] = bool(torch.equal(q, ref))
            t0 = time.perf_counter()
            for _ in range(8):
                m.query_embeddings(img, ids, mask)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / 8 * 1e3)
    bb.encode_text, bb.encode_image = enc_t, enc_i
    for name in variants:
        print(f"{dt:4s} {name:12s} " + " ".join(f"{v:.3f}" for v in res[name]) + f" ms per step   bitwise equal {same[name]}",
              flush=True)
    del m
    torch.cuda.empty_cache()
