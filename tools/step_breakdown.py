"""Per-op time breakdown of one bench step (multimodal default): wraps the mmr_amd.ops entry points
with HIP events on the current stream and prints, per (op, shape), calls / total ms / TF/s for the
GEMMs.  Diagnostic only.
usage: python tools/step_breakdown.py [--model-type multimodal|text] [--batch B] [--dim D] [--tower-dtype bf16|fp8] [--no-ln-fold]
(the towers and fusion layers run on one stream here: per-op events are exact only then)"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import ops, synthetic  # noqa: E402
from mmr_amd.model import build_bench_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model-type", default="multimodal")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--dim", type=int, default=768)
ap.add_argument("--tower-dtype", default="bf16")
ap.add_argument("--no-ln-fold", action="store_true", help="BERT with its LayerNorm passes (unfolded)")
args = ap.parse_args()
mt = args.model_type
torch.cuda.set_device(0)
dev = torch.device("cuda:0")
model = build_bench_model(device=dev, joint_dim=args.dim, model_type=mt, tower_dtype=args.tower_dtype)
model.concurrent_towers = False
if args.no_ln_fold:
    model.backbones.bert.ln_fold = False
if model.fusion is not None:
    model.fusion.side_streams = False
B = args.batch
imgs = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, synthetic.SEED))).to(dev)
ids_np, mask_np = synthetic.reports(B, 128, synthetic.SEED + 100)
ids, mask = torch.from_numpy(ids_np).to(dev), torch.from_numpy(mask_np).to(dev)

rec = []
names = ["linear", "layernorm", "add_layernorm", "scaled_add_layernorm", "bert_embed", "bert_attention",
         "swin_window_attention", "patch_im2col", "patch_merge_ln", "swin_head", "mean_tokens", "proj_head",
         "swin_mlp", "swin_attn_block", "linear_f32", "linear_f32_batched", "mha", "add_pos", "ln_rows",
         "assemble_seq", "rows_to_f32", "quantize_mxfp8", "linear_mxfp8", "linear_mxfp8_q8", "layernorm_q8",
         "linear_rw", "linear_ln", "ln_row_coef", "linear_x3", "linear_x3_batched",
         "x3_linear", "x3_attention", "x3_swin_window_attention", "x3_patch_im2col", "x3_patch_merge_ln",
         "x3_bert_embed", "x3_add_pos", "x3_assemble_seq", "x3_mean_rows", "x3_gather_rows", "x3_ffn", "x3_ln_split", "x3_attention_split", "x3_swin_window_attention_split", "x3_patch_merge_ln_split"]
depth = [0]  # ops called from inside a wrapped op (x3_ffn's unfused route) are not counted twice


def wrap(name, fn):
    def w(*a, **k):
        if depth[0]:
            return fn(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        depth[0] += 1
        try:
            out = fn(*a, **k)
        finally:
            depth[0] -= 1
        e1.record()
        key = name
        if name == "linear_mxfp8_q8":
            key = (name, a[0].q.shape[0], a[1].q.shape[0], a[0].kp, k.get("act", 0), False)
        elif name == "linear_mxfp8":
            key = (name, a[0].q.shape[0], a[1].q.shape[0], a[0].kp, k.get("act", 0), (a[3] if len(a) > 3 else k.get("residual")) is not None)
        elif name == "quantize_mxfp8":
            key = (name, a[0].numel() // a[0].shape[-1], 0, a[0].shape[-1], 0, False)
        if name == "linear_rw":
            x, pk = a[0], a[1]
            res = (k.get("residual") if "residual" in k else (a[3] if len(a) > 3 else None)) is not None
            key = (name, x.numel() // pk.k, pk.n, pk.k, 0, res)
        if name in ("linear_ln", "linear_x3", "x3_linear"):
            x, wt = a[0], a[1]
            K = x.k if isinstance(x, ops.X3Rows) else x.shape[-1]
            n_out = wt.shape[0] if name == "linear_ln" else wt.w.shape[-2]
            key = (name, x.rows if isinstance(x, ops.X3Rows) else x.numel() // K, n_out, K, k.get("act", 0),
                   k.get("ln_mode", 0) if name == "linear_ln" else (k.get("residual") is not None or len(a) > 3 and a[3] is not None))
        if name == "x3_ffn":
            x, w1, w2 = a[0], a[1], a[3]
            K = x.k if isinstance(x, ops.X3Rows) else x.shape[-1]
            key = (name, x.rows if isinstance(x, ops.X3Rows) else x.numel() // K, w1.w.shape[0], K, 1, (k.get("residual") is not None or len(a) > 5 and a[5] is not None))
        if name in ("x3_attention", "mha", "x3_attention_split"):
            key = f"{name} b={a[3]} lq={a[4]} lk={a[5]} h={a[6]} dh={a[7]}"
        if name == "linear":
            x, wt = a[0], a[1]
            K = x.shape[-1]
            key = (name, x.numel() // K, wt.shape[0], K, k.get("act", a[4] if len(a) > 4 else 0),
                   (k.get("residual") if "residual" in k else (a[3] if len(a) > 3 else None)) is not None)
        rec.append((key, e0, e1))
        return out
    return w


for n in names:
    setattr(ops, n, wrap(n, getattr(ops, n)))
# the modules imported ops functions by module reference (ops.linear), so the wrappers are seen
for _ in range(3):
    model.query_embeddings(imgs, ids, mask)
torch.cuda.synchronize()
rec.clear()
for _ in range(3):
    model.query_embeddings(imgs, ids, mask)
torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0])
for key, e0, e1 in rec:
    agg[key][0] += 1
    agg[key][1] += e0.elapsed_time(e1) / 3
tot = sum(v[1] for v in agg.values())
print(f"total {tot:.3f} ms per step (sum of op times)")
for key, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    if isinstance(key, tuple):
        nm, M, N, K, act, res = key
        tf = 2.0 * M * N * K * (c / 3) * (2 if nm == "x3_ffn" else 1) / (t * 1e-3) / 1e12
        print(f"{t:8.3f} ms {c // 3:4d}x  {nm:14s} M={M:7d} N={N:5d} K={K:5d} act={act} res={int(res)}  {tf:6.0f} TF/s")
    else:
        print(f"{t:8.3f} ms {c // 3:4d}x  {key}")
