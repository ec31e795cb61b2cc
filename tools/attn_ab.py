"""Fused Swin stage-1 attention block (mmr_swin_attn_block) at B=256: time per call (HIP events,
shift 0 and 3) and max error vs the oracle (timm semantics) on 2 images.  Run once per library
(MMR_LIBMMR) for an A/B.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402
from oracle import towers as otw  # noqa: E402


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


bf = lambda t: t.to(torch.bfloat16)  # noqa: E731
g = torch.Generator().manual_seed(7)
C, H, heads, ws, B = 96, 56, 3, 7, 256
sd = {"b.norm1.weight": 1 + 0.1 * torch.randn(C, generator=g), "b.norm1.bias": 0.1 * torch.randn(C, generator=g),
      "b.attn.qkv.weight": bf(torch.randn(3 * C, C, generator=g) * C ** -0.5).float(),
      "b.attn.qkv.bias": 0.1 * torch.randn(3 * C, generator=g),
      "b.attn.proj.weight": bf(torch.randn(C, C, generator=g) * C ** -0.5).float(),
      "b.attn.proj.bias": 0.1 * torch.randn(C, generator=g),
      "b.attn.relative_position_bias_table": torch.randn(169, heads, generator=g)}
x = bf(torch.randn(B, H, H, C, generator=g)).cuda()
d = lambda k: sd["b." + k].cuda()  # noqa: E731
pack = ops.swin_attn_block_pack(bf(d("attn.qkv.weight")), d("attn.qkv.bias"), bf(d("attn.proj.weight")),
                                d("attn.proj.bias"), d("norm1.weight"), d("norm1.bias"))
lib = os.environ.get("MMR_LIBMMR", "in-tree libmmr.so")
for shift in (0, 3):
    bias = ops.swin_attn_bias(d("attn.relative_position_bias_table"), heads, ws, H, shift)
    t = min(timeit(lambda: ops.swin_attn_block(x, pack, bias, ws, shift, 1e-5)) for _ in range(3))
    y = ops.swin_attn_block(x, pack, bias, ws, shift, 1e-5)
    ref = otw.swin_attn_half(x[:2].float().cpu(), sd, "b.", heads, ws, shift)
    err = (y[:2].float().cpu() - ref).abs().max().item() / ref.abs().max().item()
    print(f"{os.path.basename(lib)} shift={shift}: {t:7.1f} us  rel err {err:.2e}", flush=True)
