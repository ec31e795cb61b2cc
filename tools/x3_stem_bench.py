"""The fused x3 Swin stem (mmr_x3_patch_embed_ln: conv4x4/s4 on bf16x3 MFMA + LayerNorm) at the cfg2 batch
(B = 256, 224 x 224): time per call (HIP events, min of 3 x 20) and the algorithmic bytes' rate (image read
154 MB + tokens written 308 MB).  Run once per library (MMR_LIBMMR) for a same-box A/B.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import _lib, ops  # noqa: E402


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


g = torch.Generator().manual_seed(3)
B = 256
img = torch.randn(B, 3, 224, 224, generator=g).cuda()
w = (torch.randn(96, 3, 4, 4, generator=g) * 0.1).cuda()
bias, gam, bet = (torch.randn(96, generator=g).cuda() for _ in range(3))
pack = ops.x3_patch_embed_pack(w)
t = min(timeit(lambda: ops.x3_patch_embed_ln(img, pack, bias, gam, bet, 1e-5)) for _ in range(3))
nbytes = img.numel() * 4 + B * 56 * 56 * 96 * 4
print(f"{os.path.basename(_lib.LIB_PATH)}: x3 stem B={B} {t:7.1f} us  {nbytes / t / 1e6:5.2f} TB/s algorithmic", flush=True)
if hasattr(_lib.lib(), "mmr_patch_embed_ln_bf16"):
    from mmr_amd.towers import SWIN_T, SwinTower, init_swin_state  # noqa: E402
    wb = w.reshape(96, 48).to(torch.bfloat16)
    pb = ops.x3_patch_embed_pack(wb.float().contiguous())
    t1 = min(timeit(lambda: ops.patch_embed_ln_bf16(img, pb, bias, gam, bet, 1e-5)) for _ in range(3))
    wp = torch.zeros(96, 64, device="cuda", dtype=torch.bfloat16)
    wp[:, :48] = wb
    t2 = min(timeit(lambda: ops.layernorm(ops.linear(ops.patch_im2col(img, 4), wp, bias), gam, bet, 1e-5))
             for _ in range(3))
    print(f"bf16 stem B={B}: fused {t1:7.1f} us | im2col + GEMM + LayerNorm {t2:7.1f} us", flush=True)
