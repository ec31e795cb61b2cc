"""x3 (parity-grade) kernels at the cfg2 step's shapes (B = 256), for rocprofv3 --pmc passes: each op runs
REPS times in the fixed PLAN order below, so tools/pmc_x3_summary.py can label dispatches by order (BERT
O-proj and FFN2 share one instantiation).  Random operands of the towers' scales.  Diagnostic only.
usage: python tools/pmc_x3.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402

REPS = 3
# (label, kernel-name substring, dispatches per rep, algorithmic work) — work: ("mfma", bf16 MFMA flops) or
# ("hbm", bytes) per dispatch
M, C, F4, H = 32768, 768, 3072, 12
PLAN = [
    ("bert_qkv", "gemm_bf16_tn_p8<3, 0, true, false", 1, ("mfma", 3 * 2 * M * 3 * C * C)),
    ("bert_oproj", "gemm_bf16_tn_p8<3, 0, true, true", 1, ("mfma", 3 * 2 * M * C * C)),
    ("bert_ffn1", "gemm_bf16_tn_p8<3, 1, true, false", 1, ("mfma", 3 * 2 * M * F4 * C)),
    ("bert_ffn2", "gemm_bf16_tn_p8<3, 0, true, true", 1, ("mfma", 3 * 2 * M * F4 * C)),
    ("bert_ln_split", "ln_rows_split<6>", 1, ("hbm", M * C * (4 + 4 + 4 + 4))),  # x + r in, f32 + split out
    ("bert_mha", "x3_mha<2, 1", 1, ("mfma", 3 * 2 * 2 * 256 * H * 128 * 128 * 64)),
    ("swin1_attn", "x3_mha<1, 2", 1, ("mfma", 3 * 2 * 2 * 256 * 64 * 3 * 49 * 49 * 32)),
    ("swin1_mlp", "x3_swin_mlp<96", 1, ("mfma", 3 * 2 * 2 * 256 * 3136 * 96 * 384)),
    # the fused stage-1 attention half: 576 v_mfma_f32_32x32x16_bf16 per 64-token (padded) window
    ("swin1_attn_block", "x3_swin_attn_block", 1, ("mfma", 576 * 32768 * 256 * 64)),
]


def main():
    g = torch.Generator().manual_seed(6)
    dev = "cuda"
    x = torch.randn(M, C, generator=g).to(dev)
    r = torch.randn(M, C, generator=g).to(dev)
    gm, bt = (1 + 0.1 * torch.randn(C, generator=g)).to(dev), (0.1 * torch.randn(C, generator=g)).to(dev)
    wq = ops.X3W((torch.randn(3 * C, C, generator=g) * 0.02).to(dev))
    bq = (0.02 * torch.randn(3 * C, generator=g)).to(dev)
    wo = ops.X3W((torch.randn(C, C, generator=g) * 0.02).to(dev))
    bo = (0.02 * torch.randn(C, generator=g)).to(dev)
    w1 = ops.X3W((torch.randn(F4, C, generator=g) * 0.02).to(dev))
    b1 = (0.02 * torch.randn(F4, generator=g)).to(dev)
    w2 = ops.X3W((torch.randn(C, F4, generator=g) * 0.02).to(dev))
    b2 = (0.02 * torch.randn(C, generator=g)).to(dev)
    xr = ops.x3_ln_split(x, gm, bt, 1e-12)
    qkv = torch.randn(M, 3 * C, generator=g).to(dev)
    mask = torch.ones(256, 128, dtype=torch.int64, device=dev)
    ar = ops.x3_attention_split(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], 256, 128, 128, H, 64, 0.125, mask=mask)
    hl = torch.empty((M, 2 * F4), dtype=torch.bfloat16, device=dev)
    from mmr_amd import _lib
    L = _lib.lib()
    # Swin stage 1 at B = 256: 56 x 56 x 96 tokens, 3 heads, shifted windows
    hw, c1, h1 = 56, 96, 3
    table = (torch.randn(13 * 13, h1, generator=g) * 0.5).to(dev)
    sbias = ops.swin_attn_bias(table, h1, 7, hw, 3)
    sqkv = torch.randn(256, hw, hw, 3 * c1, generator=g).to(dev)
    st = torch.randn(256, hw, hw, c1, generator=g).to(dev)
    sg, sb = (1 + 0.1 * torch.randn(c1, generator=g)).to(dev), (0.1 * torch.randn(c1, generator=g)).to(dev)
    sw1 = (torch.randn(4 * c1, c1, generator=g) * 0.02).to(dev)
    sw2 = (torch.randn(c1, 4 * c1, generator=g) * 0.02).to(dev)
    sb1, sb2 = (0.02 * torch.randn(4 * c1, generator=g)).to(dev), (0.02 * torch.randn(c1, generator=g)).to(dev)
    pack = ops.x3_swin_mlp_pack(sw1, sw2)
    swq, sbq = (torch.randn(3 * c1, c1, generator=g) * c1 ** -0.5).to(dev), (0.1 * torch.randn(3 * c1, generator=g)).to(dev)
    swp, sbp = (torch.randn(c1, c1, generator=g) * c1 ** -0.5).to(dev), (0.1 * torch.randn(c1, generator=g)).to(dev)
    sab = ops.x3_swin_attn_block_pack(swq, sbq, swp, sbp, sg, sb)
    torch.cuda.synchronize()

    def ffn1():
        ops._chk(L.mmr_x3_linear_p8(_lib.ptr(xr.t), _lib.ptr(w1.w2(xr.kp, F4)), _lib.ptr(b1), None, _lib.ptr(hl), M, F4,
                                    C, 1, 1, _lib.stream_ptr()), "ffn1")

    ops_ = {
        "bert_qkv": lambda: ops.x3_linear(xr, wq, bq),
        "bert_oproj": lambda: ops.x3_linear(ar, wo, bo, residual=r),
        "bert_ffn1": ffn1,
        "bert_ffn2": lambda: ops.x3_linear(ops.X3Rows(hl, F4, F4, (M,)), w2, b2, residual=r),
        "bert_ln_split": lambda: ops.x3_ln_split(x, gm, bt, 1e-12, residual=r, keep_f32=True),
        "bert_mha": lambda: ops.x3_attention_split(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], 256, 128, 128, H, 64,
                                                   0.125, mask=mask),
        "swin1_attn": lambda: ops.x3_swin_window_attention_split(sqkv, sbias, hw, h1, 7, 3),
        "swin1_mlp": lambda: ops.x3_swin_mlp(st, sg, sb, pack, sb1, sb2, 1e-5),
        "swin1_attn_block": lambda: ops.x3_swin_attn_block(st, sab, sbias, 7, 3, 1e-5),
    }
    for name, _, _, _ in PLAN:  # warm (variant tuners, weight images) outside the labelled dispatches
        ops_[name]()
    torch.cuda.synchronize()
    print("PLAN-START", flush=True)
    for name, _, _, _ in PLAN:
        for _ in range(REPS):
            ops_[name]()
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
