"""fp32-faithful tower mode (tower_dtype="x3"): Swin, BERT and the multimodal head with f32 activations
between kernels and every contraction on bf16x3 MFMA (csrc/x3.hip).

The reference runs these towers in fp32 (Backbones.swin_features -> timm forward_features,
src/Model/fusion.py:198-199; BertModel(...).last_hidden_state fusion.py:322-325; the heads and the
multimodal fusion stack model.py:365-479, fusion.py:334-471).  The bf16 / MX-fp8 modes move embeddings
by ~1e-3 cosine and reorder near-tied gallery items; this mode holds the end-to-end lists to
BASELINE.md §3 (identical top-K up to 1e-6 ties, scores within 1e-4, identical P@10).  Same weights,
same dataflow as the bf16 towers (towers.py, fusion.py), but:
  * linears: ops.x3_linear (X f32 split in registers, W pre-split once at load: ops.X3W), bias /
    GELU(erf, erff) / residual in the f32 epilogue;
  * attention: ops.x3_attention / ops.x3_swin_window_attention (q k^T and P V both bf16x3, expf softmax);
  * LayerNorm: the f32 row kernel (ops.ln_rows), PatchMerging / BERT embeddings / means: f32 kernels;
  * Swin stages 1-2 (C = 96 / 192): LayerNorm + fc1 + GELU + fc2 + residual fused (ops.x3_swin_mlp,
    csrc/x3_mlp.hip), the hidden never leaving the CU; norm1 + qkv and proj + residual as streamed
    row-linears (ops.x3_rowlin: W^T through LDS, the x split in registers, no padded GEMM tiles).
"""
import math

import torch

from . import ops
from .towers import BERT_BASE, SWIN_T


def _f(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _x3(t, dev):
    return ops.X3W(_f(t, dev))


def _ln(x, g, b, eps, residual=None, alpha=None):
    """LayerNorm(alpha * x + residual) over the last dim, f32 rows."""
    c = x.shape[-1]
    x2 = x.reshape(-1, c)
    r2 = residual.reshape(-1, c) if residual is not None else None
    return ops.ln_rows(x2, g, b, eps, alpha=alpha, residual=r2).view(x.shape)


class SwinTowerX3:
    """timm SwinTransformer.forward_features (oracle/towers.py restatement) in the x3 mode."""

    def __init__(self, sd, cfg=SWIN_T, device="cuda"):
        self.cfg = dict(SWIN_T, **cfg)
        dev = torch.device(device)
        self.device = dev
        E = self.cfg["embed_dim"]
        w = sd["patch_embed.proj.weight"].reshape(E, -1).float()
        self.kp = -(-w.shape[1] // 32) * 32
        wp = torch.zeros((E, self.kp), dtype=torch.float32)
        wp[:, :w.shape[1]] = w
        self.pe_w, self.pe_b = _x3(wp, dev), _f(sd["patch_embed.proj.bias"], dev)
        self.pe_g, self.pe_beta = _f(sd["patch_embed.norm.weight"], dev), _f(sd["patch_embed.norm.bias"], dev)
        # Swin-T's stem (3 -> 96, 4 x 4 / 4): conv + its LayerNorm in one pass (None: im2col -> GEMM -> LN)
        self.pe_pack = (ops.x3_patch_embed_pack(_f(w, dev)) if self.cfg["patch"] == 4 and w.shape == (96, 48)
                        else None)
        self.stages = []
        res = self.cfg["img_size"] // self.cfg["patch"]
        ws0 = self.cfg["window_size"]
        for i, depth in enumerate(self.cfg["depths"]):
            if i > 0:
                res //= 2
            st = {"blocks": []}
            if i > 0:
                p = f"layers.{i}.downsample."
                st["ds_g"], st["ds_b"] = _f(sd[p + "norm.weight"], dev), _f(sd[p + "norm.bias"], dev)
                st["ds_w"] = _x3(sd[p + "reduction.weight"], dev)
            ws = min(ws0, res)
            for j in range(depth):
                p = f"layers.{i}.blocks.{j}."
                shift = 0 if (j % 2 == 0 or res <= ws0) else ws0 // 2
                table = _f(sd[p + "attn.relative_position_bias_table"], dev)
                st["blocks"].append({
                    "shift": shift,
                    "bias": ops.swin_attn_bias(table, self.cfg["num_heads"][i], ws, res, shift),
                    "n1g": _f(sd[p + "norm1.weight"], dev), "n1b": _f(sd[p + "norm1.bias"], dev),
                    "qkv_w": _x3(sd[p + "attn.qkv.weight"], dev), "qkv_b": _f(sd[p + "attn.qkv.bias"], dev),
                    "proj_w": _x3(sd[p + "attn.proj.weight"], dev), "proj_b": _f(sd[p + "attn.proj.bias"], dev),
                    "n2g": _f(sd[p + "norm2.weight"], dev), "n2b": _f(sd[p + "norm2.bias"], dev),
                    "fc1_w": _x3(sd[p + "mlp.fc1.weight"], dev), "fc1_b": _f(sd[p + "mlp.fc1.bias"], dev),
                    "fc2_w": _x3(sd[p + "mlp.fc2.weight"], dev), "fc2_b": _f(sd[p + "mlp.fc2.bias"], dev),
                })
                b_ = st["blocks"][-1]
                # C = 96 / 192: the fused MLP and the streamed row-linears (norm1 + qkv, proj + residual)
                b_["mlp_pack"] = ops.x3_swin_mlp_pack(b_["fc1_w"].w, b_["fc2_w"].w)
                b_["qkv_pack"] = ops.x3_rowlin_pack(b_["qkv_w"].w)
                b_["proj_pack"] = ops.x3_rowlin_pack(b_["proj_w"].w)
                # C = 96 (stage 1): norm1 + qkv + window attention + proj + residual in one pass
                b_["sab_pack"] = (ops.x3_swin_attn_block_pack(b_["qkv_w"].w, b_["qkv_b"], b_["proj_w"].w,
                                                              b_["proj_b"], b_["n1g"], b_["n1b"])
                                  if ws == 7 and res % 7 == 0 else None)
            self.stages.append(st)
        self.norm_g, self.norm_b = _f(sd["norm.weight"], dev), _f(sd["norm.bias"], dev)
        self.num_features = E * 2 ** (len(self.cfg["depths"]) - 1)
        self.fused_mlp = True      # the fused x3 MLP where built (A/B attribute)
        self.fused_linears = True  # the streamed x3 row-linears (norm1 + qkv, proj) where built (A/B attribute)
        self.fused_attn = True     # the fused x3 attention half (C = 96) where built (A/B attribute)

    def tokens(self, image):
        """(B,3,H,W) f32 -> (B, h, w, C) f32 tokens BEFORE the final norm."""
        cfg = self.cfg
        image = image.to(self.device, torch.float32).contiguous()
        B = image.shape[0]
        g = cfg["img_size"] // cfg["patch"]
        if self.pe_pack is not None and image.shape[1] == 3 and image.shape[2] == image.shape[3] \
                and (g * g) % 32 == 0:
            x = ops.x3_patch_embed_ln(image, self.pe_pack, self.pe_b, self.pe_g, self.pe_beta, 1e-5)
        else:
            cols = ops.x3_patch_im2col(image, cfg["patch"], self.kp)
            x = ops.x3_linear(cols, self.pe_w, self.pe_b)                    # conv 4x4/s4 as a GEMM
            x = _ln(x, self.pe_g, self.pe_beta, 1e-5).view(B, g, g, -1)
        for i, st in enumerate(self.stages):
            if i > 0:
                x = ops.x3_linear(ops.x3_patch_merge_ln_split(x, st["ds_g"], st["ds_b"], 1e-5), st["ds_w"])
            H = x.shape[1]
            heads = cfg["num_heads"][i]
            ws = min(cfg["window_size"], H)
            for bk in st["blocks"]:
                x = self._attn_half(x, bk, H, heads, ws)
                if self.fused_mlp and bk["mlp_pack"] is not None:
                    x = ops.x3_swin_mlp(x, bk["n2g"], bk["n2b"], bk["mlp_pack"], bk["fc1_b"], bk["fc2_b"], 1e-5)
                else:
                    h = ops.x3_ln_split(x, bk["n2g"], bk["n2b"], 1e-5)
                    x = ops.x3_ffn(h, bk["fc1_w"], bk["fc1_b"], bk["fc2_w"], bk["fc2_b"], residual=x)
        return x

    def _attn_half(self, x, bk, H, heads, ws):
        """x + proj(W-MSA(norm1(x))) of one block: fused in one pass at C = 96 (x3_swin_attn_block), else
        the streamed row-linears around the window attention (split rows in between), else split GEMMs."""
        C = x.shape[-1]
        if self.fused_attn and bk["sab_pack"] is not None and ws == 7:
            return ops.x3_swin_attn_block(x, bk["sab_pack"], bk["bias"], ws, bk["shift"], 1e-5)
        rowlin = self.fused_linears and bk["qkv_pack"] is not None
        if rowlin:
            qkv = ops.x3_rowlin(x, bk["qkv_pack"], bk["qkv_b"], 3 * C, ln=(bk["n1g"], bk["n1b"], 1e-5))
        else:
            h = ops.x3_ln_split(x, bk["n1g"], bk["n1b"], 1e-5)
            qkv = ops.x3_linear(h, bk["qkv_w"], bk["qkv_b"])
        a = ops.x3_swin_window_attention_split(qkv, bk["bias"], H, heads, ws, bk["shift"])
        if rowlin and bk["proj_pack"] is not None and isinstance(a, ops.X3Rows):
            return ops.x3_rowlin(a, bk["proj_pack"], bk["proj_b"], C, residual=x)
        return ops.x3_linear(a, bk["proj_w"], bk["proj_b"], residual=x)

    def forward_features(self, image):
        return _ln(self.tokens(image), self.norm_g, self.norm_b, 1e-5)

    def head(self, tok):
        """Backbones.forward image branch (fusion.py:259-265) from pre-norm tokens (B, h, w, C):
        (img_global, img_patches, pool) f32 — pool = mean over [global; patches] (the image head's
        input, model.py:463-468)."""
        B, H, W, C = tok.shape
        pf = _ln(tok, self.norm_g, self.norm_b, 1e-5).view(B, H * W, C)   # forward_features output
        patches = _ln(pf, self.norm_g, self.norm_b, 1e-5)                  # swin_norm applied again
        glob = ops.x3_mean_rows(pf)
        pool = ops.x3_mean_rows(patches, extra=glob)
        return glob, patches, pool


class BertTowerX3:
    """HF BertModel(input_ids, attention_mask).last_hidden_state in the x3 mode."""

    def __init__(self, sd, cfg=BERT_BASE, device="cuda"):
        self.cfg = dict(BERT_BASE, **cfg)
        dev = torch.device(device)
        self.device = dev
        self.word = _f(sd["embeddings.word_embeddings.weight"], dev)
        self.pos = _f(sd["embeddings.position_embeddings.weight"], dev)
        self.type0 = _f(sd["embeddings.token_type_embeddings.weight"][0], dev)
        self.eg, self.eb = _f(sd["embeddings.LayerNorm.weight"], dev), _f(sd["embeddings.LayerNorm.bias"], dev)
        self.layers = []
        for i in range(self.cfg["num_hidden_layers"]):
            p = f"encoder.layer.{i}."
            qkv_w = torch.cat([sd[p + f"attention.self.{n}.weight"] for n in ("query", "key", "value")], 0)
            qkv_b = torch.cat([sd[p + f"attention.self.{n}.bias"] for n in ("query", "key", "value")], 0)
            self.layers.append({
                "qkv_w": _x3(qkv_w, dev), "qkv_b": _f(qkv_b, dev),
                "o_w": _x3(sd[p + "attention.output.dense.weight"], dev),
                "o_b": _f(sd[p + "attention.output.dense.bias"], dev),
                "ln1_g": _f(sd[p + "attention.output.LayerNorm.weight"], dev),
                "ln1_b": _f(sd[p + "attention.output.LayerNorm.bias"], dev),
                "i_w": _x3(sd[p + "intermediate.dense.weight"], dev), "i_b": _f(sd[p + "intermediate.dense.bias"], dev),
                "f_w": _x3(sd[p + "output.dense.weight"], dev), "f_b": _f(sd[p + "output.dense.bias"], dev),
                "ln2_g": _f(sd[p + "output.LayerNorm.weight"], dev), "ln2_b": _f(sd[p + "output.LayerNorm.bias"], dev),
            })
        self.hidden = self.word.shape[1]
        self.gemm_events = None  # as BertTower.gemm_events (the bench's per-GEMM roofline pass)
        # the residual adds in the O-proj / FFN2 epilogues ((acc + b) + h, the LayerNorm kernel's own order)
        # instead of in the LayerNorm pass, which then reads one f32 row instead of two (A/B attribute)
        self.res_in_gemm = True

    def _gemm(self, name, x, w, b, act=0, residual=None):
        ev = self.gemm_events
        if ev is None:
            return ops.x3_linear(x, w, b, act=act, residual=residual)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        y = ops.x3_linear(x, w, b, act=act)
        e1.record()
        ev.setdefault(name, []).append((e0, e1))
        return y

    def forward(self, input_ids, attention_mask=None):
        """(B, L) ids / mask -> (B, L, C) f32 last_hidden_state (L truncated to max_position_embeddings)."""
        cfg = self.cfg
        ids = input_ids.to(self.device, torch.int64)
        if attention_mask is None:
            attention_mask = torch.ones_like(ids)
        mask = attention_mask.to(self.device, torch.int64)
        max_len = cfg["max_position_embeddings"]
        if ids.shape[1] > max_len:
            ids, mask = ids[:, :max_len], mask[:, :max_len]
        ids, mask = ids.contiguous(), mask.contiguous()
        B, L = ids.shape
        heads = cfg["num_attention_heads"]
        C = self.hidden
        dh = C // heads
        h = ops.x3_bert_embed(ids, self.word, self.pos, self.type0, self.eg, self.eb, 1e-12)
        hs = h  # the QKV operand: the previous layer's LayerNorm output as split rows (X3Rows)
        for li, ly in enumerate(self.layers):
            qkv = self._gemm("qkv", hs, ly["qkv_w"], ly["qkv_b"]).view(B * L, 3 * C)
            ctx = ops.x3_attention_split(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, L, L, heads, dh,
                                         1.0 / math.sqrt(dh), mask=mask)
            rg = self.res_in_gemm and self.gemm_events is None
            a = self._gemm("o", ctx, ly["o_w"], ly["o_b"], residual=h if rg else None)
            if self.gemm_events is None:
                # LN(dense(ctx) + h), kept f32 for the next residual and split for FFN1
                h, hs = ops.x3_ln_split(a, ly["ln1_g"], ly["ln1_b"], 1e-12, residual=None if rg else h, keep_f32=True)
                f = ops.x3_ffn(hs, ly["i_w"], ly["i_b"], ly["f_w"], ly["f_b"], residual=h if rg else None)
                r2 = None if rg else h
                if li + 1 < len(self.layers):
                    h, hs = ops.x3_ln_split(f, ly["ln2_g"], ly["ln2_b"], 1e-12, residual=r2, keep_f32=True)
                else:
                    h = _ln(f, ly["ln2_g"], ly["ln2_b"], 1e-12, residual=r2)
            else:
                h = _ln(a, ly["ln1_g"], ly["ln1_b"], 1e-12, residual=h)
                f = self._gemm("ffn2", self._gemm("ffn1", h, ly["i_w"], ly["i_b"], act=1), ly["f_w"], ly["f_b"])
                h = hs = _ln(f, ly["ln2_g"], ly["ln2_b"], 1e-12, residual=h)
        return h
