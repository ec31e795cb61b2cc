"""ORACLE (test infrastructure): Swin-v1 / BERT towers and the reference heads in plain torch fp32.

swin_forward_features  timm 1.0.17 SwinTransformer.forward_features (called at
                       src/Model/fusion.py:198-199): patch_embed (conv 4x4/s4 + LN, NHWC) ->
                       stages (PatchMerging at the start of stages 1..3, [x00,x10,x01,x11] channel
                       order) of (S)W-MSA blocks (roll(-shift), 7x7 windows, q*dh^-0.5, rel-pos bias,
                       -100 shift mask, proj, residual; LN -> fc1 -> GELU(erf) -> fc2, residual) ->
                       final LN.  Window/shift clamp when the resolution <= window (7x7 stage: no
                       shift).  Returns (B, H, W, C) NHWC.
bert_forward           HF BertModel(...).last_hidden_state (fusion.py:322-325): word + position +
                       token_type(0) -> LN(eps 1e-12); per layer: QKV, softmax(QK^T/sqrt(dh) +
                       (1-mask)*min_f32) V, dense + residual + LN, GELU(erf) FFN + residual + LN.
backbones_forward      Backbones.forward swin+text branch (fusion.py:255-327): img_patches =
                       swin_norm(patch_feats) (the Swin's own final norm applied a 2nd time),
                       img_global = mean of the once-normed tokens, txt_feats = last_hidden_state.
heads                  MultiModalRetrievalModel.forward (model.py:365-373, 462-479): img_emb,
                       txt_emb (unmasked mean over ALL L positions incl. PAD), text / image heads
                       through MultiHeadMLP (model.py:61-75; ffn[0] since use_shared_ffn=False,
                       configs/config.yaml).
multimodal             model_type="multimodal" (model.py:375-459): num_fusion_layers x
                       CrossModalFusion (fusion.py:334-471, PreFusionEnhancer fusion.py:20-35) +
                       pos_encoder + self_attn (nn.MultiheadAttention restated in `mha`) + residual /
                       LayerNorm / FFN / adapter chain; eval mode (dropout, stochastic depth off).
"""
import math

import torch
import torch.nn.functional as F


def _ln(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def _lin(x, sd, p, bias=True):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias") if bias else None)


def relative_position_index(ws):
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")).flatten(1)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1)  # (N, N)


def shift_mask(H, W, ws, shift):
    img = torch.zeros((1, H, W, 1))
    cnt = 0
    for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img[:, hs, wsl, :] = cnt
            cnt += 1
    mw = window_partition(img, ws).view(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)  # (nW, N, N)


def window_partition(x, ws):
    B, H, W, C = x.shape
    return x.view(B, H // ws, ws, W // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws, ws, C)


def window_reverse(w, ws, H, W):
    C = w.shape[-1]
    B = w.shape[0] // ((H // ws) * (W // ws))
    return w.view(B, H // ws, W // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, C)


def swin_attn_half(x, sd, p, heads, ws, shift, eps=1e-5):
    """x + proj(W-MSA(norm1(x))): the attention half of timm SwinTransformerBlock.forward."""
    B, H, W, C = x.shape
    hd = C // heads
    N = ws * ws
    h = _ln(x, sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
    if shift:
        h = torch.roll(h, shifts=(-shift, -shift), dims=(1, 2))
    win = window_partition(h, ws).view(-1, N, C)
    qkv = _lin(win, sd, p + "attn.qkv").view(-1, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * hd ** -0.5, qkv[1], qkv[2]
    attn = q @ k.transpose(-2, -1)
    table = sd[p + "attn.relative_position_bias_table"]
    bias = table[relative_position_index(ws).view(-1)].view(N, N, heads).permute(2, 0, 1)
    attn = attn + bias.unsqueeze(0)
    if shift:
        m = shift_mask(H, W, ws, shift)
        nW = m.shape[0]
        attn = (attn.view(-1, nW, heads, N, N) + m.unsqueeze(1).unsqueeze(0)).view(-1, heads, N, N)
    attn = attn.softmax(-1)
    o = (attn @ v).transpose(1, 2).reshape(-1, N, C)
    o = _lin(o, sd, p + "attn.proj")
    o = window_reverse(o.view(-1, ws, ws, C), ws, H, W)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    return x + o


def swin_block(x, sd, p, heads, ws, shift, eps=1e-5):
    x = swin_attn_half(x, sd, p, heads, ws, shift, eps)
    y = _ln(x, sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
    y = _lin(F.gelu(_lin(y, sd, p + "mlp.fc1")), sd, p + "mlp.fc2")
    return x + y


def patch_merging(x, sd, p, eps=1e-5):
    B, H, W, C = x.shape
    x = x.reshape(B, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 4, 2, 5).flatten(3)
    x = _ln(x, sd[p + "norm.weight"], sd[p + "norm.bias"], eps)
    return F.linear(x, sd[p + "reduction.weight"])


def swin_forward_features(x, sd, depths, num_heads, window=7, eps=1e-5, return_prenorm=False):
    x = F.conv2d(x, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=4)
    x = x.permute(0, 2, 3, 1)
    x = _ln(x, sd["patch_embed.norm.weight"], sd["patch_embed.norm.bias"], eps)
    for i, depth in enumerate(depths):
        if i > 0:
            x = patch_merging(x, sd, f"layers.{i}.downsample.", eps)
        H = x.shape[1]
        ws = min(window, H)
        for j in range(depth):
            shift = 0 if (j % 2 == 0 or H <= window) else window // 2
            x = swin_block(x, sd, f"layers.{i}.blocks.{j}.", num_heads[i], ws, shift, eps)
    pre = x
    x = _ln(x, sd["norm.weight"], sd["norm.bias"], eps)
    return (x, pre) if return_prenorm else x


def bert_forward(ids, mask, sd, num_layers, num_heads, eps=1e-12):
    B, L = ids.shape
    h = (sd["embeddings.word_embeddings.weight"][ids]
         + sd["embeddings.position_embeddings.weight"][:L][None]
         + sd["embeddings.token_type_embeddings.weight"][0][None, None])
    h = _ln(h, sd["embeddings.LayerNorm.weight"], sd["embeddings.LayerNorm.bias"], eps)
    C = h.shape[-1]
    dh = C // num_heads
    ext = (1.0 - mask.to(torch.float32))[:, None, None, :] * torch.finfo(torch.float32).min
    for i in range(num_layers):
        p = f"encoder.layer.{i}."

        def heads(t):
            return t.view(B, L, num_heads, dh).transpose(1, 2)
        q = heads(_lin(h, sd, p + "attention.self.query"))
        k = heads(_lin(h, sd, p + "attention.self.key"))
        v = heads(_lin(h, sd, p + "attention.self.value"))
        s = q @ k.transpose(-1, -2) / math.sqrt(dh) + ext
        ctx = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, L, C)
        a = _lin(ctx, sd, p + "attention.output.dense")
        h = _ln(a + h, sd[p + "attention.output.LayerNorm.weight"], sd[p + "attention.output.LayerNorm.bias"], eps)
        f = _lin(F.gelu(_lin(h, sd, p + "intermediate.dense")), sd, p + "output.dense")
        h = _ln(f + h, sd[p + "output.LayerNorm.weight"], sd[p + "output.LayerNorm.bias"], eps)
    return h


def swin_image(image, swin_sd, swin_cfg):
    """Backbones.forward image branch (fusion.py:259-265): (img_global, img_patches)."""
    feats = swin_forward_features(image, swin_sd, swin_cfg["depths"], swin_cfg["num_heads"])
    B, H, W, C = feats.shape
    pf = feats.reshape(B, H * W, C)
    img_patches = _ln(pf, swin_sd["norm.weight"], swin_sd["norm.bias"], 1e-5)  # swin_norm again
    img_global = pf.mean(dim=1)
    return img_global, img_patches


def backbones_forward(image, ids, mask, swin_sd, bert_sd, swin_cfg, bert_cfg):
    img_global, img_patches = swin_image(image, swin_sd, swin_cfg)
    txt = bert_forward(ids, mask, bert_sd, bert_cfg["num_hidden_layers"], bert_cfg["num_attention_heads"])
    return (img_global, img_patches), txt


def multi_head_mlp(x, sd, p):
    return _lin(F.gelu(_lin(x, sd, p + "linear1")), sd, p + "linear2")


def heads(img_global, img_patches, txt_feats, hsd, model_type, ffn_prefix="ffn.0.", mm_cfg=None):
    img_emb = _lin(img_global, hsd, "img_proj") if img_global is not None else None
    txt_emb = _lin(txt_feats.mean(dim=1), hsd, "txt_proj") if txt_feats is not None else None
    if model_type == "text":
        joint = multi_head_mlp(_lin(txt_feats.mean(dim=1), hsd, "txt_proj"), hsd, ffn_prefix)
    elif model_type == "image":
        g = _lin(img_global, hsd, "img_proj")
        p = _lin(img_patches, hsd, "img_proj")
        joint = multi_head_mlp(torch.cat([g.unsqueeze(1), p], 1).mean(1), hsd, ffn_prefix)
    else:
        joint = multimodal(img_global, img_patches, txt_feats, hsd, **(mm_cfg or {}))
    return {"joint_emb": joint, "img_emb": img_emb, "txt_emb": txt_emb}


def mha(q_in, k_in, v_in, sd, p, heads):
    """torch.nn.MultiheadAttention(batch_first=True).forward in eval, no masks: packed
    in_proj_weight [3E][E] (q|k|v), per-head softmax(q k^T / sqrt(dh)) v, out_proj."""
    E = sd[p + "in_proj_weight"].shape[1]
    W, b = sd[p + "in_proj_weight"], sd[p + "in_proj_bias"]
    q = F.linear(q_in, W[:E], b[:E])
    k = F.linear(k_in, W[E:2 * E], b[E:2 * E])
    v = F.linear(v_in, W[2 * E:], b[2 * E:])
    B, Lq, _ = q.shape
    Lk = k.shape[1]
    dh = E // heads

    def hd(t, L):
        return t.view(B, L, heads, dh).transpose(1, 2)
    a = (hd(q, Lq) @ hd(k, Lk).transpose(-1, -2) / math.sqrt(dh)).softmax(-1) @ hd(v, Lk)
    return _lin(a.transpose(1, 2).reshape(B, Lq, E), sd, p + "out_proj")


def prefusion_enhancer(x, sd, p, heads, eps=1e-5):
    """PreFusionEnhancer.forward (src/Model/fusion.py:30-35), eval (dropout = identity)."""
    L = x.shape[1]
    x = x + sd[p + "pos_embed"][:, :L]
    x2 = mha(x, x, x, sd, p + "self_attn.", heads)
    return _ln(sd[p + "alpha"] * x + x2, sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)


def cross_modal_fusion(img_global, img_patch, txt_feats, sd, p, heads, use_cls_only=False, eps=1e-5):
    """CrossModalFusion.forward (fusion.py:390-471) -> (B, 1+Np+1, D) sequence (use_cls_only:
    (B, D) comb_mlp vector)."""
    if txt_feats is None:  # learnable default text token (fusion.py:404-407)
        txt_feats = sd[p + "default_txt_token"].expand(img_patch.shape[0], -1, -1)
    txt = prefusion_enhancer(txt_feats, sd, p + "txt_self_attn.", heads, eps)
    g = prefusion_enhancer(img_global.unsqueeze(1), sd, p + "img_global_self_attn.", heads, eps).squeeze(1)
    pt = prefusion_enhancer(img_patch, sd, p + "img_patch_self_attn.", heads, eps)
    tp = txt[:, 0:1] if use_cls_only else txt
    att_t2i = mha(_lin(tp, sd, p + "query_txt"), _lin(pt, sd, p + "key_img"), _lin(pt, sd, p + "value_img"),
                  sd, p + "attn_txt2img.", heads)
    att_i2t = mha(_lin(pt, sd, p + "query_img"), _lin(tp, sd, p + "key_txt"), _lin(tp, sd, p + "value_txt"),
                  sd, p + "attn_img2txt.", heads)
    patches_fused = _lin(pt, sd, p + "img_patch_proj") + att_i2t
    x1 = _ln(_lin(g, sd, p + "img_global_proj") + att_t2i.mean(1), sd[p + "ln_img.weight"], sd[p + "ln_img.bias"], eps)
    x2 = _ln(_lin(txt, sd, p + "txt_proj")[:, 0] + att_i2t.mean(1), sd[p + "ln_txt.weight"], sd[p + "ln_txt.bias"], eps)
    if use_cls_only:
        cat = torch.cat([x1, patches_fused.mean(1), x2], 1)
        return _lin(F.gelu(_lin(cat, sd, p + "comb_mlp.0")), sd, p + "comb_mlp.3")
    return torch.cat([x1.unsqueeze(1), patches_fused, x2.unsqueeze(1)], 1)


def multimodal(img_global, img_patches, txt_feats, sd, num_heads=4, num_fusion_layers=None,
               use_shared_ffn=False, use_cls_only=False, eps=1e-5):
    """MultiModalRetrievalModel.forward, model_type="multimodal" (model.py:375-459), eval:
    per layer i the fusion of the SAME backbone features, + pos_encoder, self_attn, mean over the
    sequence; x = fused (i == 0) or norm1_i(joint) + alpha * fused; x += ffn(norm2_i(x));
    x += adapter_i(x)."""
    if use_cls_only:
        # model.py:428-429 indexes fused_out[:, 0, :] on the 2-D comb_mlp output: the reference
        # raises there, so there is no multimodal use_cls_only result to restate
        raise ValueError("multimodal with use_cls_only fails in the reference (model.py:428-429)")
    if num_fusion_layers is None:
        num_fusion_layers = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("fusion_layers."))
    joint = None
    for i in range(num_fusion_layers):
        seq = cross_modal_fusion(img_global, img_patches, txt_feats, sd, f"fusion_layers.{i}.", num_heads,
                                 False, eps)
        seq = seq + sd["pos_encoder.pe"][:, :seq.shape[1]]
        fused = mha(seq, seq, seq, sd, "self_attn.", num_heads).mean(1)
        if i == 0:
            x = fused
        else:
            x = _ln(joint, sd[f"norm1_layers.{i}.weight"], sd[f"norm1_layers.{i}.bias"], eps) + sd["alpha"] * fused
        xf = _ln(x, sd[f"norm2_layers.{i}.weight"], sd[f"norm2_layers.{i}.bias"], eps)
        x = x + multi_head_mlp(xf, sd, "shared_ffn." if use_shared_ffn else f"ffn.{i}.")
        x = x + _lin(F.gelu(_lin(x, sd, f"adapters.{i}.0")), sd, f"adapters.{i}.2")
        joint = x
    return joint
