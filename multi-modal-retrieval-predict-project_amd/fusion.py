"""Multimodal fusion stack on libmmr kernels — model_type="multimodal" of MultiModalRetrievalModel.

Reference (eval semantics): CrossModalFusion.forward src/Model/fusion.py:390-471,
PreFusionEnhancer fusion.py:20-35, MultiModalRetrievalModel.forward model.py:375-459 (pos_encoder
model.py:91-107, self_attn = nn.MultiheadAttention(joint_dim, num_heads), StochasticDepth = plain
residual in eval, MultiHeadMLP model.py:61-75, adapters model.py:262-268).  Restated in plain torch
in oracle/towers.py:multimodal and pinned there against the reference's own outputs.

Every fusion layer reads the SAME backbone features (img_global, img_patches, txt_feats); only the
(B, D) joint vector chains through the layers.  Per layer the device work is:

  text enhancer    X = T + pos  ->  QKV GEMM  ->  mha(L x L)  ->  out GEMM  ->  LN(a*X + .)      [B*L rows]
  patch enhancer   same over the 49 patch tokens                                                [B*49 rows]
  global enhancer  a 1-token self-attention is exactly out_proj(v_proj(x)): ONE folded f32 linear
  cross attention  nn.MultiheadAttention re-projects its inputs (in_proj after query_txt/key_img/...),
                   two affine maps in a row: folded at load into one weight (W_in . W, W_in . b + b_in),
                   so text -> [q_t2i | k_i2t | v_i2t] and patches -> [k_t2i | v_t2i | q_i2t] are one
                   GEMM each; txt2img only enters through its mean over L, and mean commutes with the
                   affine out_proj, so mha emits the mean directly (no B*L x D out_proj GEMM)
  fused sequence   [ln_img(.); img_patch_proj(P) + out_proj(img2txt); ln_txt(.)] + pe  ->  QKV GEMM
                   -> mha with mean output -> one f32 out_proj row per batch (model.py:431 mean)
  joint chain      f32 (B, D): norm1 / alpha residual, norm2 -> FFN, adapter (f32 vectors, linears on
                   bf16x3 MFMA: ops.linear_x3, ~2^-17 relative per product; exact f32 with
                   exact_query_linears=True)

bf16 activations / f32 accumulation for the token-level work, f32 for every per-query vector (its
linears on bf16x3 MFMA).
tower_dtype="fp8" (BASELINE config 5): the token-level GEMMs — each enhancer's in_proj and out_proj,
the folded text / patch cross projections + img_patch_proj, and the img2txt out-projection
(patches_fused) — run on the MX-fp8 GEMM; their activation operands come out of the producing
add-pos / attention / LayerNorm kernels (no quantise pass).  Batches whose token rows are not a 256
multiple keep bf16 there.
"""
import collections
import math

import torch

from . import ops


def _f(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _bf(t, dev):
    return t.detach().to(device=dev, dtype=torch.bfloat16).contiguous()


def _fold(w_in, b_in, w, b):
    """(W_in, b_in) o (W, b) = (W_in W, W_in b + b_in), computed in f64."""
    w_in, b_in, w, b = (t.detach().double().cpu() for t in (w_in, b_in, w, b))
    return w_in @ w, w_in @ b + b_in


def _w8(w):
    """bf16 weight -> MX-fp8 operand for a plain bias GEMM (256 x 256 tiles when N % 256 == 0)."""
    return ops.quantize_mxfp8(w, layout=2 if w.shape[0] % 256 == 0 else 1)


class _Enhancer:
    """PreFusionEnhancer weights (fusion.py:20-35)."""

    def __init__(self, sd, p, heads, dev, fp8=False, x3=False):
        C = sd[p + "self_attn.in_proj_weight"].shape[1]
        self.C, self.heads, self.dh = C, heads, C // heads
        self.pos = _f(sd[p + "pos_embed"][0], dev)                       # [max_len][C]
        if x3:  # fp32-faithful mode: f32 weights split once for the bf16x3 GEMM
            self.w_in_x3 = ops.X3W(_f(sd[p + "self_attn.in_proj_weight"], dev))
            self.w_o_x3 = ops.X3W(_f(sd[p + "self_attn.out_proj.weight"], dev))
        self.w_in, self.b_in = _bf(sd[p + "self_attn.in_proj_weight"], dev), _f(sd[p + "self_attn.in_proj_bias"], dev)
        self.w_o, self.b_o = _bf(sd[p + "self_attn.out_proj.weight"], dev), _f(sd[p + "self_attn.out_proj.bias"], dev)
        self.alpha = _f(sd[p + "alpha"].reshape(1), dev)
        self.g, self.b = _f(sd[p + "norm1.weight"], dev), _f(sd[p + "norm1.bias"], dev)
        # MX-fp8 needs C % 256 (operand panels) and head_dim % 32 (the attention core's q8 output is
        # one 32-block per lane pair); otherwise this enhancer stays bf16
        f8 = fp8 and C % 256 == 0 and self.dh % 32 == 0
        self.w_in8 = _w8(self.w_in) if f8 else None
        self.w_o8 = _w8(self.w_o) if f8 else None

    def fp8_ok(self, rows):
        return self.w_in8 is not None and rows % 256 == 0

    def __call__(self, x, B, L, eps, q8=False):
        """x (B*L, C) f32 or bf16 -> LN(alpha*(x + pos) + MHA(x + pos)) bf16 (B*L, C); q8 (fp8 path):
        (y, its MX-fp8 operand)."""
        C = self.C
        if self.fp8_ok(B * L):
            # MX-fp8: the add-pos kernel emits the in_proj operand, the attention core the out_proj one
            X, X8 = ops.add_pos(x, self.pos, L, q8=True)
            qkv = ops.linear_mxfp8(X8, self.w_in8, self.b_in)
            _, _, a8 = ops.mha(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, L, L, self.heads, self.dh,
                               1.0 / math.sqrt(self.dh), q8=True)
            x2 = ops.linear_mxfp8(a8, self.w_o8, self.b_o)
        else:
            X = ops.add_pos(x, self.pos, L)
            qkv = ops.linear(X, self.w_in, self.b_in)
            a = torch.empty_like(X)
            ops.mha(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, L, L, self.heads, self.dh,
                    1.0 / math.sqrt(self.dh), out=a)
            x2 = ops.linear(a, self.w_o, self.b_o)
        return ops.scaled_add_layernorm(X, self.alpha, x2, self.g, self.b, eps, q8=q8)

    def x3(self, x, B, L, eps, keep_f32=True):
        """x3 mode: x (B*L, C) f32 -> (y, ys): y = LN(alpha*(x + pos) + MHA(x + pos)) f32 (B*L, C) (None
        unless keep_f32) and ys its x3 split-operand rows (ops.X3Rows; the f32 rows where the row count
        does not fill 256-row tiles).  Every GEMM operand is written split by its producer: add-pos -> in_proj,
        attention -> out_proj, LayerNorm -> the cross projections (no split passes)."""
        C = self.C
        X, Xs = ops.x3_add_pos_split(x, self.pos, L)
        qkv = ops.x3_linear(Xs, self.w_in_x3, self.b_in)
        a = ops.x3_attention_split(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, L, L, self.heads, self.dh,
                                   1.0 / math.sqrt(self.dh))
        x2 = ops.x3_linear(a, self.w_o_x3, self.b_o)
        y = ops.x3_ln_split(X, self.g, self.b, eps, residual=x2, keep_f32=keep_f32, alpha=self.alpha)
        return y if keep_f32 else (None, y)


class FusionStack:
    """The multimodal head: num_fusion_layers x CrossModalFusion + combiner (model.py:375-459)."""

    def __init__(self, sd, num_heads, device="cuda", use_shared_ffn=False, eps=1e-5, tower_dtype="bf16",
                 exact_query_linears=False):
        dev = torch.device(device)
        self.device, self.heads, self.eps = dev, num_heads, eps
        # the per-query linears (phases 2-4) on bf16x3 MFMA (default, ~2^-17 relative per product) or,
        # exact_query_linears = True, on exact f32 (ops.linear_f32 / linear_f32_batched, ~5x slower)
        self.exact_query_linears = exact_query_linears
        self.side_streams = True  # patch-side layer work on a side stream (False: one stream)
        fp8 = tower_dtype == "fp8"
        self.fp8 = fp8
        x3 = tower_dtype == "x3"
        self.x3 = x3
        n = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("fusion_layers."))
        self.layers = []
        D = sd["self_attn.in_proj_weight"].shape[1]
        self.D = D
        for i in range(n):
            p = f"fusion_layers.{i}."
            g = lambda k: sd[p + k]  # noqa: E731
            L = {"txt": _Enhancer(sd, p + "txt_self_attn.", num_heads, dev, fp8, x3),
                 "patch": _Enhancer(sd, p + "img_patch_self_attn.", num_heads, dev, fp8, x3)}
            # global enhancer: softmax over ONE key is 1 -> x2 = Wo (Wv x + bv) + bo; with x = G + pos0
            # and the LN input alpha*x + x2 = alpha*G + (Wov G + Wov pos0 + bov + alpha*pos0)
            pg = "img_global_self_attn."
            Ci = g(pg + "self_attn.in_proj_weight").shape[1]
            wv = g(pg + "self_attn.in_proj_weight")[2 * Ci:]
            bv = g(pg + "self_attn.in_proj_bias")[2 * Ci:]
            wov, bov = _fold(g(pg + "self_attn.out_proj.weight"), g(pg + "self_attn.out_proj.bias"), wv, bv)
            pos0 = g(pg + "pos_embed")[0, 0].double()
            alpha_g = g(pg + "alpha").double().reshape(())
            L["g_w"] = _f(wov, dev)
            L["g_b"] = _f(wov @ pos0 + bov + alpha_g * pos0, dev)
            L["g_alpha"] = _f(g(pg + "alpha").reshape(1), dev)
            L["g_ln"] = (_f(g(pg + "norm1.weight"), dev), _f(g(pg + "norm1.bias"), dev))
            # cross attention: fold the pre-projections into nn.MultiheadAttention's in_proj
            wi1, bi1 = g("attn_txt2img.in_proj_weight"), g("attn_txt2img.in_proj_bias")
            wi2, bi2 = g("attn_img2txt.in_proj_weight"), g("attn_img2txt.in_proj_bias")
            sl = [slice(0, D), slice(D, 2 * D), slice(2 * D, 3 * D)]
            qt = _fold(wi1[sl[0]], bi1[sl[0]], g("query_txt.weight"), g("query_txt.bias"))
            kt = _fold(wi2[sl[1]], bi2[sl[1]], g("key_txt.weight"), g("key_txt.bias"))
            vt = _fold(wi2[sl[2]], bi2[sl[2]], g("value_txt.weight"), g("value_txt.bias"))
            ki = _fold(wi1[sl[1]], bi1[sl[1]], g("key_img.weight"), g("key_img.bias"))
            vi = _fold(wi1[sl[2]], bi1[sl[2]], g("value_img.weight"), g("value_img.bias"))
            qi = _fold(wi2[sl[0]], bi2[sl[0]], g("query_img.weight"), g("query_img.bias"))
            if x3:  # the folded token-level weights in f32 (folded in f64), split for bf16x3
                L["t_x3"] = ops.X3W(_f(torch.cat([qt[0], kt[0], vt[0]]), dev))
                # the patch tokens' two linears (k_t2i | v_t2i | q_i2t and img_patch_proj) as ONE N = 4D
                # GEMM: 4x the tiles of the M = B*Np launch (49 row tiles at B = 256 filled 196 of 256
                # CUs), one split pass; each column's sum is the same K loop, so the same bits
                L["ppp_x3"] = ops.X3W(_f(torch.cat([ki[0], vi[0], qi[0], g("img_patch_proj.weight")]), dev))
                L["o2_x3t"] = ops.X3W(_f(g("attn_img2txt.out_proj.weight"), dev))
                L["default_txt32"] = _f(g("default_txt_token").reshape(1, -1), dev)
            L["t_w"] = _bf(torch.cat([qt[0], kt[0], vt[0]]), dev)
            L["t_b"] = _f(torch.cat([qt[1], kt[1], vt[1]]), dev)
            L["p_w"] = _bf(torch.cat([ki[0], vi[0], qi[0]]), dev)
            L["p_b"] = _f(torch.cat([ki[1], vi[1], qi[1]]), dev)
            L["pp_w"], L["pp_b"] = _bf(g("img_patch_proj.weight"), dev), _f(g("img_patch_proj.bias"), dev)
            if x3:
                L["ppp_b"] = torch.cat([L["p_b"], L["pp_b"]])
            L["o1_w"], L["o1_b"] = _f(g("attn_txt2img.out_proj.weight"), dev), _f(g("attn_txt2img.out_proj.bias"), dev)
            L["o2_wb"] = _bf(g("attn_img2txt.out_proj.weight"), dev)
            if fp8:
                for k in ("t_w", "p_w", "pp_w", "o2_wb"):
                    L[k + "8"] = _w8(L[k])
            L["o2_w"], L["o2_b"] = _f(g("attn_img2txt.out_proj.weight"), dev), _f(g("attn_img2txt.out_proj.bias"), dev)
            L["gp_w"], L["gp_b"] = _f(g("img_global_proj.weight"), dev), _f(g("img_global_proj.bias"), dev)
            L["tp_w"], L["tp_b"] = _f(g("txt_proj.weight"), dev), _f(g("txt_proj.bias"), dev)
            L["ln_img"] = (_f(g("ln_img.weight"), dev), _f(g("ln_img.bias"), dev))
            L["ln_txt"] = (_f(g("ln_txt.weight"), dev), _f(g("ln_txt.bias"), dev))
            L["default_txt"] = _bf(g("default_txt_token").reshape(1, -1), dev)
            # combiner (model.py:227-268) for layer i
            L["n1"] = (_f(sd[f"norm1_layers.{i}.weight"], dev), _f(sd[f"norm1_layers.{i}.bias"], dev))
            L["n2"] = (_f(sd[f"norm2_layers.{i}.weight"], dev), _f(sd[f"norm2_layers.{i}.bias"], dev))
            fp = "shared_ffn." if use_shared_ffn else f"ffn.{i}."
            L["ffn"] = tuple(_f(sd[fp + k], dev) for k in ("linear1.weight", "linear1.bias", "linear2.weight",
                                                           "linear2.bias"))
            L["ad"] = tuple(_f(sd[f"adapters.{i}.{k}"], dev) for k in ("0.weight", "0.bias", "2.weight", "2.bias"))
            self.layers.append(L)
        self.s_w, self.s_b = _bf(sd["self_attn.in_proj_weight"], dev), _f(sd["self_attn.in_proj_bias"], dev)
        # combiner QKV on MX-fp8 (its operand written by the sequence assembly itself)
        self.s_w8 = _w8(self.s_w) if fp8 and D % 256 == 0 else None
        self.s_x3 = ops.X3W(_f(sd["self_attn.in_proj_weight"], dev)) if x3 else None
        self.s_ow, self.s_ob = _f(sd["self_attn.out_proj.weight"], dev), _f(sd["self_attn.out_proj.bias"], dev)
        self.pe = _f(sd["pos_encoder.pe"][0], dev)
        self.alpha = _f(sd["alpha"].reshape(1), dev)
        # per-query work of all layers batched (stacked per-layer parameters):
        #  global enhancer  LN(alpha*G + Wov G + b) = LN((Wov + alpha I) G + b): ONE linear over the
        #                   concatenated weights (same input G) + one grouped LayerNorm
        Ls = self.layers
        eye = torch.eye(Ls[0]["g_w"].shape[0], device=dev)
        self.g_w_all = torch.cat([L["g_w"] + L["g_alpha"] * eye for L in Ls]).contiguous()
        self.g_b_all = torch.cat([L["g_b"] for L in Ls]).contiguous()
        self.g_ln_all = tuple(torch.stack([L["g_ln"][k] for L in Ls]).contiguous() for k in (0, 1))
        st = lambda k: torch.stack([L[k] for L in Ls]).contiguous()  # noqa: E731
        self.o1_w_all, self.o1_b_all = st("o1_w"), st("o1_b")
        self.o2_w_all, self.o2_b_all = st("o2_w"), st("o2_b")
        self.gp_w_all, self.gp_b_all = st("gp_w"), st("gp_b")
        self.tp_w_all, self.tp_b_all = st("tp_w"), st("tp_b")
        # bf16x3 splits of every per-query weight (ops.linear_x3: 1/5 of the f32 MFMA time)
        X3 = ops.X3W
        self.g_w_x3 = X3(self.g_w_all)
        self.o1_x3, self.o2_x3, self.gp_x3, self.tp_x3 = (X3(self.o1_w_all), X3(self.o2_w_all), X3(self.gp_w_all),
                                                          X3(self.tp_w_all))
        self.s_ow_x3 = X3(self.s_ow)
        for L in Ls:
            L["ffn_x3"] = (X3(L["ffn"][0]), X3(L["ffn"][2]))
            L["ad_x3"] = (X3(L["ad"][0]), X3(L["ad"][2]))
        self.ln_img_all = tuple(torch.stack([L["ln_img"][k] for L in Ls]).contiguous() for k in (0, 1))
        self.ln_txt_all = tuple(torch.stack([L["ln_txt"][k] for L in Ls]).contiguous() for k in (0, 1))

    def _ql(self, x, wx, bias=None, residual=None, act=0, out=None):
        if self.exact_query_linears:
            return ops.linear_f32(x, wx.w, bias, residual=residual, act=act, out=out)
        return ops.linear_x3(x, wx, bias, residual=residual, act=act, out=out)

    def _qlb(self, x, wx, bias, nbatch, b, **kw):
        if self.exact_query_linears:
            return ops.linear_f32_batched(x, wx.w, bias, nbatch, b, **kw)
        return ops.linear_x3_batched(x, wx, bias, nbatch, b, **kw)

    def _side_stream(self, main):
        # one side stream per calling stream (pipelined callers keep their batches independent)
        if getattr(self, "_side", None) is None:
            self._side = collections.OrderedDict()
        return ops.side_stream(self._side, main, self.device)

    def patch_work(self, img_patches):
        """The patch-side token work of every layer (enhancer, folded k/v/q projection, patch
        projection) on the CURRENT stream, an event recorded after each layer: it depends on the
        image tower only, so a caller may start it as soon as that tower is done (the towers' side
        stream: MultiModalRetrievalModel.query_embeddings) and hand it to forward(patch_work=...).
        Returns {"pq": [...], "pp": [...], "ev": [...], "stream": the stream it ran on}."""
        B, Np, Ci = img_patches.shape
        D, eps = self.D, self.eps
        pq, pp, ev = [], [], []
        cur = torch.cuda.current_stream(self.device)
        if self.x3:
            P = img_patches.float().contiguous().view(B * Np, Ci)
        else:
            P = img_patches.contiguous().view(B * Np, Ci)
        for L in self.layers:
            if self.x3:
                _, Pes = L["patch"].x3(P, B, Np, eps, keep_f32=False)        # (B*Np, Ci), split rows
                PQPP = ops.x3_linear(Pes, L["ppp_x3"], L["ppp_b"])         # k_t2i | v_t2i | q_i2t | img_patch_proj
                PQPP = PQPP.reshape(B * Np, -1)
                pq.append(PQPP[:, :3 * D])
                pp.append(PQPP[:, 3 * D:].contiguous())
            elif L["patch"].fp8_ok(B * Np):  # MX-fp8 (config 5): the LayerNorm emits the operand
                Pe, Pe8 = L["patch"](P, B, Np, eps, q8=True)
                pq.append(ops.linear_mxfp8(Pe8, L["p_w8"], L["p_b"]))
                pp.append(ops.linear_mxfp8(Pe8, L["pp_w8"], L["pp_b"]))
            else:
                Pe = L["patch"](P, B, Np, eps)                             # (B*Np, Ci) bf16
                pq.append(ops.linear(Pe, L["p_w"], L["p_b"]))              # (B*Np, 3D): k_t2i | v_t2i | q_i2t
                pp.append(ops.linear(Pe, L["pp_w"], L["pp_b"]))            # img_patch_proj
            e = torch.cuda.Event()
            e.record(cur)
            ev.append(e)
        return {"pq": pq, "pp": pp, "ev": ev, "stream": cur}

    def _patch_side(self, img_patches, patch_work):
        """(pq, pp, ev, two) for forward: the caller's early patch work, or the patch work run here on
        a side stream (side_streams, after the first call) or in line."""
        main = torch.cuda.current_stream(self.device)
        if patch_work is not None:
            if patch_work["stream"] != main:
                for t in patch_work["pq"] + patch_work["pp"]:
                    t.record_stream(main)
            return patch_work["pq"], patch_work["pp"], patch_work["ev"], True
        two = getattr(self, "_warm", False) and self.side_streams
        self._warm = True
        if not two:
            w = self.patch_work(img_patches)
            return w["pq"], w["pp"], w["ev"], False
        side = self._side_stream(main)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            w = self.patch_work(img_patches)
        img_patches.record_stream(side)
        for t in w["pq"] + w["pp"]:
            t.record_stream(main)
        return w["pq"], w["pp"], w["ev"], True

    def forward(self, img_global, img_patches, txt_feats, patch_work=None):
        """img_global (B, Ci) f32, img_patches (B, Np, Ci) f32, txt_feats (B, L, Ct) bf16/f32 or None
        -> joint_emb (B, D) f32.  patch_work: this batch's patch_work(img_patches), started early by the
        caller (else it runs here).

        Phase 1 (per layer, token level): enhancers, folded cross projections, the two cross
        attentions (means only where only means are used), patches_fused.
        Phase 2 (all layers in single launches): global enhancer, txt2img / img2txt out-projections
        of the means, ln_img / ln_txt — batched linears and grouped LayerNorms.
        Phase 3 (all layers together): sequence assembly, the shared self_attn QKV GEMM over
        nl*B*(Np+2) rows, its attention means and out-projection.
        Phase 4 (sequential): the joint chain (norm1 / alpha, norm2 -> FFN, adapter)."""
        if self.x3:
            return self._forward_x3(img_global, img_patches, txt_feats, patch_work)
        B, Np, Ci = img_patches.shape
        D, h, eps, dev = self.D, self.heads, self.eps, self.device
        nl = len(self.layers)
        dh = D // h
        sc = 1.0 / math.sqrt(dh)
        G = img_global.float().contiguous()
        m1 = torch.empty((nl, B, D), dtype=torch.float32, device=dev)
        m2 = torch.empty((nl, B, D), dtype=torch.float32, device=dev)
        PF = torch.empty((nl, B * Np, D), dtype=torch.bfloat16, device=dev)
        cls = None
        # the patch-side token work of every layer depends only on the image tower: it runs on a side
        # stream (or the caller's early patch_work), ahead of and concurrently with the text-side work,
        # which waits per layer on an event before the cross attentions (side_streams = False: one
        # stream; first call in sequence: see MultiModalRetrievalModel._towers)
        main = torch.cuda.current_stream(dev)
        pq, pp, ev, two = self._patch_side(img_patches, patch_work)
        for i, L in enumerate(self.layers):
            if txt_feats is None:  # learnable default text token (fusion.py:404-407)
                T, Lt = L["default_txt"].expand(B, -1).contiguous(), 1
            else:
                Lt = txt_feats.shape[1]
                T = txt_feats.to(torch.bfloat16).contiguous().view(B * Lt, -1)
            t8 = L["txt"].fp8_ok(B * Lt)
            if t8:
                Te, Te8 = L["txt"](T, B, Lt, eps, q8=True)
            else:
                Te = L["txt"](T, B, Lt, eps)                           # (B*Lt, Ct) bf16
            Ct = Te.shape[1]
            if cls is None:
                cls = torch.empty((nl, B, Ct), dtype=torch.float32, device=dev)
            ops.rows_to_f32(Te, B, Ct, Lt * Ct, out=cls[i])            # CLS rows (fusion.py:447)
            if t8:
                TQ = ops.linear_mxfp8(Te8, L["t_w8"], L["t_b"])
            else:
                TQ = ops.linear(Te, L["t_w"], L["t_b"])                # (B*Lt, 3D): q_t2i | k_i2t | v_i2t
            if two:
                main.wait_event(ev[i])
            PQ, PP = pq[i], pp[i]
            ops.mha(TQ[:, :D], PQ[:, :D], PQ[:, D:2 * D], B, Lt, Np, h, dh, sc, mean_out=m1[i])
            if self.fp8 and (B * Np) % 256 == 0 and D % 256 == 0 and dh % 32 == 0:  # the attention core emits the o2 operand
                _, _, a28 = ops.mha(PQ[:, 2 * D:], TQ[:, D:2 * D], TQ[:, 2 * D:], B, Np, Lt, h, dh, sc, mean_out=m2[i],
                                    q8=True)
                ops.linear_mxfp8(a28, L["o2_wb8"], L["o2_b"], residual=PP, out=PF[i])  # patches_fused (fusion.py:437)
            else:
                a2 = torch.empty((B * Np, D), dtype=torch.bfloat16, device=dev)
                ops.mha(PQ[:, 2 * D:], TQ[:, D:2 * D], TQ[:, 2 * D:], B, Np, Lt, h, dh, sc, out=a2, mean_out=m2[i])
                ops.linear(a2, L["o2_wb"], L["o2_b"], residual=PP, out=PF[i])  # patches_fused (fusion.py:437)
        del pq, pp
        return self._finish(G, m1, m2, cls, PF, B, Np, Ci)

    def _forward_x3(self, img_global, img_patches, txt_feats, patch_work=None):
        """Phase 1 of forward in the fp32-faithful mode: f32 token rows, every GEMM and attention on
        bf16x3 (ops.x3_linear / ops.x3_attention).  As in the bf16 path, the patch-side work of every
        layer (enhancer, folded k/v/q + patch projections) runs on a side stream (or early, by the
        caller) ahead of the text side, which waits per layer on an event before the cross attentions:
        the same kernels on the same operands, so the results are those of one stream."""
        B, Np, Ci = img_patches.shape
        D, h, eps, dev = self.D, self.heads, self.eps, self.device
        nl = len(self.layers)
        dh = D // h
        sc = 1.0 / math.sqrt(dh)
        G = img_global.float().contiguous()
        m1 = torch.empty((nl, B, D), dtype=torch.float32, device=dev)
        m2 = torch.empty((nl, B, D), dtype=torch.float32, device=dev)
        PF = torch.empty((nl, B * Np, D), dtype=torch.float32, device=dev)
        main = torch.cuda.current_stream(dev)
        pq, pp, ev, two = self._patch_side(img_patches, patch_work)
        cls = torch.empty((nl, B, self.layers[0]["txt"].C), dtype=torch.float32, device=dev)
        for i, L in enumerate(self.layers):
            PQ, PP = pq[i], pp[i]
            if txt_feats is None:  # learnable default text token (fusion.py:404-407)
                T, Lt = L["default_txt32"].expand(B, -1).contiguous(), 1
            else:
                Lt = txt_feats.shape[1]
                T = txt_feats.float().contiguous().view(B * Lt, -1)
            Te, Tes = L["txt"].x3(T, B, Lt, eps)                             # (B*Lt, Ct) f32 + split rows
            Ct = Te.shape[1]
            ops.x3_gather_rows(Te, B, Ct, Lt * Ct, out=cls[i])              # CLS rows (fusion.py:447)
            TQ = ops.x3_linear(Tes, L["t_x3"], L["t_b"]).reshape(B * Lt, -1)  # q_t2i | k_i2t | v_i2t
            if two:
                main.wait_event(ev[i])
            ops.x3_attention(TQ[:, :D], PQ[:, :D], PQ[:, D:2 * D], B, Lt, Np, h, dh, sc, mean_out=m1[i])
            a2 = ops.x3_attention_split(PQ[:, 2 * D:], TQ[:, D:2 * D], TQ[:, 2 * D:], B, Np, Lt, h, dh, sc,
                                        mean_out=m2[i])
            ops.x3_linear(a2, L["o2_x3t"], L["o2_b"], residual=PP, out=PF[i])  # patches_fused (fusion.py:437)
        del pq, pp
        return self._finish(G, m1, m2, cls, PF, B, Np, Ci)

    def _finish(self, G, m1, m2, cls, PF, B, Np, Ci):
        """Phases 2-4 of forward (shared by the bf16 / fp8 and x3 modes)."""
        D, h, eps, dev = self.D, self.heads, self.eps, self.device
        nl = len(self.layers)
        dh = D // h
        sc = 1.0 / math.sqrt(dh)
        # phase 2: per-query vectors of all layers
        Ge = self._ql(G, self.g_w_x3, self.g_b_all)               # (B, nl*Ci), layer-minor
        Ge = ops.ln_rows(Ge.view(B * nl, Ci), *self.g_ln_all, eps, groups=nl).view(B, nl * Ci)
        t2i = self._qlb(m1, self.o1_x3, self.o1_b_all, nl, B)              # mean_L att_txt2img
        x1 = self._qlb(Ge, self.gp_x3, self.gp_b_all, nl, B, residual=t2i, ldx=nl * Ci, bsx=Ci)
        x1 = ops.ln_rows(x1.view(nl * B, D), *self.ln_img_all, eps, groups=nl, group_div=B)
        i2t = self._qlb(m2, self.o2_x3, self.o2_b_all, nl, B)              # mean_Np att_img2txt
        x2 = self._qlb(cls, self.tp_x3, self.tp_b_all, nl, B, residual=i2t)
        x2 = ops.ln_rows(x2.view(nl * B, D), *self.ln_txt_all, eps, groups=nl, group_div=B)
        # phase 3: the shared combiner self-attention over every layer's fused sequence
        m3 = torch.empty((nl * B, D), dtype=torch.float32, device=dev)
        if self.x3:
            S = ops.x3_assemble_seq_split(x1, PF.view(nl * B * Np, D), x2, self.pe, Np)
            SQ = ops.x3_linear(S, self.s_x3, self.s_b).reshape(nl * B * (Np + 2), -1)
            ops.x3_attention(SQ[:, :D], SQ[:, D:2 * D], SQ[:, 2 * D:], nl * B, Np + 2, Np + 2, h, dh, sc, mean_out=m3)
        elif self.s_w8 is not None and (nl * B * (Np + 2)) % 256 == 0:
            S8 = ops.assemble_seq(x1, PF.view(nl * B * Np, D), x2, self.pe, Np, q8=True)
            SQ = ops.linear_mxfp8(S8, self.s_w8, self.s_b)
        else:
            S = ops.assemble_seq(x1, PF.view(nl * B * Np, D), x2, self.pe, Np).view(nl * B * (Np + 2), D)
            SQ = ops.linear(S, self.s_w, self.s_b)
        if not self.x3:
            ops.mha(SQ[:, :D], SQ[:, D:2 * D], SQ[:, 2 * D:], nl * B, Np + 2, Np + 2, h, dh, sc, mean_out=m3)
        fused = self._ql(m3, self.s_ow_x3, self.s_ob).view(nl, B, D)  # mean of self_attn output
        # phase 4: the joint chain
        joint = None
        for i, L in enumerate(self.layers):
            if i == 0:
                x = fused[0]
            else:  # norm1(joint) + alpha * fused  (StochasticDepth in eval = plain residual)
                x = ops.ln_rows(joint, *L["n1"], eps, post=fused[i], post_scale=self.alpha)
            xf = ops.ln_rows(x, *L["n2"], eps)
            _, b1, _, b2 = L["ffn"]
            w1, w2 = L["ffn_x3"]
            self._ql(self._ql(xf, w1, b1, act=1), w2, b2, residual=x, out=x)
            _, c1, _, c2 = L["ad"]
            a1, a2 = L["ad_x3"]
            self._ql(self._ql(x, a1, c1, act=1), a2, c2, residual=x, out=x)
            joint = x
        return joint.contiguous()
