"""Encoder API — mirrors src/Model/fusion.py `Backbones` and src/Model/model.py
`MultiModalRetrievalModel` for the Swin + ClinicalBERT branches, on libmmr kernels.

Backbones.forward(image, input_ids, attention_mask) -> ((img_global, img_patches), txt_feats)
    fusion.py:255-327: img_patches = swin_norm(patch_feats) — swin_norm IS the Swin's own final
    norm, so patches are LayerNorm'd twice — and img_global = mean of the once-normed tokens;
    txt_feats = BertModel(...).last_hidden_state (truncated to max_position_embeddings).
MultiModalRetrievalModel.forward(...) -> {"joint_emb", "img_emb", "txt_emb", "logits", "attn"}
    model.py:365-373: img_emb = img_proj(img_global); txt_emb = txt_proj(mean over ALL L tokens,
    PAD included) (CLS only with use_cls_only).
    model.py:462-479 heads: "text"  joint = ffn0(txt_proj(mean(txt)))
                            "image" joint = ffn0(mean(cat[img_proj(g), img_proj(p)]))
                                          = ffn0(img_proj(mean(cat[g, p])))  (affine proj)
    ffn0 = MultiHeadMLP (Linear D->2D, GELU, Linear 2D->D), model.py:61-75; shared_ffn when
    use_shared_ffn (reference default True, configs/config.yaml false).
    "multimodal" (5x CrossModalFusion, fusion.py:334-471) is the next row of SURVEY.md §8f and
    raises NotImplementedError; the classifier (logits) is classification, out of scope -> None.
"""
import torch

from . import ops
from .towers import BERT_BASE, SWIN_T, BertTower, SwinTower, init_bert_state, init_swin_state


def _sub(sd, prefix):
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


class Backbones:
    def __init__(self, img_backbone="swin", swin_state=None, bert_state=None, swin_cfg=None, bert_cfg=None,
                 device="cuda", pretrained=False, seed=2709):
        if img_backbone != "swin":
            raise ValueError(f"image backbone {img_backbone!r} is outside the accelerated path (swin only)")
        self.img_backbone = img_backbone
        self.device = torch.device(device)
        swin_cfg = dict(SWIN_T, **(swin_cfg or {}))
        bert_cfg = dict(BERT_BASE, **(bert_cfg or {}))
        self.vision = SwinTower(swin_state if swin_state is not None else init_swin_state(swin_cfg, seed),
                                swin_cfg, self.device)
        self.swin = self.vision
        self.bert = BertTower(bert_state if bert_state is not None else init_bert_state(bert_cfg, seed + 1),
                              bert_cfg, self.device)
        self.img_dim = self.vision.num_features
        self.txt_dim = self.bert.hidden

    # fast path: bf16 hidden states + fused pooling, no f32 copies of the full token grids
    def encode_image(self, image, want_patches=True):
        tok = self.vision.tokens(image)
        B, H, W, C = tok.shape
        patches, glob, pool = ops.swin_head(tok.view(B, H * W, C), self.vision.norm_g, self.vision.norm_b, 1e-5,
                                            want_patches=want_patches)
        return glob, patches, pool

    def encode_text(self, input_ids, attention_mask=None):
        return self.bert.forward(input_ids, attention_mask)

    def swin_features(self, image):
        return self.vision.forward_features(image).float()

    def forward(self, image, input_ids=None, attention_mask=None):
        img_global = img_patches = None
        if image is not None:
            img_global, img_patches, _ = self.encode_image(image)
        txt_feats = None
        if input_ids is not None:
            txt_feats = self.encode_text(input_ids, attention_mask).float()
        return (img_global, img_patches), txt_feats

    __call__ = forward

    def extract_global(self, image):
        (g, _), _ = self.forward(image)
        return g


class MultiModalRetrievalModel:
    def __init__(self, joint_dim=256, num_heads=4, model_type="multimodal", use_shared_ffn=False,
                 use_cls_only=False, backbones=None, head_state=None, device="cuda", retriever=None,
                 swin_cfg=None, bert_cfg=None, seed=2709):
        if model_type not in ("multimodal", "image", "text"):
            raise ValueError(f"Unknown model_type {model_type!r}")
        self.model_type = model_type
        self.device = torch.device(device)
        self.backbones = backbones or Backbones(swin_cfg=swin_cfg, bert_cfg=bert_cfg, device=device, seed=seed)
        self.joint_dim = joint_dim
        self.use_shared_ffn = use_shared_ffn
        self.use_cls_only = use_cls_only
        self.retriever = retriever
        hs = head_state if head_state is not None else init_head_state(self.backbones.img_dim,
                                                                       self.backbones.txt_dim, joint_dim, seed + 2)
        f = lambda k: hs[k].detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        self.img_proj = (f("img_proj.weight"), f("img_proj.bias"))
        self.txt_proj = (f("txt_proj.weight"), f("txt_proj.bias"))
        pre = "shared_ffn." if use_shared_ffn else "ffn.0."
        self.ffn = (f(pre + "linear1.weight"), f(pre + "linear1.bias"), f(pre + "linear2.weight"), f(pre + "linear2.bias"))

    @classmethod
    def from_reference_state_dict(cls, sd, swin_cfg, bert_cfg, joint_dim, model_type="text", device="cuda",
                                  use_shared_ffn=False):
        """Build from a reference checkpoint state dict (model.py:282-287 layout)."""
        vis = _sub(sd, "backbones.vision.")
        bb = Backbones(swin_state=vis, bert_state=_sub(sd, "backbones.bert."), swin_cfg=swin_cfg,
                       bert_cfg=bert_cfg, device=device)
        return cls(joint_dim=joint_dim, model_type=model_type, backbones=bb, head_state=sd, device=device,
                   use_shared_ffn=use_shared_ffn)

    def set_retriever(self, retriever):
        self.retriever = retriever

    def _txt_pool(self, hidden):
        return hidden[:, 0, :].float().contiguous() if self.use_cls_only else ops.mean_tokens(hidden)

    def _head(self, x, proj, l2norm=False):
        return ops.proj_head(x, proj[0], proj[1], *self.ffn, l2norm=l2norm)

    def forward(self, image, input_ids, attention_mask, return_attention=False):
        if self.model_type == "multimodal":
            raise NotImplementedError("multimodal fusion stack (fusion.py:334-471) is SURVEY.md §8f row 1 (next)")
        img_global = pool = txt_mean = None
        if image is not None:
            img_global, _, pool = self.backbones.encode_image(image, want_patches=False)
        if input_ids is not None:
            txt_mean = self._txt_pool(self.backbones.encode_text(input_ids, attention_mask))
        img_emb = ops.proj_head(img_global, *self.img_proj) if img_global is not None else None
        txt_emb = ops.proj_head(txt_mean, *self.txt_proj) if txt_mean is not None else None
        if self.model_type == "image":
            joint = self._head(pool, self.img_proj)
        else:
            joint = self._head(txt_mean, self.txt_proj)
        return {"joint_emb": joint, "img_emb": img_emb, "txt_emb": txt_emb, "logits": None, "attn": None}

    __call__ = forward

    def query_embeddings(self, image, input_ids, attention_mask):
        """Both single-modality heads on one (image, report) batch: (2B, D) f32 = [image-head joint
        embeddings; text-head joint embeddings] — the retrieval keys of model_type image / text."""
        _, _, pool = self.backbones.encode_image(image, want_patches=False)
        txt_mean = self._txt_pool(self.backbones.encode_text(input_ids, attention_mask))
        return torch.cat([self._head(pool, self.img_proj), self._head(txt_mean, self.txt_proj)], 0)


def init_head_state(img_dim, txt_dim, joint_dim, seed=2711):
    g = torch.Generator().manual_seed(seed)

    def rn(*shape):
        return torch.randn(*shape, generator=g) * 0.02
    D = joint_dim
    sd = {"img_proj.weight": rn(D, img_dim), "img_proj.bias": rn(D),
          "txt_proj.weight": rn(D, txt_dim), "txt_proj.bias": rn(D)}
    for pre in ("ffn.0.", "shared_ffn."):
        sd.update({pre + "linear1.weight": rn(2 * D, D), pre + "linear1.bias": rn(2 * D),
                   pre + "linear2.weight": rn(D, 2 * D), pre + "linear2.bias": rn(D)})
    return sd


def build_bench_model(device="cuda", joint_dim=768, seed=2709):
    """Swin-Tiny + ClinicalBERT-base geometry, random init (no checkpoints offline)."""
    return MultiModalRetrievalModel(joint_dim=joint_dim, model_type="text", device=device, seed=seed)
