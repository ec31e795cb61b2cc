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
    "multimodal" = num_fusion_layers x CrossModalFusion (fusion.py:334-471) + combiner
    (model.py:375-459) on libmmr kernels (mmr_amd/fusion.py); the classifier (logits) is
    classification, out of scope -> None; attention maps (return_attention) are not produced.
"""
import collections
import json
import os
from pathlib import Path

import torch

from . import ops
from .fusion import FusionStack
from .towers import BERT_BASE, SWIN_T, SWIN_ARCHS, BertTower, SwinTower, init_bert_state, init_swin_state
from .towers_x3 import BertTowerX3, SwinTowerX3


def _sub(sd, prefix):
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


def _load_tensors(path):
    """A weights file as a state dict, executing nothing from it: .safetensors via safetensors,
    anything else via torch.load(..., weights_only=True) (a dict, or {"state_dict" / "model": dict})."""
    path = str(path)
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path, device="cpu")
    sd = torch.load(path, map_location="cpu", weights_only=True)
    for key in ("state_dict", "model"):
        if isinstance(sd, dict) and key in sd and isinstance(sd[key], dict):
            sd = sd[key]
    return sd


def swin_cfg_from_state(sd, base=None):
    """timm Swin geometry read off a timm-keyed state dict (embed dim, depths, heads per stage,
    window), so a checkpoint of any Swin size builds the matching tower."""
    cfg = dict(base or SWIN_T)
    if "patch_embed.proj.weight" not in sd:
        return cfg
    cfg["embed_dim"] = int(sd["patch_embed.proj.weight"].shape[0])
    depths, heads = [], []
    i = 0
    while any(k.startswith(f"layers.{i}.") for k in sd):
        j = 0
        while f"layers.{i}.blocks.{j}.norm1.weight" in sd:
            j += 1
        depths.append(j)
        heads.append(int(sd[f"layers.{i}.blocks.0.attn.relative_position_bias_table"].shape[1]))
        i += 1
    if depths:
        cfg["depths"], cfg["num_heads"] = depths, heads
        t = int(sd["layers.0.blocks.0.attn.relative_position_bias_table"].shape[0])
        cfg["window_size"] = (int(round(t ** 0.5)) + 1) // 2
    return cfg


def bert_cfg_from_state(sd, user=None):
    """BERT geometry read off an HF BertModel state dict (user keys override nothing the weights
    fix); heads are not visible in the weights: the user's / config.json's num_attention_heads,
    else hidden / 64 (every BERT-family checkpoint of the reference; Bio_ClinicalBERT: 12)."""
    user = dict(user or {})
    cfg = dict(BERT_BASE, **user)
    if "embeddings.word_embeddings.weight" not in sd:
        return cfg
    v, h = sd["embeddings.word_embeddings.weight"].shape
    n = 0
    while f"encoder.layer.{n}.attention.self.query.weight" in sd:
        n += 1
    cfg.update(vocab_size=int(v), hidden_size=int(h), num_hidden_layers=n,
               intermediate_size=int(sd["encoder.layer.0.intermediate.dense.weight"].shape[0]),
               max_position_embeddings=int(sd["embeddings.position_embeddings.weight"].shape[0]),
               type_vocab_size=int(sd["embeddings.token_type_embeddings.weight"].shape[0]))
    cfg["num_attention_heads"] = int(user.get("num_attention_heads", max(1, int(h) // 64)))
    return cfg


def load_bert_dir(local_dir):
    """Helpers/model_utils.py:11-55 local branch (AutoModel.from_pretrained(local_dir)) without
    transformers: config.json for the geometry + model.safetensors / pytorch_model.bin weights
    (a "bert." prefix of BertFor* checkpoints is stripped).  Nothing is downloaded."""
    d = Path(local_dir)
    cfg = {}
    if (d / "config.json").exists():
        c = json.loads((d / "config.json").read_text())
        cfg = {k: c[k] for k in ("vocab_size", "hidden_size", "num_hidden_layers", "num_attention_heads",
                                 "intermediate_size", "max_position_embeddings", "type_vocab_size") if k in c}
    for name in ("model.safetensors", "pytorch_model.bin"):
        if (d / name).exists():
            sd = _load_tensors(d / name)
            if any(k.startswith("bert.") for k in sd):
                sd = _sub(sd, "bert.")
            return sd, cfg
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin in {d}")


class Backbones:
    """src/Model/fusion.py:37-332 Backbones (Swin + ClinicalBERT branches) on libmmr kernels.

    Reference arguments (fusion.py:42-53), same names and order: img_backbone ('swin' only — the
    CNN / MedCLIP branches are outside the accelerated path), swin_model_name (a timm Swin name:
    its geometry, SWIN_ARCHS), cnn_model_name (accepted, unused), bert_model_name,
    swin_checkpoint_path (timm-keyed weights, .safetensors or a torch state dict), bert_local_dir
    (an HF save_pretrained directory, Helpers/model_utils.py:11-55), pretrained, img_dim, txt_dim.
    There is no hub access: pretrained=True needs swin_checkpoint_path / bert_local_dir (or the
    explicit states below); pretrained=False builds seeded random weights (the benchmark).
    The reference collapses patch_embed.proj.weight to one input channel before loading
    (fusion.py:92-96), which cannot load into its in_chans=3 model (it falls back to a download,
    :101-107); here a 3-channel weight loads as is and a 1-channel weight w is expanded to w/3 per
    channel (the same response on the grey-replicated inputs, tensorDICOM.py:150).
    Extras (keyword-only): swin_state / bert_state (state dicts), swin_cfg / bert_cfg (geometry
    overrides), device, seed, tower_dtype ("bf16" configs 1-4, "fp8" config 5: MX-fp8 linears in
    every BERT layer and Swin stages 3-4, "x3": the fp32-faithful parity mode — f32 activations,
    every contraction on bf16x3 MFMA, towers_x3.py)."""

    def __init__(self, img_backbone="swin", swin_model_name="swin_base_patch4_window7_224", cnn_model_name="resnet50",
                 bert_model_name="emilyalsentzer/Bio_ClinicalBERT", swin_checkpoint_path=None, bert_local_dir=None,
                 pretrained=True, img_dim=None, txt_dim=None, *, swin_state=None, bert_state=None, swin_cfg=None,
                 bert_cfg=None, device="cuda", seed=2709, tower_dtype="bf16"):
        if tower_dtype not in ("bf16", "fp8", "x3"):
            raise ValueError(f"tower_dtype {tower_dtype!r}: bf16, fp8 or x3")
        self.tower_dtype = tower_dtype
        if img_backbone != "swin":
            raise ValueError(f"image backbone {img_backbone!r} is outside the accelerated path (swin only)")
        self.img_backbone = img_backbone
        self.swin_model_name, self.bert_model_name = swin_model_name, bert_model_name
        self.device = torch.device(device)
        arch = SWIN_ARCHS.get(swin_model_name)
        # fusion.py:83: the checkpoint is read only when pretrained (pretrained=False builds random weights)
        if swin_state is None and swin_checkpoint_path and pretrained:
            if not Path(str(swin_checkpoint_path)).exists():
                raise FileNotFoundError(f"Swin checkpoint not found at {swin_checkpoint_path} (no hub access here)")
            swin_state = _load_tensors(swin_checkpoint_path)
        if swin_state is not None:
            w = swin_state.get("patch_embed.proj.weight")
            if w is not None and w.shape[1] == 1:
                swin_state = dict(swin_state, **{"patch_embed.proj.weight": w.expand(-1, 3, -1, -1) / 3.0})
            swin_cfg = dict(swin_cfg_from_state(swin_state, arch), **(swin_cfg or {}))
        else:
            if pretrained and swin_cfg is None:
                raise ValueError(f"pretrained Swin {swin_model_name!r} needs swin_checkpoint_path (no hub access)")
            if swin_cfg is None and arch is None:
                raise ValueError(f"unknown Swin name {swin_model_name!r}: pass swin_cfg (known: {sorted(SWIN_ARCHS)})")
            swin_cfg = dict(arch or SWIN_T, **(swin_cfg or {}))
            swin_state = init_swin_state(swin_cfg, seed)
        if bert_state is None and bert_local_dir:
            bert_state, dir_cfg = load_bert_dir(bert_local_dir)
            bert_cfg = dict(dir_cfg, **(bert_cfg or {}))
        if bert_state is not None:
            bert_cfg = bert_cfg_from_state(bert_state, bert_cfg)
        else:
            if pretrained and bert_cfg is None:
                raise ValueError(f"pretrained {bert_model_name!r} needs bert_local_dir (no hub access)")
            bert_cfg = dict(BERT_BASE, **(bert_cfg or {}))
            bert_state = init_bert_state(bert_cfg, seed + 1)
        fp8 = tower_dtype == "fp8"
        self.swin_cfg, self.bert_cfg = swin_cfg, bert_cfg
        if tower_dtype == "x3":  # fp32-faithful mode (towers_x3.py): f32 activations, bf16x3 contractions
            self.vision = SwinTowerX3(swin_state, swin_cfg, self.device)
            self.bert = BertTowerX3(bert_state, bert_cfg, self.device)
        else:
            self.vision = SwinTower(swin_state, swin_cfg, self.device, fp8_stages=(2, 3) if fp8 else ())
            self.bert = BertTower(bert_state, bert_cfg, self.device, fp8=fp8)
        self.swin = self.vision
        self.img_dim = self.vision.num_features if img_dim is None else img_dim
        self.txt_dim = self.bert.hidden if txt_dim is None else txt_dim
        if self.img_dim != self.vision.num_features or self.txt_dim != self.bert.hidden:
            raise ValueError(f"img_dim/txt_dim {self.img_dim}/{self.txt_dim} differ from the towers' "
                             f"{self.vision.num_features}/{self.bert.hidden}")

    # fast path: bf16 hidden states + fused pooling, no f32 copies of the full token grids
    def encode_image(self, image, want_patches=True):
        tok = self.vision.tokens(image)
        if self.tower_dtype == "x3":
            return self.vision.head(tok)
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
    """src/Model/model.py:114-328 MultiModalRetrievalModel (inference) on libmmr kernels.

    Reference arguments (model.py:116-137), same names, order and defaults: joint_dim, num_heads,
    num_classes (the classifier is classification, out of scope: accepted, logits None),
    num_fusion_layers, fusion_type ("cross" only, as in the reference), img_backbone, swin_name,
    cnn_name, bert_name, img_dim, txt_dim, swin_ckpt_path, bert_local_dir, pretrained,
    checkpoint_path (a state dict of the whole reference model, loaded with torch.load(...,
    weights_only=True) as model.py:282-287 loads it — tower and head weights; geometry read off
    it), device (a GPU: there is no CPU path; default "cuda"), training (False: like the
    reference, weights must come from checkpoint_path — or head_state / backbones below — else
    ValueError, model.py:288-289), use_shared_ffn, use_cls_only, model_type, retriever (with
    training=False and no retriever: a DLS engine over $MMR_EMBEDDINGS_DIR/val_joint_embeddings.npy
    + val_ids.json when that directory is set, as model.py:294-312 does over EMBEDDINGS_DIR).
    Extras (keyword-only): backbones (a built Backbones), head_state (head / fusion weights under
    the reference's keys), swin_cfg / bert_cfg, seed, tower_dtype."""

    def __init__(self, joint_dim=256, num_heads=4, num_classes=22, num_fusion_layers=3, fusion_type="cross",
                 img_backbone="swin", swin_name="swin_base_patch4_window7_224", cnn_name="resnet50",
                 bert_name="emilyalsentzer/Bio_ClinicalBERT", img_dim=None, txt_dim=None, swin_ckpt_path=None,
                 bert_local_dir=None, pretrained=True, checkpoint_path=None, device="cuda", training=False,
                 use_shared_ffn=True, use_cls_only=False, model_type="multimodal", retriever=None, *,
                 backbones=None, head_state=None, swin_cfg=None, bert_cfg=None, seed=2709, tower_dtype="bf16"):
        if model_type not in ("multimodal", "image", "text"):
            raise ValueError(f"Unknown model_type {model_type!r}")
        if fusion_type != "cross":
            raise ValueError(f"Unknown fusion_type {fusion_type!r}")
        self.model_type = model_type
        self.device = torch.device(device)
        sd = None
        if checkpoint_path:
            sd = _load_tensors(checkpoint_path)
            if any(k.startswith("module.") for k in sd):  # DataParallel-saved
                sd = _sub(sd, "module.")
        elif not training and head_state is None:
            raise ValueError("checkpoint_path must be provided for inference")
        if backbones is None:
            if sd is not None:
                backbones = Backbones(img_backbone, swin_name, cnn_name, bert_name, None, None, False, img_dim, txt_dim,
                                      swin_state=_sub(sd, "backbones.vision."), bert_state=_sub(sd, "backbones.bert."),
                                      swin_cfg=swin_cfg, bert_cfg=bert_cfg, device=device, seed=seed,
                                      tower_dtype=tower_dtype)
            else:
                backbones = Backbones(img_backbone, swin_name, cnn_name, bert_name, swin_ckpt_path, bert_local_dir,
                                      pretrained and (swin_ckpt_path is not None or bert_local_dir is not None),
                                      img_dim, txt_dim, swin_cfg=swin_cfg, bert_cfg=bert_cfg, device=device, seed=seed,
                                      tower_dtype=tower_dtype)
        self.backbones = backbones
        self.joint_dim = joint_dim
        self.num_classes = num_classes
        self.use_shared_ffn = use_shared_ffn
        self.use_cls_only = use_cls_only
        self.retriever = retriever
        self._side = None
        self._warm = False
        self.concurrent_towers = True  # Swin tower on a side stream beside BERT (False: in sequence)
        hs = head_state if head_state is not None else sd
        if hs is None:  # training=True without a checkpoint: seeded random init (the reference's fresh model)
            hs = init_head_state(self.backbones.img_dim, self.backbones.txt_dim, joint_dim, seed + 2)
            if model_type == "multimodal":
                hs.update(init_fusion_state(self.backbones.img_dim, self.backbones.txt_dim, joint_dim, num_heads,
                                            num_fusion_layers, seed + 3, use_shared_ffn=use_shared_ffn))
        f = lambda k: hs[k].detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        self.img_proj = (f("img_proj.weight"), f("img_proj.bias"))
        self.txt_proj = (f("txt_proj.weight"), f("txt_proj.bias"))
        if self.img_proj[0].shape[0] != joint_dim:
            raise ValueError(f"joint_dim {joint_dim} does not match the weights' {self.img_proj[0].shape[0]}")
        pre = "shared_ffn." if use_shared_ffn else "ffn.0."
        self.ffn = (f(pre + "linear1.weight"), f(pre + "linear1.bias"), f(pre + "linear2.weight"), f(pre + "linear2.bias"))
        self.num_heads = num_heads
        self.fusion = None
        if model_type == "multimodal":
            if use_cls_only:  # model.py:428-429 indexes the 2-D comb_mlp output: the reference raises
                raise ValueError("model_type='multimodal' with use_cls_only fails in the reference (model.py:428)")
            if not any(k.startswith("fusion_layers.") for k in hs):
                raise ValueError("head_state has no fusion_layers.* weights for model_type='multimodal'")
            nfl = len({k.split(".")[1] for k in hs if k.startswith("fusion_layers.")})
            if nfl != num_fusion_layers and (checkpoint_path or head_state is not None):
                num_fusion_layers = nfl  # the weights decide (a checkpoint of another depth)
            self.fusion = FusionStack(hs, num_heads, device=self.device, use_shared_ffn=use_shared_ffn,
                                      tower_dtype=getattr(self.backbones, "tower_dtype", tower_dtype))
        self.num_fusion_layers = num_fusion_layers
        if self.retriever is None and not training and os.environ.get("MMR_EMBEDDINGS_DIR"):
            from .retrieval import make_retrieval_engine
            d = Path(os.environ["MMR_EMBEDDINGS_DIR"])
            fp, ip = d / "val_joint_embeddings.npy", d / "val_ids.json"
            if not fp.exists() or not ip.exists():
                raise FileNotFoundError(f"Expected embeddings at {fp} and IDs at {ip}")
            self.retriever = make_retrieval_engine(str(fp), str(ip), method="dls", link_threshold=0.5, max_links=10)

    @classmethod
    def from_reference_state_dict(cls, sd, swin_cfg=None, bert_cfg=None, joint_dim=None, model_type="text",
                                  device="cuda", use_shared_ffn=False, num_heads=4, tower_dtype="bf16"):
        """Build from a reference model state dict (the model.py:282-287 layout) already in memory."""
        vis = _sub(sd, "backbones.vision.")
        bb = Backbones(pretrained=False, swin_state=vis, bert_state=_sub(sd, "backbones.bert."), swin_cfg=swin_cfg,
                       bert_cfg=bert_cfg, device=device, tower_dtype=tower_dtype)
        jd = joint_dim or int(sd["img_proj.weight"].shape[0])
        return cls(joint_dim=jd, num_heads=num_heads, model_type=model_type, backbones=bb, head_state=sd,
                   device=device, use_shared_ffn=use_shared_ffn, training=True)

    def set_retriever(self, retriever):
        self.retriever = retriever

    def _txt_pool(self, hidden):
        if self.use_cls_only:
            return hidden[:, 0, :].float().contiguous()
        return ops.x3_mean_rows(hidden) if hidden.dtype == torch.float32 else ops.mean_tokens(hidden)

    def _head(self, x, proj, l2norm=False):
        return ops.proj_head(x, proj[0], proj[1], *self.ffn, l2norm=l2norm)

    def forward(self, image, input_ids, attention_mask, return_attention=False):
        mm = self.model_type == "multimodal"
        img_global = patches = pool = txt_mean = txt = None
        if image is not None:
            img_global, patches, pool = self.backbones.encode_image(image, want_patches=mm)
        elif mm:  # CrossModalFusion unpacks img_patch.shape (fusion.py:421): the reference needs the image
            raise ValueError("model_type='multimodal' needs an image (fusion.py:421)")
        if input_ids is not None:
            txt = self.backbones.encode_text(input_ids, attention_mask)
            txt_mean = self._txt_pool(txt)
        img_emb = ops.proj_head(img_global, *self.img_proj) if img_global is not None else None
        txt_emb = ops.proj_head(txt_mean, *self.txt_proj) if txt_mean is not None else None
        if mm:
            joint = self.fusion.forward(img_global, patches, txt)
        elif self.model_type == "image":
            joint = self._head(pool, self.img_proj)
        else:
            joint = self._head(txt_mean, self.txt_proj)
        return {"joint_emb": joint, "img_emb": img_emb, "txt_emb": txt_emb, "logits": None, "attn": None}

    __call__ = forward

    def query_embeddings(self, image, input_ids, attention_mask):
        """Retrieval keys of one batch.  multimodal: (B, D) f32 joint embeddings of (image, report)
        pairs; image / text with both inputs: both single-modality heads, (2B, D) = [image-head;
        text-head]; text with image=None: the text tower + text head only, (B, D) (BASELINE cfg3:
        text-only ClinicalBERT queries, model.py:472-479); image with input_ids=None: the image
        tower + image head only (model.py:462-469)."""
        mm = self.model_type == "multimodal"
        if not mm and image is None:
            txt = self.backbones.encode_text(input_ids, attention_mask)
            return self._head(self._txt_pool(txt), self.txt_proj)
        if not mm and input_ids is None:
            _, _, pool = self.backbones.encode_image(image, want_patches=False)
            return self._head(pool, self.img_proj)
        # multimodal: the fusion stack's patch-side work (image tower only) starts on the towers'
        # side stream as soon as the Swin tower is done, beside the BERT tower's tail
        early = (lambda img: self.fusion.patch_work(img[1])) if mm and self.fusion.side_streams else None
        (g, p, pool), txt, pw = self._towers(image, input_ids, attention_mask, mm, after_image=early)
        if mm:
            return self.fusion.forward(g, p, txt, patch_work=pw)
        return torch.cat([self._head(pool, self.img_proj), self._head(self._txt_pool(txt), self.txt_proj)], 0)

    def _towers(self, image, input_ids, attention_mask, want_patches, after_image=None):
        """Both towers, the Swin tower on a side stream so its kernels fill the CUs the BERT
        kernels leave idle (wave-quantisation tails, small LayerNorm / attention launches); the
        two towers share no data until the heads.  The first call runs them in sequence: the GEMM
        launcher times its variants per shape on first use, which concurrent kernels would skew.
        concurrent_towers = False always runs them in sequence.  after_image(img) runs on the side
        stream right after the image tower (its result is returned third; None in sequence)."""
        first = not self._warm
        self._warm = True
        if first or not self.concurrent_towers:
            return (self.backbones.encode_image(image, want_patches=want_patches),
                    self.backbones.encode_text(input_ids, attention_mask), None)
        main = torch.cuda.current_stream(self.device)
        # one side stream per calling stream: callers that pipeline batches over several streams
        # (bench.py --pipeline) keep their batches independent
        if self._side is None:
            self._side = collections.OrderedDict()
        side = ops.side_stream(self._side, main, self.device)
        side.wait_stream(main)                        # the image batch is ready
        with torch.cuda.stream(side):
            img = self.backbones.encode_image(image, want_patches=want_patches)
            img_done = torch.cuda.Event()
            img_done.record(side)
            extra = after_image(img) if after_image is not None else None  # carries its own events
        image.record_stream(side)                     # caching allocator: in use on the side stream
        txt = self.backbones.encode_text(input_ids, attention_mask)
        main.wait_event(img_done)                     # the image tower, not the early work after it
        for t in img:
            if t is not None:
                t.record_stream(main)
        return img, txt, extra


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


def init_fusion_state(img_dim, txt_dim, joint_dim, num_heads=8, num_fusion_layers=5, seed=2712,
                      pos_len=512, use_shared_ffn=False):
    """Random weights under the reference's key names for the multimodal head (fusion_layers.*,
    self_attn, norm1/2_layers, pos_encoder, alpha, ffn.i / shared_ffn, adapters.i); nn.Linear-like
    fan-in scaling, LayerNorm affine near identity, positional tables std 0.02."""
    g = torch.Generator().manual_seed(seed)
    D = joint_dim

    def lin(sd, p, o, i):
        sd[p + ".weight"] = torch.randn(o, i, generator=g) * i ** -0.5
        sd[p + ".bias"] = torch.randn(o, generator=g) * 0.02

    def ln(sd, p, c):
        sd[p + ".weight"] = 1 + 0.05 * torch.randn(c, generator=g)
        sd[p + ".bias"] = 0.05 * torch.randn(c, generator=g)

    def mha(sd, p, e):
        sd[p + "in_proj_weight"] = torch.randn(3 * e, e, generator=g) * e ** -0.5
        sd[p + "in_proj_bias"] = torch.randn(3 * e, generator=g) * 0.02
        lin(sd, p + "out_proj", e, e)

    sd = {}
    for i in range(num_fusion_layers):
        p = f"fusion_layers.{i}."
        for name, c in (("txt_self_attn.", txt_dim), ("img_patch_self_attn.", img_dim), ("img_global_self_attn.", img_dim)):
            sd[p + name + "pos_embed"] = torch.randn(1, pos_len, c, generator=g) * 0.02
            mha(sd, p + name + "self_attn.", c)
            ln(sd, p + name + "norm1", c)
            sd[p + name + "alpha"] = torch.ones(1)
        ln(sd, p + "ln_img", D)
        ln(sd, p + "ln_txt", D)
        for name, c in (("query_txt", txt_dim), ("key_img", img_dim), ("value_img", img_dim), ("query_img", img_dim),
                        ("key_txt", txt_dim), ("value_txt", txt_dim), ("txt_proj", txt_dim),
                        ("img_patch_proj", img_dim), ("img_global_proj", img_dim)):
            lin(sd, p + name, D, c)
        mha(sd, p + "attn_txt2img.", D)
        mha(sd, p + "attn_img2txt.", D)
        sd[p + "default_txt_token"] = torch.randn(1, 1, txt_dim, generator=g) * 0.02
        lin(sd, p + "comb_mlp.0", D, 3 * D)
        lin(sd, p + "comb_mlp.3", D, D)
        ln(sd, f"norm1_layers.{i}", D)
        ln(sd, f"norm2_layers.{i}", D)
        if not use_shared_ffn:
            lin(sd, f"ffn.{i}.linear1", 2 * D, D)
            lin(sd, f"ffn.{i}.linear2", D, 2 * D)
        lin(sd, f"adapters.{i}.0", D // 2, D)
        lin(sd, f"adapters.{i}.2", D, D // 2)
    mha(sd, "self_attn.", D)
    sd["alpha"] = torch.ones(1)
    sd["pos_encoder.pe"] = torch.randn(1, txt_dim, D, generator=g) * 0.02
    if use_shared_ffn:
        lin(sd, "shared_ffn.linear1", 2 * D, D)
        lin(sd, "shared_ffn.linear2", D, 2 * D)
    return sd


def build_bench_model(device="cuda", joint_dim=768, seed=2709, model_type="multimodal", num_heads=8,
                      num_fusion_layers=5, tower_dtype="bf16"):
    """Swin-Tiny + ClinicalBERT-base geometry, random init (no checkpoints offline); multimodal head
    with configs/config.yaml's num_heads 8 / num_fusion_layers 5 at joint_dim 768 (config 5: 1024,
    tower_dtype "fp8")."""
    hs = init_head_state(768, 768, joint_dim, seed + 2)
    if model_type == "multimodal":
        hs.update(init_fusion_state(768, 768, joint_dim, num_heads, num_fusion_layers, seed + 3))
    bb = Backbones("swin", "swin_tiny_patch4_window7_224", pretrained=False, device=device, seed=seed,
                   tower_dtype=tower_dtype)
    return MultiModalRetrievalModel(joint_dim=joint_dim, num_heads=num_heads, num_fusion_layers=num_fusion_layers,
                                    model_type=model_type, backbones=bb, head_state=hs, device=device, seed=seed,
                                    use_shared_ffn=False, training=True, tower_dtype=tower_dtype)
