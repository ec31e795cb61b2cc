"""CPU: the host side of the drop-in boundary (no GPU calls).

* constructor signatures mirror the reference's (src/Model/fusion.py:42-53 Backbones,
  src/Model/model.py:116-137 MultiModalRetrievalModel) — names, order, defaults;
* make_retrieval_engine defaults to method="dls" (src/Retrieval/retrieval.py:276);
* checkpoint geometry: a reference-layout state dict (tests/golden/towers_mini.npz re-keyed to
  backbones.vision.* / backbones.bert.* / head keys, the model.py:282-287 layout) saved with
  torch.save and re-read with weights_only=True yields the golden's Swin / BERT geometry;
* the memmap-preserving engine base (ShardedRetrievalEngine keeps the .npy mapped);
* the host shard merge carries a payload; the host rerank mix equals oracle/dls.rerank.
"""
import inspect
import json
import os

import numpy as np
import torch

from mmr_amd import synthetic
from mmr_amd.model import Backbones, MultiModalRetrievalModel, _load_tensors, bert_cfg_from_state, swin_cfg_from_state
from mmr_amd.parallel import merge_topk_host, rerank_mix_host
from mmr_amd.retrieval import RetrievalEngine, make_retrieval_engine
from oracle import dls as odls

from conftest import GOLDEN

# reference signatures (names in order, default) — fusion.py:42-53, model.py:116-137
REF_BACKBONES = [("img_backbone", "swin"), ("swin_model_name", "swin_base_patch4_window7_224"),
                 ("cnn_model_name", "resnet50"), ("bert_model_name", "emilyalsentzer/Bio_ClinicalBERT"),
                 ("swin_checkpoint_path", None), ("bert_local_dir", None), ("pretrained", True),
                 ("img_dim", None), ("txt_dim", None)]
REF_MODEL = [("joint_dim", 256), ("num_heads", 4), ("num_classes", 22), ("num_fusion_layers", 3),
             ("fusion_type", "cross"), ("img_backbone", "swin"), ("swin_name", "swin_base_patch4_window7_224"),
             ("cnn_name", "resnet50"), ("bert_name", "emilyalsentzer/Bio_ClinicalBERT"), ("img_dim", None),
             ("txt_dim", None), ("swin_ckpt_path", None), ("bert_local_dir", None), ("pretrained", True),
             ("checkpoint_path", None), ("device", None), ("training", False), ("use_shared_ffn", True),
             ("use_cls_only", False), ("model_type", "multimodal"), ("retriever", None)]


def _positional(fn):
    ps = [p for p in inspect.signature(fn).parameters.values() if p.name != "self"]
    return [(p.name, p.default) for p in ps if p.kind == p.POSITIONAL_OR_KEYWORD]


def test_constructor_signatures_mirror_reference():
    assert _positional(Backbones.__init__) == REF_BACKBONES
    got = _positional(MultiModalRetrievalModel.__init__)
    assert [n for n, _ in got] == [n for n, _ in REF_MODEL]
    for (n, d), (_, rd) in zip(got, REF_MODEL):
        if n != "device":  # the reference defaults to cpu; this path is GPU-only
            assert d == rd, n
    assert inspect.signature(make_retrieval_engine).parameters["method"].default == "dls"


def _reference_layout_state():
    f = np.load(os.path.join(GOLDEN, "towers_mini.npz"), allow_pickle=False)
    cfg = json.loads(bytes(f["cfg"]).decode())
    sd = {}
    for k in f.files:
        if not k.startswith("w:"):
            continue
        v = torch.from_numpy(synthetic.bf16_bits_to_f32(f[k]).copy())
        name = k[2:]
        if name.startswith("swin."):
            sd["backbones.vision." + name[5:]] = v
        elif name.startswith("bert."):
            sd["backbones.bert." + name[5:]] = v
        else:
            sd[name[5:]] = v  # head.*
    return sd, cfg


def test_checkpoint_geometry_from_reference_layout(tmp_path):
    sd, cfg = _reference_layout_state()
    p = tmp_path / "model_best.pt"
    torch.save(sd, p)
    back = _load_tensors(p)  # torch.load(..., weights_only=True)
    assert set(back) == set(sd) and all(torch.equal(back[k], sd[k]) for k in sd)
    vis = {k[len("backbones.vision."):]: v for k, v in back.items() if k.startswith("backbones.vision.")}
    bert = {k[len("backbones.bert."):]: v for k, v in back.items() if k.startswith("backbones.bert.")}
    sc = swin_cfg_from_state(vis)
    assert sc["embed_dim"] == cfg["swin"]["embed_dim"] and sc["depths"] == cfg["swin"]["depths"]
    assert sc["num_heads"] == cfg["swin"]["num_heads"] and sc["window_size"] == 7
    bc = bert_cfg_from_state(bert)
    for k in ("hidden_size", "num_hidden_layers", "intermediate_size", "vocab_size"):
        assert bc[k] == cfg["bert"][k], k
    assert bc["num_attention_heads"] == cfg["bert"]["num_attention_heads"]
    # {"state_dict": ...} wrappers load the same way
    torch.save({"state_dict": sd}, tmp_path / "wrapped.pt")
    assert set(_load_tensors(tmp_path / "wrapped.pt")) == set(sd)


class _Probe(RetrievalEngine):
    def retrieve(self, query_emb, K=5, **kw):
        return [], []


def test_lazy_engine_keeps_memmap(tmp_path):
    G = synthetic.gauss_gallery(1000, 16, 3).astype(np.float64)
    np.save(tmp_path / "g.npy", G)
    mm = np.load(tmp_path / "g.npy", mmap_mode="r")
    e = _Probe(None, None, embs=mm, ids=[str(i) for i in range(1000)], lazy=True)
    assert isinstance(e.embs, np.memmap) and e.embs.dtype == np.float64  # no whole-gallery copy
    rows = e.get_embeddings_for_ids(["3", "nope", "999"])
    assert rows.dtype == np.float32 and np.array_equal(rows[0], G[3].astype(np.float32)) and not rows[1].any()
    e2 = _Probe(None, None, embs=mm, ids=[str(i) for i in range(1000)])
    assert e2.embs.dtype == np.float32 and not isinstance(e2.embs, np.memmap)  # the reference's astype copy


def test_host_merge_carries_payload():
    s = torch.tensor([[[0.9, 0.5, -np.inf]], [[0.9, 0.7, -np.inf]]], dtype=torch.float64)
    i = torch.tensor([[[7, 2, -1]], [[3, 9, -1]]])
    pay = torch.arange(2 * 1 * 3 * 3, dtype=torch.float64).view(2, 1, 3, 3)
    mi, _, m64, mp = merge_topk_host(s, i, 5, payload=pay)
    assert mi.tolist() == [[3, 7, 9, 2, -1]]
    # sources: 3 = list 1 slot 0, 7 = list 0 slot 0, 9 = list 1 slot 1, 2 = list 0 slot 1
    exp = [pay[1, 0, 0], pay[0, 0, 0], pay[1, 0, 1], pay[0, 0, 1]]
    for r, e in enumerate(exp):
        assert torch.equal(mp[0, r], e)
    assert not mp[0, 4].any()


def test_host_rerank_mix_matches_oracle():
    rng = np.random.default_rng(9)
    for trial in range(20):
        kc = int(rng.integers(1, 16))
        D, DK = 32, 8
        q = rng.standard_normal(D)
        C = rng.standard_normal((kc, D))
        if trial % 3 == 0:
            C[kc // 2] = C[0]  # equal finals: later candidate first
        ql = set(rng.choice(10, size=2, replace=False).tolist())
        cl = [set(rng.choice(10, size=int(rng.integers(0, 4)), replace=False).tolist()) for _ in range(kc)]
        if trial % 3 == 0:
            cl[kc // 2] = cl[0]
        qk, ck = rng.standard_normal(DK), rng.standard_normal((kc, DK))
        if trial % 3 == 0:
            ck[kc // 2] = ck[0]
        comp = np.stack([[odls._cos(q, C[j]), odls._jac(ql, cl[j]), odls._cos(qk, ck[j])] for j in range(kc)])
        cand = torch.arange(100, 100 + kc).view(1, kc)
        oi, fi, e, l, k = rerank_mix_host(cand, torch.from_numpy(comp).view(1, kc, 3), kc)
        order, final, re_, rl, rk = odls.rerank(q, C, ql, cl, qk, ck)
        assert (oi[0].numpy() - 100).tolist() == list(order)
        np.testing.assert_allclose(fi[0].numpy(), final, rtol=0, atol=1e-15)
        np.testing.assert_allclose(e[0].numpy(), re_, rtol=0, atol=1e-15)
    # empty slots are skipped and padded with -1
    cand = torch.tensor([[5, -1, 6]])
    comp = torch.tensor([[[0.5, 0.0, 0.1], [9.0, 9.0, 9.0], [0.7, 1.0, 0.2]]], dtype=torch.float64)
    oi, fi, *_ = rerank_mix_host(cand, comp, 3)
    assert oi.tolist() == [[6, 5, -1]] and fi[0, 0] == 1.0
