"""Golden-vector generator: runs the REFERENCE code (read-only, /root/reference) in this
container and commits only its inputs/outputs as small fixtures under tests/golden/.

Nothing here ships or travels: this script is the only file that imports the reference, and it
is run by hand (`python tests/golden/make_golden.py`) in the build container, never by the test
suite, bench.py or smoke(). The fixtures it writes are data (seeds, inputs, expected outputs).

What is pinned:
  knn_*.npz        sklearn `cosine_similarity` + `np.argsort(...)[::-1]`, the exact brute-force path
                   of src/Evaluate/retrieval_overlap.py:84-90 (and retrieval.py:128-137).
  ranking.json     `compute_ranking_metrics` itself (retrieval_overlap.py:84-115) on a labelled
                   synthetic gallery, plus `Helpers/retrieval_metrics.py` P@k/R@k/AP/mAP/MRR/nDCG.
  towers_mini.npz  `Backbones.forward` (fusion.py:255-327) + `MultiModalRetrievalModel.forward`
                   (model.py:330-489, model_type text / image / multimodal) with seeded mini towers.
                   timm (absent here) is replaced by a facade around transformers' SwinModel, which
                   implements the same Swin-v1 arithmetic; its weights are exported under timm's key
                   names so the oracle (timm semantics) loads them directly.

Third-party pins the reference names but this image lacks or differs on:
  timm 1.0.17 (requirements.txt:10): absent -> HF SwinModel stand-in (parity at the timm boundary is
  pinned only through this stand-in).  transformers 4.53.2 (requirements.txt:7): 5.15.0 here.
  scikit-learn 1.7.0 (requirements.txt:13): 1.7.2 here.
"""
import importlib
import importlib.util
import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference/src")
OUT = Path(__file__).resolve().parent
SEED = 2709  # configs/config.yaml:6

os.environ.setdefault("HF_HUB_OFFLINE", "1")
os.environ.setdefault("TRANSFORMERS_OFFLINE", "1")


# ----------------------------------------------------------------------------------------------
# stub loader (third-party modules absent from the image; reference packages whose __init__ pulls
# in unrelated heavy deps are registered as bare namespace packages over the real directories)
# ----------------------------------------------------------------------------------------------
def _pkg(name, path=None, **attrs):
    m = types.ModuleType(name)
    if path is not None:
        m.__path__ = [str(path)]
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def _load_file(modname, path):
    spec = importlib.util.spec_from_file_location(modname, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


SWIN_MINI = dict(embed_dim=32, depths=[2, 2, 2, 2], num_heads=[1, 2, 4, 8], window_size=7)
BERT_MINI = dict(vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=512, max_position_embeddings=512, type_vocab_size=2)


def install_stubs():
    import torch
    import transformers  # noqa: F401  (must be imported before a fake timm is registered)
    from transformers import SwinConfig, SwinModel

    sys.path.insert(0, str(REF))

    class TimmSwinFacade(torch.nn.Module):
        """timm-like facade: forward_features -> (B,H,W,C) NHWC after the final norm, `.norm`,
        `.num_features` (what fusion.py:177-199,236-252 reads)."""

        def __init__(self):
            super().__init__()
            cfg = SwinConfig(image_size=224, patch_size=4, num_channels=3,
                             embed_dim=SWIN_MINI["embed_dim"], depths=SWIN_MINI["depths"],
                             num_heads=SWIN_MINI["num_heads"], window_size=7, mlp_ratio=4.0,
                             hidden_act="gelu", layer_norm_eps=1e-5)
            self.hf = SwinModel(cfg, add_pooling_layer=False)
            self.norm = self.hf.layernorm
            self.num_features = self.hf.num_features

        def forward_features(self, x):
            out = self.hf(pixel_values=x).last_hidden_state       # (B, 49, C), final-normed
            B, L, C = out.shape
            g = int(round(L ** 0.5))
            return out.view(B, g, g, C)

    _pkg("timm", create_model=lambda *a, **k: TimmSwinFacade())

    class _Dummy:  # medclip / captum symbols referenced at import time only
        def __init__(self, *a, **k):
            pass

    _pkg("medclip", MedCLIPModel=_Dummy, MedCLIPVisionModelViT=_Dummy)
    _pkg("captum")
    _pkg("captum.attr", IntegratedGradients=_Dummy)
    sys.modules["captum"].attr = sys.modules["captum.attr"]

    # Helpers: real model_utils / config / retrieval_metrics, no heavy __init__
    H = _pkg("Helpers", REF / "Helpers")
    mu = importlib.import_module("Helpers.model_utils")
    cfg = importlib.import_module("Helpers.config")
    rm = importlib.import_module("Helpers.retrieval_metrics")
    H.load_hf_model_or_local = mu.load_hf_model_or_local
    H.download_swin = lambda *a, **k: None
    H.Config = cfg.Config
    for n in ("precision_at_k", "recall_at_k", "mean_average_precision", "mean_reciprocal_rank",
              "ndcg_at_k", "average_precision"):
        setattr(H, n, getattr(rm, n))

    _pkg("KnowledgeGraph", REF / "KnowledgeGraph")
    la = importlib.import_module("KnowledgeGraph.label_attention")
    sys.modules["KnowledgeGraph"].LabelAttention = la.LabelAttention
    sys.modules["KnowledgeGraph"].ensure_label_embeddings = lambda *a, **k: None
    kgl = _pkg("KnowledgeGraph.kg_label_create", ensure_label_embeddings=lambda *a, **k: None)
    del kgl
    _pkg("DataHandler", REF / "DataHandler", parse_openi_xml=None, build_dataloader=None)
    _pkg("DataHandler.TripletGenerate", LabelEmbeddingLookup=None)
    lab = _load_file("LabelData.labeledData", REF / "LabelData" / "labeledData.py")
    _pkg("LabelData", REF / "LabelData", **{k: getattr(lab, k) for k in dir(lab) if k.endswith("_groups")})
    return rm


# ----------------------------------------------------------------------------------------------
# synthetic data — the same generators live in oracle/data.py for the tests
# ----------------------------------------------------------------------------------------------
sys.path.insert(0, str(OUT.parent.parent))
from mmr_amd import synthetic as odata  # noqa: E402  (generators only; no compute path)


def gen_knn(rm):
    from sklearn.metrics.pairwise import cosine_similarity
    cases = [("knn_gauss_1k", 1000, 768, 64, (10, 50), "gauss"),
             ("knn_gauss_10k", 10000, 768, 64, (10, 50), "gauss"),
             ("knn_labelled_2k", 2000, 768, 64, (10,), "labelled")]
    for name, N, D, Q, Ks, kind in cases:
        if kind == "gauss":
            G = odata.gauss_gallery(N, D, SEED)
            Qm = odata.gauss_gallery(Q, D, SEED + 1)
            zero_rows = []
        else:
            G, gl = odata.labelled_gallery(N, D, SEED)
            Qm, ql = odata.labelled_gallery(Q, D, SEED + 1)
            zero_rows = [7, 11]  # sklearn maps zero-norm rows to similarity 0 (normalize())
            G[zero_rows] = 0.0
        sim = cosine_similarity(Qm, G)  # retrieval_overlap.py:85
        rec = dict(N=N, D=D, Q=Q, seed=SEED, kind=kind, g_sum=np.float64(G.astype(np.float64).sum()),
                   q_sum=np.float64(Qm.astype(np.float64).sum()), zero_rows=np.array(zero_rows, np.int64))
        for K in Ks:
            idx = np.stack([np.argsort(sim[i])[::-1][:K] for i in range(Q)])  # retrieval_overlap.py:90
            rec[f"idx_k{K}"] = idx.astype(np.int64)
            rec[f"score_k{K}"] = np.take_along_axis(sim, idx, 1).astype(np.float32)
        np.savez_compressed(OUT / f"{name}.npz", **rec)
        print("wrote", name)


def gen_ranking(rm):
    # compute_ranking_metrics (retrieval_overlap.py:84-115) — import the real module with stubs
    _pkg("Model", REF / "Model", MultiModalRetrievalModel=None)
    _pkg("Retrieval", REF / "Retrieval")
    sys.modules["Retrieval"].reranker = types.SimpleNamespace(Reranker=None)
    sys.modules["Retrieval.reranker"] = sys.modules["Retrieval"].reranker
    sys.modules["Helpers"].Config = importlib.import_module("Helpers.config").Config
    ro = _load_file("Evaluate_retrieval_overlap", REF / "Evaluate" / "retrieval_overlap.py")
    G, gl = odata.labelled_gallery(600, 768, SEED + 2)
    Qm, ql = odata.labelled_gallery(40, 768, SEED + 3)
    out = {"n_gallery": 600, "n_query": 40, "D": 768, "seed_g": SEED + 2, "seed_q": SEED + 3, "cases": {}}
    for k in (1, 5, 10):
        mrr, hit, rec = ro.compute_ranking_metrics(Qm, G, ql, gl, k=k)
        out["cases"][str(k)] = {"mrr": float(mrr), "hit_at_k": float(hit), "recall_at_k": float(rec)}
    # Helpers/retrieval_metrics.py on id lists (same ranking, string ids)
    rng = np.random.default_rng(SEED + 4)
    lists = []
    for _ in range(12):
        ret = [f"id{int(x)}" for x in rng.permutation(60)[:20]]
        rel = sorted({f"id{int(x)}" for x in rng.choice(60, size=int(rng.integers(0, 15)), replace=False)})
        lists.append((ret, rel))
    m = {"lists": lists, "per_list": []}
    for ret, rel in lists:
        rs = set(rel)
        row = {}
        for k in (1, 5, 10, 20):
            row[f"p@{k}"] = rm.precision_at_k(ret, rel, k)
            row[f"r@{k}"] = rm.recall_at_k(ret, rel, k)
            row[f"ndcg@{k}"] = rm.ndcg_at_k(ret, rel, k)
        row["ap"] = rm.average_precision(ret, rs)
        row["ap@10"] = rm.average_precision(ret, rs, 10)
        m["per_list"].append(row)
    m["map"] = rm.mean_average_precision([r for r, _ in lists], [set(x) for _, x in lists])
    m["map@10"] = rm.mean_average_precision([r for r, _ in lists], [set(x) for _, x in lists], 10)
    m["mrr"] = rm.mean_reciprocal_rank([r for r, _ in lists], [set(x) for _, x in lists])
    out["metrics"] = m
    (OUT / "ranking.json").write_text(json.dumps(out, indent=1))
    print("wrote ranking.json")


# HF Swin -> timm key names (timm 1.0.x: PatchMerging at the START of stages 1..3)
def hf_swin_to_timm(sd, depths):
    out = {}
    out["patch_embed.proj.weight"] = sd["hf.embeddings.patch_embeddings.projection.weight"]
    out["patch_embed.proj.bias"] = sd["hf.embeddings.patch_embeddings.projection.bias"]
    out["patch_embed.norm.weight"] = sd["hf.embeddings.norm.weight"]
    out["patch_embed.norm.bias"] = sd["hf.embeddings.norm.bias"]
    for i, d in enumerate(depths):
        for j in range(d):
            p = f"hf.encoder.layers.{i}.blocks.{j}."
            q = f"layers.{i}.blocks.{j}."
            out[q + "norm1.weight"] = sd[p + "layernorm_before.weight"]
            out[q + "norm1.bias"] = sd[p + "layernorm_before.bias"]
            out[q + "attn.qkv.weight"] = np.concatenate(
                [sd[p + f"attention.{n}_proj.weight"] for n in ("q", "k", "v")], 0)
            out[q + "attn.qkv.bias"] = np.concatenate(
                [sd[p + f"attention.{n}_proj.bias"] for n in ("q", "k", "v")], 0)
            out[q + "attn.relative_position_bias_table"] = sd[
                p + "attention.relative_position_bias.relative_position_bias_table"]
            out[q + "attn.proj.weight"] = sd[p + "attention.o_proj.weight"]
            out[q + "attn.proj.bias"] = sd[p + "attention.o_proj.bias"]
            out[q + "norm2.weight"] = sd[p + "layernorm_after.weight"]
            out[q + "norm2.bias"] = sd[p + "layernorm_after.bias"]
            for n in ("fc1", "fc2"):
                out[q + f"mlp.{n}.weight"] = sd[p + f"mlp.{n}.weight"]
                out[q + f"mlp.{n}.bias"] = sd[p + f"mlp.{n}.bias"]
        if i + 1 < len(depths):
            p = f"hf.encoder.layers.{i}.downsample."
            q = f"layers.{i + 1}.downsample."
            out[q + "norm.weight"] = sd[p + "norm.weight"]
            out[q + "norm.bias"] = sd[p + "norm.bias"]
            out[q + "reduction.weight"] = sd[p + "reduction.weight"]
    out["norm.weight"] = sd["hf.layernorm.weight"]
    out["norm.bias"] = sd["hf.layernorm.bias"]
    return out


def _bf16_round_(module):
    import torch
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(p.to(torch.bfloat16).to(torch.float32))


def gen_towers(rm):
    import torch
    from transformers import BertConfig, BertModel
    torch.manual_seed(SEED)
    tmp = Path(tempfile.mkdtemp(prefix="mmr_golden_"))
    bert_dir = tmp / "bert"
    BertModel(BertConfig(**BERT_MINI, hidden_act="gelu", layer_norm_eps=1e-12)).save_pretrained(str(bert_dir))

    _pkg("Retrieval", REF / "Retrieval")
    rr = types.ModuleType("Retrieval.reranker")
    rr.Reranker = None
    sys.modules["Retrieval.reranker"] = rr
    retr = _load_file("Retrieval.retrieval", REF / "Retrieval" / "retrieval.py")
    sys.modules["Retrieval"].RetrievalEngine = retr.RetrievalEngine
    sys.modules["Retrieval"].make_retrieval_engine = retr.make_retrieval_engine
    for n in list(sys.modules):
        if n == "Model" or n.startswith("Model."):
            del sys.modules[n]
    _pkg("Model", REF / "Model")
    _pkg("Model.explain", ExplanationEngine=None)
    fusion = importlib.import_module("Model.fusion")
    model_mod = importlib.import_module("Model.model")
    model_mod.EMBEDDINGS_DIR = tmp  # training=True writes dummy files (model.py:316-323)

    B, L = 2, 128
    rng = np.random.default_rng(SEED + 5)
    img_u8 = rng.integers(0, 256, size=(B, 224, 224), dtype=np.uint8)
    image = odata.image_from_u8(img_u8)
    ids, mask = odata.reports(B, L, SEED + 6, vocab=BERT_MINI["vocab_size"])

    rec = {"img_u8": img_u8, "input_ids": ids, "attention_mask": mask}
    models = {}
    for mt in ("text", "image", "multimodal"):
        torch.manual_seed(SEED + 7)
        m = model_mod.MultiModalRetrievalModel(
            joint_dim=64, num_heads=4, num_classes=43, num_fusion_layers=2, img_backbone="swin",
            swin_name="swin_mini", bert_name="bert_mini", bert_local_dir=str(bert_dir),
            pretrained=False, training=True, use_shared_ffn=False, use_cls_only=False, model_type=mt)
        # HF zero-inits the rel-pos bias table; randomise it so the bias path is exercised
        with torch.no_grad():
            for n, p in m.named_parameters():
                if "relative_position_bias_table" in n:
                    p.normal_(0, 0.5)
        _bf16_round_(m)
        m.eval()
        models[mt] = m
    # one weight set for all three heads: copy the text model's weights into the others
    sd0 = models["text"].state_dict()
    for mt in ("image", "multimodal"):
        models[mt].load_state_dict(sd0)

    with torch.no_grad():
        x = torch.from_numpy(image)
        ii = torch.from_numpy(ids)
        mm = torch.from_numpy(mask)
        (g, p), t = models["text"].backbones(x, ii, mm)
        rec["img_global"] = g.numpy()
        rec["img_patches"] = p.numpy()
        rec["txt_feats"] = t.numpy()
        for mt, m in models.items():
            o = m(x, ii, mm)
            rec[f"{mt}_joint_emb"] = o["joint_emb"].numpy()
            rec[f"{mt}_img_emb"] = o["img_emb"].numpy()
            rec[f"{mt}_txt_emb"] = o["txt_emb"].numpy()

    sd = {k: v.detach().float().numpy() for k, v in sd0.items()}
    vis = {k[len("backbones.vision."):]: v for k, v in sd.items() if k.startswith("backbones.vision.")}
    timm_sd = hf_swin_to_timm(vis, SWIN_MINI["depths"])
    weights = {}
    for k, v in timm_sd.items():
        weights["swin." + k] = v
    for k, v in sd.items():
        if k.startswith("backbones.bert."):
            weights["bert." + k[len("backbones.bert."):]] = v
        elif not k.startswith("backbones."):
            weights["head." + k] = v
    # store weights as bf16 bit patterns (they are bf16-exact by construction)
    for k, v in weights.items():
        assert np.array_equal(v, odata.bf16_bits_to_f32(odata.f32_to_bf16_bits(v))), k
        rec["w:" + k] = odata.f32_to_bf16_bits(v)
    rec["cfg"] = np.frombuffer(json.dumps({"swin": SWIN_MINI, "bert": BERT_MINI, "joint_dim": 64,
                                           "num_heads": 4, "num_fusion_layers": 2}).encode(), np.uint8)
    np.savez_compressed(OUT / "towers_mini.npz", **rec)
    print("wrote towers_mini.npz", sum(v.nbytes for v in rec.values()) / 1e6, "MB raw")


DLS_N, DLS_Q, DLS_ZERO, DLS_DUP, LABEL_NAMES = odata.DLS_N, odata.DLS_Q, odata.DLS_ZERO, odata.DLS_DUP, odata.LABEL_NAMES


def gen_dls_rerank(rm):
    """DLSRetrievalEngine._build_link_graph (retrieval.py:121-138) at two (threshold, max_links)
    settings, its greedy walk retrieve (retrieval.py:140-271, explicit seed), and Reranker.rerank
    (reranker.py:240-333) over exact top-15 candidates, with synthetic KG / labels files."""
    import pandas as pd
    tmp = Path(tempfile.mkdtemp(prefix="mmr_golden_dls_"))
    for n in list(sys.modules):
        if n == "Retrieval" or n.startswith("Retrieval."):
            del sys.modules[n]
    _pkg("Retrieval", REF / "Retrieval")
    rer = _load_file("Retrieval.reranker", REF / "Retrieval" / "reranker.py")
    sys.modules["Retrieval"].reranker = rer
    retr = _load_file("Retrieval.retrieval", REF / "Retrieval" / "retrieval.py")

    G, gl = odata.dls_gallery()
    ids = [f"r{i}" for i in range(DLS_N)]
    np.save(tmp / "g.npy", G)
    (tmp / "ids.json").write_text(json.dumps(ids))
    rec = {"N": DLS_N, "D": odata.DLS_D, "seed": SEED + 11, "g_sum": np.float64(G.astype(np.float64).sum())}
    for tag, thr, ml in (("t50_m10", 0.5, 10), ("t30_m8", 0.3, 8)):
        eng = retr.make_retrieval_engine(str(tmp / "g.npy"), str(tmp / "ids.json"), method="dls",
                                         link_threshold=thr, max_links=ml, fdb_path=str(tmp / f"{tag}.pkl"))
        graph = eng.link_graph
        rec[f"graph_{tag}_offsets"] = np.cumsum([0] + [len(x) for x in graph]).astype(np.int64)
        rec[f"graph_{tag}_flat"] = np.array([j for x in graph for j in x], np.int64)
        if tag == "t50_m10":
            Qm, _ = odata.labelled_gallery(DLS_Q, odata.DLS_D, SEED + 12)
            out_i, out_s = [], []
            for qi in range(DLS_Q):
                r_ids, r_sc = eng.retrieve(Qm[qi], K=5, seed=SEED + qi)
                out_i.append([int(x[1:]) for x in r_ids] + [-1] * (5 - len(r_ids)))
                out_s.append(list(r_sc) + [np.nan] * (5 - len(r_sc)))
            rec["walk_idx"] = np.array(out_i, np.int64)
            rec["walk_score"] = np.array(out_s, np.float64)

    # reranker: synthetic KG dir + labels CSV
    rng = np.random.default_rng(SEED + 13)
    node2id = odata.kg_node2id(DLS_N)
    nemb = rng.standard_normal((len(node2id), 300)).astype(np.float32)
    kg = tmp / "kg"
    kg.mkdir()
    (kg / "node2id.json").write_text(json.dumps(node2id))
    np.save(kg / "node_embeddings_best.npy", nemb)
    df = pd.DataFrame(gl.astype(np.int64), columns=LABEL_NAMES)
    df.insert(0, "id", ids)
    df["report"] = ["text"] * DLS_N                       # non-numeric column (skipped)
    df.to_csv(tmp / "labels.csv", index=False)
    R = rer.Reranker(kg_dir=kg, labels_csv=tmp / "labels.csv")
    from sklearn.metrics.pairwise import cosine_similarity
    qrows = list(range(0, 4 * DLS_Q, 4)) + [DLS_ZERO[0], DLS_DUP[0]]
    sim = cosine_similarity(G[qrows], G)
    cand = np.stack([np.argsort(sim[i])[::-1][:15] for i in range(len(qrows))])
    r_order, r_final, r_e, r_l, r_k = [], [], [], [], []
    for qn, qi in enumerate(qrows):
        cids = [ids[j] for j in cand[qn]]
        lookup = {c: G[j] for c, j in zip(cids, cand[qn])}
        lookup[ids[qi]] = G[qi]
        out = R.rerank(ids[qi], cids, candidate_embs=G[cand[qn]], candidate_emb_lookup=lookup, topk=10)
        r_order.append([int(t[0][1:]) for t in out])
        r_final.append([t[1] for t in out])
        r_e.append([t[2] for t in out])
        r_l.append([t[3] for t in out])
        r_k.append([t[4] for t in out])
    rec.update(rr_queries=np.array(qrows, np.int64), rr_cand=cand.astype(np.int64),
               rr_order=np.array(r_order, np.int64), rr_final=np.array(r_final), rr_emb=np.array(r_e),
               rr_lab=np.array(r_l), rr_kg=np.array(r_k), kg_node_emb=nemb,
               kg_node2id=np.frombuffer(json.dumps(node2id).encode(), np.uint8))
    np.savez_compressed(OUT / "dls_rerank.npz", **rec)
    print("wrote dls_rerank.npz")


if __name__ == "__main__":
    rm = install_stubs()
    which = sys.argv[1:] or ["knn", "ranking", "towers", "dls"]
    if "dls" in which:
        gen_dls_rerank(rm)
    if "knn" in which:
        gen_knn(rm)
    if "ranking" in which:
        gen_ranking(rm)
    if "towers" in which:
        gen_towers(rm)
