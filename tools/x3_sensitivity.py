"""Per-contraction-class sensitivity of the parity-grade (x3) line: the bench model in the
x3 mode at B = 256, with chosen classes of linears degraded from the bf16x3 split (x.w ~ xh.wh + xh.wl + xl.wh)
to one bf16 product (xh.wh: the w image's wl and second-wh segments zeroed) or to bf16 weights only
(x.wh: the wl segment zeroed), each variant's top-10 over the 100k x 768 labelled gallery compared with the
fp32 oracle path exactly as tests/test_x3_gpu.py::test_e2e_x3_batch_256_identical_topk does (tie-aware
equivalence, exact list match, identical P@10).  Diagnostic only: the product path never degrades."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.model import build_bench_model, init_fusion_state, init_head_state  # noqa: E402
from mmr_amd.retrieval import MI355XRetrievalEngine  # noqa: E402
from mmr_amd.towers import BERT_BASE, SWIN_T, init_bert_state, init_swin_state  # noqa: E402
from oracle import knn as oknn  # noqa: E402
from oracle import towers as otw  # noqa: E402

DEV = "cuda"
B = 256
img = torch.from_numpy(synthetic.image_from_u8(synthetic.image_u8(B, 71)))
ids, mask = (torch.from_numpy(a) for a in synthetic.reports(B, 128, 72))
ssd, bsd = init_swin_state(SWIN_T, 2709), init_bert_state(BERT_BASE, 2710)
hsd = init_head_state(768, 768, 768, 2711)
hsd.update(init_fusion_state(768, 768, 768, 8, 5, 2712))
with torch.no_grad():
    (g, p), t = otw.backbones_forward(img, ids, mask, ssd, bsd, SWIN_T, BERT_BASE)
    q_cpu = otw.heads(g, p, t, hsd, "multimodal", mm_cfg={"num_heads": 8})["joint_emb"].numpy()
G, gl = synthetic.labelled_gallery(100_000, 768, 73)
gbits = synthetic.labels_to_bits(gl)
ci, cs = oknn.sklearn_topk(q_cpu, G, 10)
eng = MI355XRetrievalEngine(embs=G, ids=[str(i) for i in range(len(G))], dtype="fp32")
rng = np.random.default_rng(74)
qlab = np.zeros((B, synthetic.NUM_LABELS), np.uint8)
for i in range(B):
    qlab[i, rng.choice(synthetic.NUM_LABELS, size=int(rng.integers(1, 4)), replace=False)] = 1
qbits = synthetic.labels_to_bits(qlab)


def p10(idx):
    return float(np.mean([np.count_nonzero(gbits[idx[i]] & qbits[i]) / 10 for i in range(B)]))


class Wrap:
    """An X3W stand-in whose split-GEMM weight image [w_hi | w_lo] has its lo segment zeroed (the weight
    rounded to bf16; x keeps its split — the round-5 record in profiles/r05_x3_sensitivity.txt was taken on
    the earlier [w_hi | w_lo | w_hi] image, where one bf16 product could be isolated)."""
    def __init__(self, wx, how):
        self.__dict__.update(w=wx.w, hi=wx.hi, lo=wx.lo, _inner=wx, _how=how, _img=None)

    def w2(self, kp, npad):
        if self._img is None:
            img = self._inner.w2(kp, npad).clone()
            img[:, kp:] = 0
            self._img = img
        return self._img

    def bias_padded(self, bias, npad):
        return self._inner.bias_padded(bias, npad)


def run(name, patch):
    m = build_bench_model(device=DEV, joint_dim=768, model_type="multimodal", tower_dtype="x3")
    patch(m)
    q = m.query_embeddings(img.to(DEV), ids.to(DEV), mask.to(DEV)).float().cpu().numpy()
    gi, gs = eng.search(np.ascontiguousarray(q), K=10)
    gi = gi.cpu().numpy() if isinstance(gi, torch.Tensor) else np.asarray(gi)
    gs = gs.cpu().numpy() if isinstance(gs, torch.Tensor) else np.asarray(gs)
    ok, msg = oknn.topk_equivalent(ci, cs, gi, gs, tie_tol=1e-6, score_tol=1e-4)
    print(json.dumps({"variant": name, "topk_equivalent": bool(ok), "msg": msg[:80],
                      "exact_list_match": float(np.mean([np.array_equal(gi[i], ci[i]) for i in range(B)])),
                      "max_score_err": float(np.abs(gs - cs).max()),
                      "max_rel_emb_err": float(np.abs(q - q_cpu).max() / np.abs(q_cpu).max()),
                      "p10_gpu": p10(gi), "p10_cpu": p10(ci)}), flush=True)


def bert(m, keys, how, layers=None):
    for i, ly in enumerate(m.backbones.bert.layers):
        if layers is None or i in layers:
            for k in keys:
                ly[k] = Wrap(ly[k], how)


def swin(m, stages, how):
    sw = m.backbones.vision
    sw.fused_mlp = sw.fused_linears = False
    for s in stages:
        st = sw.stages[s]
        for bk in st["blocks"]:
            for k in ("qkv_w", "proj_w", "fc1_w", "fc2_w"):
                bk[k] = Wrap(bk[k], how)
        if "ds_w" in st:
            st["ds_w"] = Wrap(st["ds_w"], how)


def fusion(m, how):
    f = m.fusion
    for L in f.layers:
        for k in ("t_x3", "ppp_x3", "o2_x3t"):
            L[k] = Wrap(L[k], how)
        for e in ("txt", "patch"):
            L[e].w_in_x3 = Wrap(L[e].w_in_x3, how)
            L[e].w_o_x3 = Wrap(L[e].w_o_x3, how)
    f.s_x3 = Wrap(f.s_x3, how)


run("x3 (baseline)", lambda m: None)
run("BERT FFN bf16 weights", lambda m: bert(m, ("i_w", "f_w"), "bf16w"))
run("BERT FFN bf16", lambda m: bert(m, ("i_w", "f_w"), "bf16"))
run("BERT QKV+O bf16", lambda m: bert(m, ("qkv_w", "o_w"), "bf16"))
run("BERT layers 0-3 FFN bf16", lambda m: bert(m, ("i_w", "f_w"), "bf16", layers=range(4)))
run("BERT layer 11 FFN bf16", lambda m: bert(m, ("i_w", "f_w"), "bf16", layers=[11]))
run("Swin stages 3-4 bf16", lambda m: swin(m, (2, 3), "bf16"))
run("Swin stages 1-2 bf16", lambda m: swin(m, (0, 1), "bf16"))
run("fusion token linears bf16", lambda m: fusion(m, "bf16"))
