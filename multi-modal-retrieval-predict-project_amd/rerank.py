"""KG / label Reranker — mirrors src/Retrieval/reranker.py (Reranker) on the fused device kernel
mmr_index_rerank (include/mmr.h).

Tables (built once, like the reference's _try_precompute_record_kg, reranker.py:222-238):
  label sets   labels CSV (index_col "id"); a record's set = the columns whose value int()s to 1
               (get_record_label_set, :161-179) -> one uint64 bitset per record (<= 64 label columns)
  KG vectors   node embeddings L2-normalised in f32 (_load_kg, :88-129); per record the
               "report:<id>" / "<id>" node, else the mean (or LabelAttention-pooled) vectors of its
               label nodes (label:<l>, <l>, <l>.lower(), <l> with "_"), else zeros
               (get_record_kg_vec, :181-220)
Scoring (rerank, :240-333) runs on the GPU: cosines in f64, Jaccard on the bitsets, per-list
min-max, alpha/beta/gamma mix, rank by final desc (equal finals: later candidate first).
"""
import json
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib


class Reranker:
    def __init__(self, kg_dir, labels_csv, alpha: float = 0.6, beta: float = 0.25, gamma: float = 0.15,
                 label_attention_state: Optional[Dict[str, torch.Tensor]] = None, device=None):
        import pandas as pd
        self.kg_dir, self.labels_csv = Path(kg_dir), Path(labels_csv)
        self.alpha, self.beta, self.gamma = alpha, beta, gamma
        self.kg = self._load_kg(self.kg_dir)
        self.labels_df = pd.read_csv(self.labels_csv, index_col="id")
        self.labels_df.index = self.labels_df.index.astype(str)
        self.columns = [str(c) for c in self.labels_df.columns]
        self._row = {rid: i for i, rid in enumerate(self.labels_df.index)}
        self._bits = self._label_bits()
        self.attn = None
        if label_attention_state is not None:  # KnowledgeGraph/label_attention.py:13-17 weights
            sd = label_attention_state
            self.attn = tuple(np.asarray(sd[k], np.float64) for k in
                              ("attn.0.weight", "attn.0.bias", "attn.2.weight", "attn.2.bias"))
        self.device = torch.cuda.current_device() if device is None else int(device)
        self._bound = None

    # ---------------------------------------------------------------- tables
    @staticmethod
    def _load_kg(kg_dir: Path):
        node2id_path = kg_dir / "node2id.json"
        if not node2id_path.exists():
            raise FileNotFoundError(f"KG node2id.json not found at {node2id_path}")
        node2id = json.load(open(node2id_path, "r", encoding="utf8"))
        best = sorted(kg_dir.glob("node_embeddings_best.npy"))
        files = best or sorted(kg_dir.glob("node_embeddings_epoch*.npy")) or sorted(kg_dir.glob("node_embeddings*.npy"))
        if not files:
            raise FileNotFoundError("No .npy embeddings found in KG dir")
        node_emb = np.load(files[-1], allow_pickle=False)
        node_emb = node_emb / (np.linalg.norm(node_emb, axis=1, keepdims=True) + 1e-12)
        return {"node2id": node2id, "node_emb": node_emb}

    def _label_bits(self):
        """(n_records,) uint64: bit j set iff int(value of the j-th label-carrying column) == 1
        (non-numeric -> skipped); only columns that ever hold a 1 get a bit (<= 64)."""
        bits = np.zeros(len(self.labels_df), np.uint64)
        self._bitcols = []
        for c in self.columns:
            col = self.labels_df[c]
            hit = np.zeros(len(col), bool)
            for i, v in enumerate(col.tolist()):
                try:
                    hit[i] = int(v) == 1
                except (ValueError, TypeError):
                    pass
            if hit.any():
                if len(self._bitcols) == 64:
                    raise ValueError("more than 64 label columns carry labels (uint64 label sets)")
                bits |= hit.astype(np.uint64) << np.uint64(len(self._bitcols))
                self._bitcols.append(c)
        return bits

    def record_bits(self, rec_id) -> int:
        i = self._row.get(str(rec_id))
        return 0 if i is None else int(self._bits[i])

    def get_record_label_set(self, rec_id):
        b = self.record_bits(rec_id)
        return {c for j, c in enumerate(self._bitcols) if (b >> j) & 1}

    def get_record_kg_vec(self, rec_id) -> np.ndarray:
        node2id, ne = self.kg["node2id"], self.kg["node_emb"]
        for key in (f"report:{rec_id}", str(rec_id)):
            if key in node2id:
                return ne[node2id[key]]
        vecs = []
        for lab in sorted(self.get_record_label_set(rec_id)):
            for ck in (f"label:{lab}", lab, lab.lower(), lab.replace(" ", "_")):
                if ck in node2id:
                    vecs.append(ne[node2id[ck]])
                    break
        if not vecs:
            return np.zeros(ne.shape[1], dtype=np.float32)
        L = np.stack(vecs)
        if self.attn is None:
            return L.mean(axis=0)
        w1, b1, w2, b2 = self.attn
        s = np.tanh(L.astype(np.float64) @ w1.T + b1) @ w2.T + b2
        s = np.exp(s[:, 0] - s[:, 0].max())
        return ((s / s.sum()) @ L.astype(np.float64)).astype(np.float32)

    def tables(self, ids: List[str]):
        """Device tables for a record list: (bits (n,) uint64-as-int64, kg (n, dk) f32)."""
        dev = torch.device(f"cuda:{self.device}")
        bits = np.array([self.record_bits(r) for r in ids], np.uint64).view(np.int64)
        kg = np.stack([np.asarray(self.get_record_kg_vec(r), np.float32) for r in ids]) if ids else \
            np.zeros((0, self.kg["node_emb"].shape[1]), np.float32)
        return torch.from_numpy(bits).to(dev), torch.from_numpy(np.ascontiguousarray(kg)).to(dev)

    def bind(self, engine):
        """Precompute the gallery tables of an MI355X engine (one row per engine id)."""
        self._bound = (engine, *self.tables([str(i) for i in engine.ids]))
        return self

    # ---------------------------------------------------------------- scoring
    def rerank_batch(self, engine, q_emb, query_ids, cand, topk):
        """Device path (config 5 "KG-rerank head fused"): q_emb (nq, D) f32 device, cand (nq, kc)
        int64 device top-K indices of `engine` -> (idx, final, emb_n, lab_n, kg_n) device tensors."""
        if self._bound is None or self._bound[0] is not engine:
            self.bind(engine)
        _, gbits, gkg = self._bound
        qbits, qkg = self.tables([str(q) for q in query_ids])
        return engine.index.rerank(q_emb, cand, qbits, gbits, qkg, gkg, topk, self.alpha, self.beta, self.gamma)

    def rerank(self, query_id, candidate_ids, candidate_embs=None, candidate_emb_lookup=None, topk=None,
               query_emb=None):
        """reranker.py:240-333 signature -> [(id, final, emb_n, lab_n, kg_n)] on the device kernel."""
        from .retrieval import GalleryIndex
        _lib.require_gpu()
        N = len(candidate_ids)
        if candidate_embs is None:
            if candidate_emb_lookup is None:
                raise ValueError("Please provide candidate_embs or candidate_emb_lookup.")
            zero = np.zeros(next(iter(candidate_emb_lookup.values())).shape, dtype=float)
            candidate_embs = np.vstack([candidate_emb_lookup.get(str(c), zero) for c in candidate_ids])
        candidate_embs = np.asarray(candidate_embs, np.float32)
        if candidate_embs.shape[0] != N:
            raise ValueError("candidate_embs rows must match candidate_ids length")
        q = None
        if candidate_emb_lookup is not None and str(query_id) in candidate_emb_lookup:
            q = candidate_emb_lookup[str(query_id)]
        elif query_emb is not None:
            q = query_emb
        else:
            for i, c in enumerate(candidate_ids):
                if str(c) == str(query_id):
                    q = candidate_embs[i]
                    break
        if q is None:
            raise ValueError("Query embedding not found. Provide candidate_emb_lookup keyed by query_id, or include "
                             "the query_id in candidate_ids with matching candidate_embs, or pass query_emb.")
        if N == 0:
            return []
        if N > 64:
            raise ValueError("at most 64 candidates per query on the fused rerank kernel")
        dev = torch.device(f"cuda:{self.device}")
        ix = GalleryIndex(candidate_embs, device=self.device)
        try:
            gbits, gkg = self.tables([str(c) for c in candidate_ids])
            qbits, qkg = self.tables([str(query_id)])
            qe = torch.from_numpy(np.asarray(q, np.float32).reshape(1, -1)).to(dev)
            cand = torch.arange(N, dtype=torch.int64, device=dev).view(1, N)
            k = int(topk) if topk else N
            k = min(k, N)
            oi, fi, e, l, g = ix.rerank(qe, cand, qbits, gbits, qkg, gkg, k, self.alpha, self.beta, self.gamma)
            oi, fi, e, l, g = (t[0].cpu().numpy() for t in (oi, fi, e, l, g))
        finally:
            ix.close()
        return [(candidate_ids[int(i)], float(fi[r]), float(e[r]), float(l[r]), float(g[r]))
                for r, i in enumerate(oi) if i >= 0]
