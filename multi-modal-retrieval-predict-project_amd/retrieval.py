"""Query interface — mirrors src/Retrieval/retrieval.py (RetrievalEngine ABC + make_retrieval_engine).

RetrievalEngine            retrieval.py:18-50   (.npy f32 gallery + ids.json, id2idx, retrieve(), get_embeddings_for_ids())
MI355XRetrievalEngine      exact brute-force cosine top-K on the GPU (libmmr, include/mmr.h) with
                           the reference's exact-path semantics (retrieval_overlap.py:84-90):
                           cosine of the raw rows, descending; ties -> lower gallery index.
DLSRetrievalEngine         retrieval.py:53-271: link graph = exact GPU self-join (SURVEY.md §8f row
                           2); the approximate random-seeded greedy walk (3.75 % recall@10 vs exact in
                           the survey probe, §8a-a11) stays the reference's host algorithm.
make_retrieval_engine      retrieval.py:273-304  (string switch; unknown method -> ValueError)
"""
import abc
import ctypes
import json
import threading
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib


class RetrievalEngine(abc.ABC):
    """Loads embeddings once; id -> index map; abstract retrieve (retrieval.py:18-50)."""

    def __init__(self, features_path: Optional[str], ids_path: Optional[str], embs=None, ids=None,
                 lazy: bool = False):
        """lazy: keep `embs` as given (e.g. an np.load(..., mmap_mode="r") memmap of any float dtype)
        instead of materialising a float32 copy — the sharded engine converts only its rows."""
        if embs is None:
            embs = np.load(features_path)
        self._raw = embs if isinstance(embs, np.ndarray) else None  # the file's own dtype (fp16 galleries)
        if lazy:
            self.embs = embs if isinstance(embs, np.ndarray) else np.asarray(embs)
        else:
            self.embs = np.ascontiguousarray(np.asarray(embs).astype("float32"))  # (N, D)
        if ids is None:
            with open(ids_path, "r") as f:
                ids = json.load(f)
        self.ids = list(ids)
        self.id2idx = {str(self.ids[i]): i for i in range(len(self.ids))}
        assert self.embs.shape[0] == len(self.ids), "embeddings count != ids count"

    @abc.abstractmethod
    def retrieve(self, query_emb: np.ndarray, K: int = 5, **kwargs) -> Tuple[List[str], List[float]]:
        """Given a query embedding (D,) or (1,D), return top-K IDs and their scores."""

    def get_embeddings_for_ids(self, ids: List[str]) -> np.ndarray:
        """Embeddings in the order of ids (zeros if missing) — retrieval.py:41-50."""
        rows = []
        for _id in ids:
            idx = self.id2idx.get(str(_id), None)
            rows.append(np.zeros(self.embs.shape[1], dtype=np.float32) if idx is None
                        else np.asarray(self.embs[idx], dtype=np.float32))
        return np.vstack(rows)


class GalleryIndex:
    """Owning wrapper of an mmr_index (one device-resident gallery shard).

    Scan modes (all exact: candidates re-scored in f64 from the gallery's own rows): "x3" bf16 3-term
    split GEMM (default; Q <= 32 use the skinny f32 stream), "f32" f32 MFMA, "f16" fp16 unit-row copy
    of the gallery (half the scan bytes, wider candidate margin).  An fp16 gallery (numpy float16 /
    torch.float16 rows: BASELINE config 5) builds a NATIVE fp16 index (MMR_F16): its raw fp16 rows are
    the only device copy (2 B per element + norms), scanned in mode "f16" and re-scored exactly (fp16 is
    exact in f64) — the same results as an index of the f32-upcast rows (the reference's
    .astype("float32"), retrieval.py:24-32).  Heavily tied galleries (more candidates within the
    margin than the selection buffer holds) are handled inside the selection kernel by batched exact
    merging, so the per-query status is always 0 (checked by callers that ask for it)."""

    MODES = {"f32": 0, "x3": 1, "f16": 2}

    def __init__(self, embs, device=None, idx_base: int = 0, mode=None):
        """mode None: "f16" for fp16 rows (a native fp16 index is f16-only), else "x3".  An fp16 gallery
        with an explicit other mode raises ValueError (upcast the rows to f32 for an x3 / f32 index)."""
        _lib.require_gpu()
        L = _lib.lib()
        if device is None:
            device = torch.cuda.current_device()
        self.device = int(device)
        if isinstance(embs, torch.Tensor):
            half = embs.dtype == torch.float16
            src = embs.detach().to(torch.float16 if half else torch.float32).contiguous()
            is_host = 0 if src.is_cuda else 1
            if src.is_cuda and src.device.index != self.device:
                src = src.to(f"cuda:{self.device}")
            n, d = src.shape
            p = ctypes.c_void_p(src.data_ptr())
            keep = src
        else:
            half = np.asarray(embs).dtype == np.float16
            keep = np.ascontiguousarray(np.asarray(embs, dtype=np.float16 if half else np.float32))
            n, d = keep.shape
            is_host = 1
            p = keep.ctypes.data_as(ctypes.c_void_p)
        if not is_host:
            torch.cuda.synchronize(self.device)  # the copy runs on the default stream
        h = ctypes.c_void_p()
        self.native_f16 = bool(half)
        if mode is None:
            mode = "f16" if half else "x3"
        if mode not in self.MODES:
            raise ValueError(f"scan mode {mode!r} (x3 | f32 | f16)")
        if half and mode != "f16":
            raise ValueError(f"an fp16 gallery builds a native fp16 index, which scans only in mode 'f16' (asked "
                             f"{mode!r}): pass f32 rows for an {mode} index")
        _lib.check(L.mmr_index_create(p, n, d, 1 if half else 0, is_host, idx_base, self.device, ctypes.byref(h)),
                   "mmr_index_create")
        del keep
        self._h = h
        _lib.check(L.mmr_index_set_mode(h, self.MODES[mode]), "mmr_index_set_mode")
        self.mode = mode
        self.n, self.d, self.idx_base = int(n), int(d), int(idx_base)
        # held across a set_mode / search / set_mode sequence (per-call mode override) and by every
        # search, so no search of another host thread runs in a temporarily switched mode
        self._lock = threading.RLock()

    def set_mode(self, mode: str):
        if mode not in self.MODES:
            raise ValueError(f"scan mode {mode!r} (x3 | f32 | f16)")
        if self.native_f16 and mode != "f16":
            raise ValueError(f"a native fp16 index scans only in mode 'f16' (asked {mode!r})")
        with self._lock:
            _lib.check(_lib.lib().mmr_index_set_mode(self._h, self.MODES[mode]), "mmr_index_set_mode")
            self.mode = mode

    def device_bytes(self):
        """(gallery bytes, workspace bytes) this index holds on its GPU (mmr_index_device_bytes)."""
        g, w = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib().mmr_index_device_bytes(self._h, ctypes.byref(g), ctypes.byref(w)),
                   "mmr_index_device_bytes")
        return int(g.value), int(w.value)

    def reserve(self, max_q: int):
        _lib.check(_lib.lib().mmr_index_reserve(self._h, int(max_q)), "mmr_index_reserve")

    def search(self, q: torch.Tensor, k: int, want_f64: bool = False, want_status: bool = False, mode=None):
        """q (B, D) f32 device tensor -> (idx int64 (B,k), score f32 (B,k)[, score64][, status]).
        mode: run this one search in another scan mode (the index's mode is restored after)."""
        if mode is not None and mode != self.mode:
            with self._lock:
                prev = self.mode
                self.set_mode(mode)
                try:
                    return self.search(q, k, want_f64, want_status)
                finally:
                    self.set_mode(prev)
        with self._lock:
            return self._search(q, k, want_f64, want_status)

    def _search(self, q, k, want_f64, want_status):
        _lib.require_gpu(q)
        if q.dim() != 2 or q.shape[1] != self.d:
            raise ValueError(f"query shape {tuple(q.shape)} does not match gallery dim {self.d}")
        if not 1 <= k <= _lib.lib().mmr_max_k():
            raise ValueError(f"K={k} outside [1, {_lib.lib().mmr_max_k()}]")
        q = q.to(torch.float32).contiguous()
        B = q.shape[0]
        dev = q.device
        idx = torch.empty((B, k), dtype=torch.int64, device=dev)
        sc = torch.empty((B, k), dtype=torch.float32, device=dev)
        sc64 = torch.empty((B, k), dtype=torch.float64, device=dev) if want_f64 else None
        st = torch.empty((B,), dtype=torch.int32, device=dev) if want_status else None
        _lib.check(_lib.lib().mmr_index_search(self._h, _lib.ptr(q), B, k, _lib.ptr(idx), _lib.ptr(sc),
                                               _lib.ptr(sc64), _lib.ptr(st), _lib.stream_ptr(dev)),
                   "mmr_index_search")
        out = [idx, sc]
        if want_f64:
            out.append(sc64)
        if want_status:
            out.append(st)
        return tuple(out)

    def link_graph(self, threshold: float, max_links: int, batch: int = 8192, stream_dev=None):
        """DLS link graph of this shard (retrieval.py:121-138) on the device: (nbr (n, max_links)
        int64 local indices, -1 padded; cnt (n,) int32) as device tensors."""
        dev = torch.device(f"cuda:{self.device}")
        nbr = torch.empty((self.n, max_links), dtype=torch.int64, device=dev)
        cnt = torch.empty((self.n,), dtype=torch.int32, device=dev)
        for r0 in range(0, self.n, batch):
            nr = min(batch, self.n - r0)
            _lib.check(_lib.lib().mmr_index_link_graph(self._h, float(threshold), int(max_links), r0, nr,
                                                       _lib.ptr(nbr[r0:]), _lib.ptr(cnt[r0:]), _lib.stream_ptr(dev)),
                       "mmr_index_link_graph")
        return nbr, cnt

    def rerank(self, q_emb, cand, q_labels, g_labels, q_kg, g_kg, topk, alpha=0.6, beta=0.25, gamma=0.15,
               want_components=True):
        """Fused KG / label rerank of device top-K candidates (mmr_index_rerank).  Returns
        (idx (nq, topk) int64, final, emb_n, lab_n, kg_n (nq, topk) f64 or None)."""
        q_emb = q_emb.to(torch.float32).contiguous()
        nq, kc = cand.shape
        dev = cand.device
        out_i = torch.empty((nq, topk), dtype=torch.int64, device=dev)
        outs = [torch.empty((nq, topk), dtype=torch.float64, device=dev) if want_components else None
                for _ in range(4)]
        _lib.check(_lib.lib().mmr_index_rerank(
            self._h, _lib.ptr(q_emb), nq, _lib.ptr(cand.contiguous()), kc, _lib.ptr(q_labels), _lib.ptr(g_labels),
            _lib.ptr(q_kg), _lib.ptr(g_kg), q_kg.shape[1], float(alpha), float(beta), float(gamma), int(topk),
            _lib.ptr(out_i), *(_lib.ptr(o) for o in outs), _lib.stream_ptr(dev)), "mmr_index_rerank")
        return (out_i, *outs)

    def rerank_components(self, q_emb, cand, q_labels, g_labels, q_kg, g_kg):
        """Shard side of the sharded rerank (mmr_index_rerank_components): the raw {emb cosine, label
        Jaccard, KG cosine} of this shard's candidates cand (nq, kc) -> (nq, kc, 3) f64 device."""
        q_emb = q_emb.to(torch.float32).contiguous()
        nq, kc = cand.shape
        comp = torch.empty((nq, kc, 3), dtype=torch.float64, device=cand.device)
        _lib.check(_lib.lib().mmr_index_rerank_components(
            self._h, _lib.ptr(q_emb), nq, _lib.ptr(cand.contiguous()), kc, _lib.ptr(q_labels), _lib.ptr(g_labels),
            _lib.ptr(q_kg), _lib.ptr(g_kg), q_kg.shape[1], _lib.ptr(comp), _lib.stream_ptr(cand.device)),
            "mmr_index_rerank_components")
        return comp

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            _lib.lib().mmr_index_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def check_status(st: torch.Tensor):
    """Raise if mmr_index_search flagged a query (status != 0).  The selection kernel resolves
    candidate-buffer overflow itself (batched exact merge), so this is a guard, not a code path."""
    if st.numel() and int(st.max().item()) != 0:
        raise RuntimeError(f"mmr_index_search returned status {int(st.max().item())} for "
                           f"{int((st != 0).sum().item())} queries")


def merge_topk(scores64: torch.Tensor, idx: torch.Tensor, k_out: int, payload=None, q0: int = 0, nq=None):
    """[L][B][k_in] f64 scores + int64 idx (-1 = empty) -> global top-k_out (idx, f32, f64) on device
    for queries [q0, q0 + nq) (default: all B).  payload [L][B][k_in][P] f64 (optional) rides with
    each entry: then a 4th output (nq, k_out, P) is returned."""
    _lib.require_gpu(scores64)
    L_, B, k_in = idx.shape
    nq = B - q0 if nq is None else nq
    dev = idx.device
    oi = torch.empty((nq, k_out), dtype=torch.int64, device=dev)
    os_ = torch.empty((nq, k_out), dtype=torch.float32, device=dev)
    o64 = torch.empty((nq, k_out), dtype=torch.float64, device=dev)
    P = 0 if payload is None else payload.shape[-1]
    op = None if payload is None else torch.empty((nq, k_out, P), dtype=torch.float64, device=dev)
    _lib.check(_lib.lib().mmr_merge_topk_payload(
        _lib.ptr(scores64.contiguous()), _lib.ptr(idx.contiguous()),
        _lib.ptr(None if payload is None else payload.contiguous()), P, L_, B, q0, nq, k_in, k_out, _lib.ptr(oi),
        _lib.ptr(os_), _lib.ptr(o64), _lib.ptr(op), _lib.stream_ptr(dev)), "mmr_merge_topk_payload")
    return (oi, os_, o64) if payload is None else (oi, os_, o64, op)


def merge_topk_packed(packed: torch.Tensor, k_out: int, payload_width: int = 0, q0: int = 0, nq=None):
    """Merge of ONE packed all-gather buffer [L][B][k_in][2 + P] of 8-byte words per entry = {f64 score,
    int64 index bits, P f64 payload} (parallel.pack_lists) for queries [q0, q0 + nq) on device
    (mmr_merge_topk_packed) -> (idx, f32, f64) or (idx, f32, f64, payload (nq, k_out, P))."""
    _lib.require_gpu(packed)
    L_, B, k_in, W = packed.shape
    assert W == 2 + payload_width and packed.dtype == torch.float64
    packed = packed.contiguous()
    nq = B - q0 if nq is None else nq
    dev = packed.device
    oi = torch.empty((nq, k_out), dtype=torch.int64, device=dev)
    os_ = torch.empty((nq, k_out), dtype=torch.float32, device=dev)
    o64 = torch.empty((nq, k_out), dtype=torch.float64, device=dev)
    op = torch.empty((nq, k_out, payload_width), dtype=torch.float64, device=dev) if payload_width else None
    _lib.check(_lib.lib().mmr_merge_topk_packed(_lib.ptr(packed), payload_width, L_, B, q0, nq, k_in, k_out,
                                                _lib.ptr(oi), _lib.ptr(os_), _lib.ptr(o64), _lib.ptr(op),
                                                _lib.stream_ptr(dev)), "mmr_merge_topk_packed")
    return (oi, os_, o64) if op is None else (oi, os_, o64, op)


def rerank_mix(cand: torch.Tensor, comp: torch.Tensor, topk: int, alpha=0.6, beta=0.25, gamma=0.15,
               want_components=True):
    """After the shard merge (mmr_rerank_mix): cand (nq, kc) global indices (-1 = empty) + their raw
    components (nq, kc, 3) -> (idx (nq, topk), final, emb_n, lab_n, kg_n (nq, topk) f64 or None),
    bit-identical to GalleryIndex.rerank on one index holding the whole gallery."""
    _lib.require_gpu(cand)
    nq, kc = cand.shape
    dev = cand.device
    out_i = torch.empty((nq, topk), dtype=torch.int64, device=dev)
    outs = [torch.empty((nq, topk), dtype=torch.float64, device=dev) if want_components else None for _ in range(4)]
    _lib.check(_lib.lib().mmr_rerank_mix(_lib.ptr(cand.contiguous()), _lib.ptr(comp.contiguous()), nq, kc,
                                         float(alpha), float(beta), float(gamma), int(topk), _lib.ptr(out_i),
                                         *(_lib.ptr(o) for o in outs), _lib.stream_ptr(dev)), "mmr_rerank_mix")
    return (out_i, *outs)


class MI355XRetrievalEngine(RetrievalEngine):
    """Exact batched-cosine top-K on one MI355X (the brute-force path of retrieval_overlap.py:84-90)."""

    def __init__(self, features_path: Optional[str] = None, ids_path: Optional[str] = None,
                 device=None, dtype: str = "fp32", embs=None, ids=None, **_ignored):
        super().__init__(features_path, ids_path, embs=embs, ids=ids)
        if dtype not in ("fp32", "fp16"):
            raise ValueError(f"gallery dtype {dtype!r} (fp32 | fp16)")
        # fp16: an fp16 gallery file (BASELINE cfg5's fp16 gallery) builds the native fp16 index (its raw
        # rows are the only device copy, re-scored exactly); an f32 gallery keeps its f32 rows for the
        # exact f64 re-score and scans an fp16 copy of the unit rows — either way the results equal the
        # fp32 engine's (the reference upcasts with .astype("float32"), retrieval.py:24-32)
        src = self._raw if (dtype == "fp16" and self._raw is not None and self._raw.dtype == np.float16) else self.embs
        self.index = GalleryIndex(src, device=device, mode="f16" if dtype == "fp16" else "x3")
        self._raw = None
        self.device = self.index.device

    def search(self, Q, K: int = 10, check: bool = True):
        """Batched top-K. Q: (B,D) numpy or torch. Returns (idx (B,K') int64, scores (B,K') f32) with
        K' = min(K, N), as torch device tensors for torch input, numpy otherwise."""
        is_np = not isinstance(Q, torch.Tensor)
        q = torch.as_tensor(np.asarray(Q, np.float32) if is_np else Q)
        if q.dim() == 1:
            q = q[None]
        q = q.to(f"cuda:{self.device}", torch.float32)
        k_eff = min(int(K), len(self.ids))
        if k_eff <= 0:
            e = torch.empty((q.shape[0], 0))
            return (e.long().numpy(), e.numpy()) if is_np else (e.long(), e)
        idx, sc, st = self.index.search(q, k_eff, want_status=True)
        if check:
            check_status(st)
        if is_np:
            return idx.cpu().numpy(), sc.cpu().numpy()
        return idx, sc

    def retrieve(self, query_emb, K: int = 5, reranker=None, query_id=None, rerank_topk=None, **kwargs):
        """(D,) or (1,D) query -> (top-K ids, scores) descending (retrieval.py:34-39 contract).
        With a reranker and query_id, candidates are re-scored like retrieval.py:256-269."""
        q = np.asarray(query_emb, dtype=np.float32).reshape(1, -1)
        idx, sc = self.search(q, K)
        ids = [self.ids[i] for i in idx[0].tolist()]
        scores = [float(s) for s in sc[0].tolist()]
        if reranker is not None and query_id is not None:
            cand_embs = self.get_embeddings_for_ids(ids)
            lookup = {str(r): e for r, e in zip(ids, cand_embs)}
            lookup[str(query_id)] = (self.embs[self.id2idx[str(query_id)]]
                                     if str(query_id) in self.id2idx else q.reshape(-1))
            reranked = reranker.rerank(query_id=query_id, candidate_ids=ids, candidate_embs=cand_embs,
                                       candidate_emb_lookup=lookup, topk=rerank_topk or K)
            ids = [t[0] for t in reranked]
            scores = [t[1] for t in reranked]
        return ids, scores

    def close(self):
        self.index.close()


class DLSRetrievalEngine(MI355XRetrievalEngine):
    """DenseLinkSearch (retrieval.py:53-271).  The O(N^2) part — the link graph of
    _build_link_graph (retrieval.py:121-138) — is an exact self-join on the GPU
    (mmr_index_link_graph: the row itself excluded, score >= link_threshold, first max_links by
    score desc / index asc).  The query-time greedy walk (retrieval.py:140-271) is the reference's
    sequential, approximate host algorithm (random seeds, a (-sim, idx) heap, the visited set) and
    runs here exactly as there; exact retrieval is MI355XRetrievalEngine.search.
    The graph cache is an .npz (offsets + flat neighbours + dim), never a pickle."""

    def __init__(self, features_path: Optional[str] = None, ids_path: Optional[str] = None,
                 link_threshold: float = 0.5, max_links: int = 10, fdb_path: Optional[str] = None,
                 name: Optional[str] = None, device=None, embs=None, ids=None, **_ignored):
        super().__init__(features_path, ids_path, device=device, embs=embs, ids=ids)
        self.fdb_path = self.cache_path(features_path, fdb_path, name)
        graph = self._load_cache()
        if graph is None:
            graph = self._build_link_graph(link_threshold, max_links)
            self._save_cache(graph)
        self.link_graph = graph

    @staticmethod
    def cache_path(features_path, fdb_path=None, name=None):
        """Link-graph cache file (retrieval.py:72-79): fdb_path if given, else `name` or
        '<features stem>_link_graph' inside the feature-DB directory — $MMR_FEATURE_DB_DIR when set
        (the reference's FEATURES_PATH), else the features file's directory; always an .npz (a '.pkl'
        suffix is replaced, any other name gets '.npz' appended — np.savez would append it anyway).
        The parent directory is created (retrieval.py:82).  None for an in-memory gallery with
        neither a path nor a name."""
        import os
        db_dir = os.environ.get("MMR_FEATURE_DB_DIR")
        if fdb_path:
            p = str(fdb_path)
        elif features_path is not None or (name and db_dir):
            d = db_dir or os.path.dirname(os.path.abspath(str(features_path)))
            stem = os.path.splitext(os.path.basename(str(features_path)))[0] if features_path is not None else ""
            p = os.path.join(d, str(name) if name else f"{stem}_link_graph")
        elif name:
            p = str(name)
        else:
            return None
        if p.endswith(".pkl"):
            p = p[:-4]
        p = p if p.endswith(".npz") else p + ".npz"
        os.makedirs(os.path.dirname(os.path.abspath(p)), exist_ok=True)
        return p

    def _load_cache(self):
        import os
        if not self.fdb_path or not os.path.exists(self.fdb_path):
            return None
        try:
            f = np.load(self.fdb_path, allow_pickle=False)
            off, flat, dim = f["offsets"], f["flat"], int(f["dim"])
        except (OSError, KeyError, ValueError):
            return None
        if len(off) - 1 != self.embs.shape[0] or dim != self.embs.shape[1]:
            return None  # shape mismatch -> rebuild (retrieval.py:102-108)
        return [flat[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]

    def _save_cache(self, graph):
        if not self.fdb_path:
            return
        off = np.cumsum([0] + [len(x) for x in graph]).astype(np.int64)
        flat = np.array([j for x in graph for j in x], np.int64)
        np.savez(self.fdb_path, offsets=off, flat=flat, dim=np.int64(self.embs.shape[1]))

    def _build_link_graph(self, threshold: float, max_links: int) -> List[List[int]]:
        nbr, cnt = self.index.link_graph(threshold, max_links)
        nbr, cnt = nbr.cpu().numpy(), cnt.cpu().numpy()
        return [nbr[i, :cnt[i]].tolist() for i in range(len(cnt))]

    def retrieve(self, query_emb, K: int = 5, seed_size: int = 5, max_steps: int = 100,
                 candidate_multiplier: int = 10, reranker=None, query_id=None, rerank_topk=None,
                 seed=None, **kwargs):
        import heapq
        q = np.asarray(query_emb).astype("float32").reshape(-1)
        N = self.embs.shape[0]
        if len(self.link_graph) != N:
            raise RuntimeError(f"Link graph size {len(self.link_graph)} != embeddings {N}. Rebuild or delete "
                               f"your cache.")
        if seed is not None:
            np.random.seed(seed)
        elif query_id is not None:
            np.random.seed(abs(hash(str(query_id))) % (2 ** 32))  # process-salted, as in the reference
        else:
            np.random.seed(None)
        seeds = np.random.choice(N, size=min(seed_size, N), replace=False).tolist()
        visited = set(seeds)
        q_norm = np.linalg.norm(q) + 1e-6

        def sim(i):
            e = self.embs[i]
            return float(e @ q / (np.linalg.norm(e) * q_norm + 1e-12))
        heap = []
        for i in seeds:
            heapq.heappush(heap, (-sim(i), i))
        R = max(candidate_multiplier * K, seed_size)
        steps = 0
        while steps < max_steps and heap:
            _, best = heapq.heappop(heap)
            improved = False
            for nbr in self.link_graph[best]:
                if nbr < 0 or nbr >= N or nbr in visited:
                    continue
                visited.add(nbr)
                heapq.heappush(heap, (-sim(nbr), nbr))
                improved = True
            if len(heap) > R:
                heap = heapq.nsmallest(R, heap)
                heapq.heapify(heap)
            if not improved:
                break
            steps += 1
        top = sorted([(-ns, i) for ns, i in heapq.nsmallest(K, heap)], reverse=True)
        ids = [self.ids[i] for _, i in top]
        scores = [s for s, _ in top]
        if reranker is not None and query_id is not None:
            cand_embs = self.get_embeddings_for_ids(ids)
            lookup = {str(r): e for r, e in zip(ids, cand_embs)}
            lookup[str(query_id)] = (self.embs[self.id2idx[str(query_id)]] if str(query_id) in self.id2idx else q)
            out = reranker.rerank(query_id=query_id, candidate_ids=ids, candidate_embs=cand_embs,
                                  candidate_emb_lookup=lookup, topk=rerank_topk or K)
            ids = [t[0] for t in out]
            scores = [t[1] for t in out]
        return ids, scores


def make_retrieval_engine(features_path: str, ids_path: str, method: str = "dls", **kwargs) -> RetrievalEngine:
    """Factory (retrieval.py:273-304; default method "dls" as there). method: "dls" ->
    DenseLinkSearch with the GPU-built link graph (link_threshold, max_links, fdb_path, name as in
    the reference); "mi355x" (aliases "exact", "brute") -> exact GPU engine; "mi355x_sharded" ->
    row-sharded over torch.distributed ranks."""
    method = method.lower()
    if method in ("mi355x", "exact", "brute", "bruteforce"):
        return MI355XRetrievalEngine(features_path, ids_path, device=kwargs.get("device"),
                                     dtype=kwargs.get("dtype", "fp32"))
    if method in ("mi355x_sharded", "sharded"):
        from .parallel import ShardedRetrievalEngine
        return ShardedRetrievalEngine(features_path, ids_path, dtype=kwargs.get("dtype", "fp32"))
    if method == "dls":
        return DLSRetrievalEngine(features_path, ids_path, link_threshold=kwargs.get("link_threshold", 0.5),
                                  max_links=kwargs.get("max_links", 10), fdb_path=kwargs.get("fdb_path"),
                                  name=kwargs.get("name"), device=kwargs.get("device"))
    raise ValueError(f"Unknown retrieval method: {method}")
