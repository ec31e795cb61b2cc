"""Gallery row-sharding over one process per GPU (torch.distributed: RCCL over xGMI on MI355X,
gloo on CPU for tests).  SURVEY.md §8e: the reference is single-process; this is the one
multi-GPU component the path needs.

Each rank owns rows [start_r, end_r) of the gallery (balanced split).  A search:
  1. all-gather the ranks' query batches (every rank scores every query against its shard),
  2. local exact top-K on the shard (libmmr; global index = local + start_r, f64 scores),
  3. ONE all-gather of the per-shard lists packed into 8-byte words per entry {f64 score, int64
     index (+ the rerank payload)} (pack_lists) — 16*Q*K bytes per rank, latency-bound (30 KB at
     Q=256, K=10): one collective per query batch for the results, no data-path exchange,
  4. deterministic k-way merge straight from the gathered buffer (merge_gathered ->
     mmr_merge_topk_packed): score desc, then global index asc — so the sharded result is
     bit-identical to the single-device result (ranking on the same f64 scores).
Sharded rerank (BASELINE config 5's KG-rerank head at world > 1; Reranker.rerank,
src/Retrieval/reranker.py:240-333, min-max scales each component over the FINAL candidate list, so
it must run after the merge): each shard computes its candidates' raw {emb cosine, label Jaccard, KG
cosine} where the rows and tables live (mmr_index_rerank_components), the components ride with the
(score, index) lists through the same all-gather and the merge (mmr_merge_topk_payload), and the
min-max / mix / rank runs on the merged list (mmr_rerank_mix) — bit-identical to one index.
"""
import numpy as np
import torch
import torch.distributed as dist

from .retrieval import GalleryIndex, RetrievalEngine, merge_topk_packed, rerank_mix


def shard_bounds(n, world):
    """Balanced contiguous row ranges: [(start, end)] per rank."""
    base, rem = divmod(int(n), int(world))
    out, s = [], 0
    for r in range(world):
        e = s + base + (1 if r < rem else 0)
        out.append((s, e))
        s = e
    return out


def merge_topk_host(scores64, idx, k_out, payload=None):
    """Same merge as the HIP kernel (mmr_merge_topk[_payload]) for host-resident lists [L][B][k_in]
    (a CPU coordinator, or the gloo test path): score desc, index asc, idx -1 = empty; payload
    [L][B][k_in][P] rides with each entry (4th output (B, k_out, P), zeros for empty slots)."""
    L_, B, k_in = idx.shape
    src = torch.arange(L_ * k_in).view(1, -1).expand(B, -1)
    s = scores64.permute(1, 0, 2).reshape(B, L_ * k_in).to(torch.float64)
    i = idx.permute(1, 0, 2).reshape(B, L_ * k_in).to(torch.int64)
    valid = i >= 0
    s = torch.where(valid, s, torch.full_like(s, -float("inf")))
    ikey = torch.where(valid, i, torch.full_like(i, torch.iinfo(torch.int64).max))
    o1 = torch.argsort(ikey, dim=1, stable=True)
    s1, i1, src1 = torch.gather(s, 1, o1), torch.gather(ikey, 1, o1), torch.gather(src, 1, o1)
    o2 = torch.argsort(s1, dim=1, descending=True, stable=True)
    s2, i2 = torch.gather(s1, 1, o2)[:, :k_out], torch.gather(i1, 1, o2)[:, :k_out]
    src2 = torch.gather(src1, 1, o2)[:, :k_out]
    bad = i2 == torch.iinfo(torch.int64).max
    i2 = torch.where(bad, torch.full_like(i2, -1), i2)
    if s2.shape[1] < k_out:  # fewer candidates than k_out in total
        pad = k_out - s2.shape[1]
        s2 = torch.cat([s2, torch.full((B, pad), -float("inf"), dtype=s2.dtype)], 1)
        i2 = torch.cat([i2, torch.full((B, pad), -1, dtype=i2.dtype)], 1)
        src2 = torch.cat([src2, torch.zeros((B, pad), dtype=src2.dtype)], 1)
    if payload is None:
        return i2, s2.to(torch.float32), s2
    P = payload.shape[-1]
    pf = payload.permute(1, 0, 2, 3).reshape(B, L_ * k_in, P).to(torch.float64)
    pay = torch.gather(pf, 1, src2.unsqueeze(-1).expand(-1, -1, P))
    pay = torch.where((i2 >= 0).unsqueeze(-1), pay, torch.zeros_like(pay))
    return i2, s2.to(torch.float32), s2, pay


def rerank_mix_host(cand, comp, topk, alpha=0.6, beta=0.25, gamma=0.15):
    """Host form of mmr_rerank_mix (the gloo / CPU-coordinator path): per query, min-max scale each
    raw component over the valid candidates (constant -> 0, reranker.py:151-159), final =
    alpha e + beta l + gamma k, rank by final desc with equal finals -> later candidate first
    (np.argsort(final)[::-1]); -> (idx (nq, topk) int64, -1 padded; final, emb_n, lab_n, kg_n f64)."""
    cand = cand.to(torch.int64)
    comp = comp.to(torch.float64)
    nq, kc = cand.shape
    out = [torch.full((nq, topk), -1, dtype=torch.int64)] + [torch.zeros((nq, topk), dtype=torch.float64)
                                                            for _ in range(4)]
    for qi in range(nq):
        valid = [c for c in range(kc) if int(cand[qi, c]) >= 0]
        if not valid:
            continue
        scaled = []
        for p in range(3):
            x = [float(comp[qi, c, p]) for c in valid]
            lo, hi = min(x), max(x)
            scaled.append([0.0 if hi - lo == 0 else (v - lo) / (hi - lo) for v in x])
        fin = [alpha * scaled[0][j] + beta * scaled[1][j] + gamma * scaled[2][j] for j in range(len(valid))]
        order = sorted(range(len(valid)), key=lambda j: (-fin[j], -j))[:topk]
        for r, j in enumerate(order):
            out[0][qi, r] = cand[qi, valid[j]]
            out[1][qi, r] = fin[j]
            for p in range(3):
                out[2 + p][qi, r] = scaled[p][j]
    return tuple(out)


def pack_lists(idx, s64, comp=None, status=None):
    """One rank's search result as the single all-gather payload: (Q, K) int64 + (Q, K) f64 (+ (Q, K, P)
    f64 rerank components) -> (Q + 1, K, 2 + P) f64 words {score, index bits, payload} (int64 bits
    carried in an 8-byte slot: copies and all-gathers move bytes, nothing re-interprets them).  Row Q is
    the rank's status row: word [Q, 0, 0] = its max per-query search status (a device scalar or None =
    0), so every rank sees every rank's status after the one exchange and all raise together (a rank
    raising alone before the exchange would leave the others blocked in the collective)."""
    parts = [s64.to(torch.float64).unsqueeze(-1), idx.to(torch.int64).contiguous().view(torch.float64).unsqueeze(-1)]
    if comp is not None:
        parts.append(comp.to(torch.float64))
    body = torch.cat(parts, -1)
    srow = torch.zeros((1,) + tuple(body.shape[1:]), dtype=torch.float64, device=body.device)
    if status is not None:
        srow[0, 0, 0] = status.to(device=body.device, dtype=torch.float64)
    return torch.cat([body, srow], 0).contiguous()


def gathered_status(gathered):
    """Max status over the ranks of an all-gathered pack_lists buffer [world][Q + 1][K][W] (host int)."""
    return int(gathered[:, -1, 0, 0].max().item())


def merge_gathered(gathered, q0, nq, k_out, payload_width=0):
    """The post-gather merge: gathered [world][Q + 1][K][2 + P] (all ranks' pack_lists, world = shards)
    -> this rank's queries [q0, q0 + nq): (idx, f32, f64) (+ payload (nq, k_out, P)).  Device tensors:
    mmr_merge_topk_packed reads the gathered buffer directly; host tensors (gloo): merge_topk_host."""
    if gathered.is_cuda:
        return merge_topk_packed(gathered, k_out, payload_width, q0=q0, nq=nq)
    g = gathered[:, q0:q0 + nq]
    s = g[..., 0].contiguous()
    i = g[..., 1].contiguous().view(torch.int64)
    pay = g[..., 2:].contiguous() if payload_width else None
    return merge_topk_host(s, i, k_out, payload=pay)


class ShardedIndex:
    """This rank's gallery shard + the collective search.

    `local_search(q, k) -> (idx, f64) or (idx, f64, status)` may be injected (tests); by default it
    is the rank's GPU GalleryIndex in `mode` ("x3" | "f16" | "f32").  A non-zero per-query status
    would flag an inexact list; the selection kernel resolves candidate-buffer overflow in-kernel, so
    it never occurs — this is a guard: an injected `fallback_search` re-runs such queries, else the
    status rides in the result exchange (pack_lists' status row) and EVERY rank raises after it (no
    mode switch inside a collective: ADVICE r03; no rank raising alone before it: ADVICE r04)."""

    def __init__(self, gallery_rows, n_total, start, group=None, device=None, local_search=None, mode="x3",
                 fallback_search=None, local_components=None, index=None, status_out=None):
        """index: an existing GalleryIndex of this rank's rows (instead of building one from
        gallery_rows).  status_out: a device int32 scalar that accumulates the max per-query
        search status without a host sync (a benchmark loop checks it once afterwards; the
        selection kernel resolves every overflow in-kernel, so the re-run path is a guard) —
        with it, flagged queries are not re-run here."""
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.n_total, self.start = int(n_total), int(start)
        self.index = index
        self.status_out = status_out
        if local_search is None and index is not None:
            local_search = self._index_search
        if local_search is None:
            # fp16 rows build the native fp16 index in f16 mode only; any other mode takes them upcast
            # (as from_full does: GalleryIndex rejects fp16 rows with a non-f16 mode — ADVICE r05)
            if mode != "f16":
                if isinstance(gallery_rows, torch.Tensor) and gallery_rows.dtype == torch.float16:
                    gallery_rows = gallery_rows.float()
                elif isinstance(gallery_rows, np.ndarray) and gallery_rows.dtype == np.float16:
                    gallery_rows = gallery_rows.astype(np.float32)
            self.index = GalleryIndex(gallery_rows, device=device, idx_base=start, mode=mode)
            local_search = self._index_search
        self.local_search = local_search
        self.fallback_search = fallback_search
        self.local_components = local_components  # (q, cand) -> (nq, kc, 3) raw rerank components
        self.reruns = 0  # queries re-run through fallback_search (diagnostic)

    def _index_search(self, q, k):
        i, _, s64, st = self.index.search(q, k, want_f64=True, want_status=True)
        return i, s64, st

    @classmethod
    def from_full(cls, gallery, group=None, device=None, local_search=None, mode="x3", fallback_search=None):
        """gallery may be a memmap: only this rank's rows are read (and converted to f32)."""
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        s, e = shard_bounds(len(gallery), world)[rank]
        if isinstance(gallery, torch.Tensor):  # fp16 rows stay fp16 only for an f16 index (GalleryIndex)
            rows = gallery[s:e]
            if rows.dtype == torch.float16 and mode != "f16":
                rows = rows.float()
        else:  # an fp16 gallery in f16 mode stays fp16 (the native fp16 index: 2 B per element on device)
            keep16 = np.asarray(gallery[:0]).dtype == np.float16 and mode == "f16"
            rows = np.ascontiguousarray(gallery[s:e], dtype=np.float16 if keep16 else np.float32)
        return cls(rows, len(gallery), s, group=group, device=device, local_search=local_search, mode=mode,
                   fallback_search=fallback_search)

    def _local(self, q, k):
        """-> (idx, f64, status): status = the device max of the per-query statuses still flagged after
        the fallback re-run (None when there is nothing to report: no status, or status_out took it)."""
        out = self.local_search(q, k)
        i, s64 = out[0], out[1]
        st = out[2] if len(out) > 2 else None
        if st is None or not st.numel():
            return i, s64, None
        if self.status_out is not None:
            torch.maximum(self.status_out, st.max().to(self.status_out.dtype), out=self.status_out)
            return i, s64, None
        if self.fallback_search is None:
            return i, s64, st.max()  # raised on every rank after the exchange (_raise_status)
        if int(st.max().item()) != 0:
            bad = torch.nonzero(st != 0).flatten()
            i2, s2 = self.fallback_search(q[bad.to(q.device)].contiguous(), k)
            i, s64 = i.clone(), s64.clone()
            i[bad.to(i.device)] = i2.to(i.device, i.dtype)
            s64[bad.to(s64.device)] = s2.to(s64.device, s64.dtype)
            self.reruns += int(bad.numel())
        return i, s64, None

    @staticmethod
    def _raise_status(g, st):
        """After the exchange: every rank holds every rank's status row, so all raise together."""
        if st is not None:
            worst = gathered_status(g)
            if worst != 0:
                raise RuntimeError(f"mmr_index_search returned status {worst} on a shard (collective search)")

    def search(self, q_local, k):
        """Collective: every rank passes its own (b, D) queries (same b on every rank); returns
        this rank's (idx int64 (b,k), score f32 (b,k), score f64 (b,k)) over the whole gallery.
        Two collectives: the queries' all-gather and ONE packed all-gather of the result lists."""
        b = q_local.shape[0]
        allq = self._gather_queries(q_local)
        i, s64, st = self._local(allq, k)
        g = self._gather(pack_lists(i, s64, status=st))
        self._raise_status(g, st)
        return merge_gathered(g, self.rank * b, b, k)

    def _gather_queries(self, q_local):
        allq = torch.empty((self.world * q_local.shape[0],) + tuple(q_local.shape[1:]), dtype=q_local.dtype,
                           device=q_local.device)
        dist.all_gather_into_tensor(allq, q_local.contiguous(), group=self.group)
        return allq

    def _gather(self, packed):
        g = torch.empty((self.world * packed.shape[0],) + tuple(packed.shape[1:]), dtype=packed.dtype,
                        device=packed.device)
        dist.all_gather_into_tensor(g, packed, group=self.group)
        return g.view((self.world,) + tuple(packed.shape))

    def _components(self, q, cand, tables):
        """Raw rerank components of this shard's candidates (nq, kc, 3) f64."""
        if self.local_components is not None:
            return self.local_components(q, cand)
        q_lab, g_lab, q_kg, g_kg = tables
        return self.index.rerank_components(q, cand, q_lab, g_lab, q_kg, g_kg)

    def search_rerank(self, q_local, k, tables=None, topk=None, alpha=0.6, beta=0.25, gamma=0.15):
        """Collective exact top-k + the KG / label rerank of those k candidates (config 5 at world >
        1).  tables = (q_labels for ALL world*b queries in all-gather order, this shard's g_labels,
        q_kg for all queries, this shard's g_kg) as device tensors (GPU path), or None when
        `local_components` was injected.  Returns this rank's (idx (b, topk), final, emb_n, lab_n,
        kg_n) — bit-identical to GalleryIndex.rerank of the single-index top-k."""
        b = q_local.shape[0]
        topk = k if topk is None else topk
        allq = self._gather_queries(q_local)
        i, s64, st = self._local(allq, k)
        comp = self._components(allq, i, tables).to(s64.device)
        g = self._gather(pack_lists(i, s64, comp, status=st))   # one collective: lists + components
        self._raise_status(g, st)
        mi, _, _, mc = merge_gathered(g, self.rank * b, b, k, payload_width=comp.shape[-1])
        if mi.is_cuda:
            return rerank_mix(mi, mc, topk, alpha, beta, gamma)
        return rerank_mix_host(mi, mc, topk, alpha, beta, gamma)


class ShardedRetrievalEngine(RetrievalEngine):
    """make_retrieval_engine(method="mi355x_sharded"): every rank mmaps the .npy, keeps its row
    shard on its GPU; retrieve()/search() are collective calls (all ranks, same batch size).
    dtype "fp32" scans the bf16x3 split copy, "fp16" the fp16 scan (an fp16 .npy — BASELINE cfg5's fp16
    gallery — becomes a native fp16 index per shard: its raw rows are the only device copy); both rank
    exactly (f64 re-score from the gallery's own rows), so results are identical.
    Host memory: `embs` stays the memmap (no whole-gallery f32 copy per rank, unlike the ABC's
    astype), so a rank's resident host bytes are its shard's, read once into its GPU."""

    def __init__(self, features_path=None, ids_path=None, dtype="fp32", embs=None, ids=None, group=None):
        if embs is None:
            embs = np.load(features_path, mmap_mode="r")
        super().__init__(features_path, ids_path, embs=embs, ids=ids, lazy=True)
        if dtype not in ("fp32", "fp16"):
            raise ValueError(f"gallery dtype {dtype!r} (fp32 | fp16)")
        self.sharded = ShardedIndex.from_full(self.embs, group=group, device=torch.cuda.current_device(),
                                              mode="f16" if dtype == "fp16" else "x3")

    def search(self, Q, K=10):
        is_np = not isinstance(Q, torch.Tensor)
        q = torch.as_tensor(np.asarray(Q, np.float32) if is_np else Q).to("cuda", torch.float32)
        k_eff = min(int(K), len(self.ids))
        i, s, _ = self.sharded.search(q, k_eff)
        return (i.cpu().numpy(), s.cpu().numpy()) if is_np else (i, s)

    def retrieve(self, query_emb, K=5, **kwargs):
        idx, sc = self.search(np.asarray(query_emb, np.float32).reshape(1, -1), K)
        return [self.ids[j] for j in idx[0].tolist()], [float(x) for x in sc[0].tolist()]
