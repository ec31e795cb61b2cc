"""Gallery row-sharding over one process per GPU (torch.distributed: RCCL over xGMI on MI355X,
gloo on CPU for tests).  SURVEY.md §8e: the reference is single-process; this is the one
multi-GPU component the path needs.

Each rank owns rows [start_r, end_r) of the gallery (balanced split).  A search:
  1. all-gather the ranks' query batches (every rank scores every query against its shard),
  2. local exact top-K on the shard (libmmr; global index = local + start_r, f64 scores),
  3. all-gather the per-shard (f64 score, int64 index) lists — 16*Q*K bytes per rank, latency-
     bound (30 KB at Q=256, K=10): one collective per query batch, no data-path exchange,
  4. deterministic k-way merge: score desc, then global index asc — so the sharded result is
     bit-identical to the single-device result (ranking on the same f64 scores).
"""
import numpy as np
import torch
import torch.distributed as dist

from .retrieval import GalleryIndex, RetrievalEngine, check_status, merge_topk


def shard_bounds(n, world):
    """Balanced contiguous row ranges: [(start, end)] per rank."""
    base, rem = divmod(int(n), int(world))
    out, s = [], 0
    for r in range(world):
        e = s + base + (1 if r < rem else 0)
        out.append((s, e))
        s = e
    return out


def merge_topk_host(scores64, idx, k_out):
    """Same merge as the HIP kernel (mmr_merge_topk) for host-resident lists [L][B][k_in]
    (a CPU coordinator, or the gloo test path): score desc, index asc, idx -1 = empty."""
    L_, B, k_in = idx.shape
    s = scores64.permute(1, 0, 2).reshape(B, L_ * k_in).to(torch.float64)
    i = idx.permute(1, 0, 2).reshape(B, L_ * k_in).to(torch.int64)
    valid = i >= 0
    s = torch.where(valid, s, torch.full_like(s, -float("inf")))
    ikey = torch.where(valid, i, torch.full_like(i, torch.iinfo(torch.int64).max))
    o1 = torch.argsort(ikey, dim=1, stable=True)
    s1, i1 = torch.gather(s, 1, o1), torch.gather(ikey, 1, o1)
    o2 = torch.argsort(s1, dim=1, descending=True, stable=True)
    s2, i2 = torch.gather(s1, 1, o2)[:, :k_out], torch.gather(i1, 1, o2)[:, :k_out]
    bad = i2 == torch.iinfo(torch.int64).max
    i2 = torch.where(bad, torch.full_like(i2, -1), i2)
    if s2.shape[1] < k_out:  # fewer candidates than k_out in total
        pad = k_out - s2.shape[1]
        s2 = torch.cat([s2, torch.full((B, pad), -float("inf"), dtype=s2.dtype)], 1)
        i2 = torch.cat([i2, torch.full((B, pad), -1, dtype=i2.dtype)], 1)
    return i2, s2.to(torch.float32), s2


class ShardedIndex:
    """This rank's gallery shard + the collective search.

    `local_search(q, k) -> (idx, f64) or (idx, f64, status)` may be injected (tests); by default it
    is the rank's GPU GalleryIndex in `mode` ("x3" | "f16" | "f32").  A non-zero per-query status
    (candidate-buffer overflow — the library now resolves it in-kernel, so this is a guard) makes
    those queries re-run through `fallback_search` (default: the same index in "x3", as
    MI355XRetrievalEngine did) before the lists are exchanged, so every rank always contributes an
    exact list."""

    def __init__(self, gallery_rows, n_total, start, group=None, device=None, local_search=None, mode="x3",
                 fallback_search=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.n_total, self.start = int(n_total), int(start)
        self.index = None
        if local_search is None:
            self.index = GalleryIndex(gallery_rows, device=device, idx_base=start, mode=mode)
            local_search = self._index_search
            if fallback_search is None:
                fallback_search = self._index_search_x3
        self.local_search = local_search
        self.fallback_search = fallback_search
        self.reruns = 0  # queries re-run through fallback_search (diagnostic)

    def _index_search(self, q, k):
        i, _, s64, st = self.index.search(q, k, want_f64=True, want_status=True)
        return i, s64, st

    def _index_search_x3(self, q, k):
        mode = self.index.mode
        self.index.set_mode("x3")
        try:
            i, _, s64, st = self.index.search(q, k, want_f64=True, want_status=True)
        finally:
            self.index.set_mode(mode)
        check_status(st)
        return i, s64

    @classmethod
    def from_full(cls, gallery, group=None, device=None, local_search=None, mode="x3", fallback_search=None):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        s, e = shard_bounds(len(gallery), world)[rank]
        rows = gallery[s:e]
        return cls(rows, len(gallery), s, group=group, device=device, local_search=local_search, mode=mode,
                   fallback_search=fallback_search)

    def _local(self, q, k):
        out = self.local_search(q, k)
        i, s64 = out[0], out[1]
        st = out[2] if len(out) > 2 else None
        if st is not None and st.numel() and int(st.max().item()) != 0:
            if self.fallback_search is None:
                check_status(st)
            bad = torch.nonzero(st != 0).flatten()
            i2, s2 = self.fallback_search(q[bad.to(q.device)].contiguous(), k)
            i, s64 = i.clone(), s64.clone()
            i[bad.to(i.device)] = i2.to(i.device, i.dtype)
            s64[bad.to(s64.device)] = s2.to(s64.device, s64.dtype)
            self.reruns += int(bad.numel())
        return i, s64

    def search(self, q_local, k):
        """Collective: every rank passes its own (b, D) queries (same b on every rank); returns
        this rank's (idx int64 (b,k), score f32 (b,k), score f64 (b,k)) over the whole gallery."""
        b = q_local.shape[0]
        allq = torch.empty((self.world * b,) + tuple(q_local.shape[1:]), dtype=q_local.dtype,
                           device=q_local.device)
        dist.all_gather_into_tensor(allq, q_local.contiguous(), group=self.group)
        i, s64 = self._local(allq, k)
        gi = torch.empty((self.world * i.shape[0], i.shape[1]), dtype=i.dtype, device=i.device)
        gs = torch.empty((self.world * s64.shape[0], s64.shape[1]), dtype=s64.dtype, device=s64.device)
        dist.all_gather_into_tensor(gi, i.contiguous(), group=self.group)
        dist.all_gather_into_tensor(gs, s64.contiguous(), group=self.group)
        gi = gi.view(self.world, i.shape[0], i.shape[1])
        gs = gs.view(self.world, s64.shape[0], s64.shape[1])
        if gi.is_cuda:
            mi, ms, m64 = merge_topk(gs, gi, k)
        else:
            mi, ms, m64 = merge_topk_host(gs, gi, k)
        sl = slice(self.rank * b, (self.rank + 1) * b)
        return mi[sl], ms[sl], m64[sl]


class ShardedRetrievalEngine(RetrievalEngine):
    """make_retrieval_engine(method="mi355x_sharded"): every rank mmaps the .npy, keeps its row
    shard on its GPU; retrieve()/search() are collective calls (all ranks, same batch size).
    dtype "fp32" scans the bf16x3 split copy, "fp16" the fp16 unit-row copy (BASELINE cfg5's fp16
    gallery); both rank exactly (f64 re-score from the f32 rows), so results are identical."""

    def __init__(self, features_path=None, ids_path=None, dtype="fp32", embs=None, ids=None, group=None):
        if embs is None:
            embs = np.load(features_path, mmap_mode="r")
        super().__init__(features_path, ids_path, embs=embs, ids=ids)
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
