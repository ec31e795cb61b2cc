"""ORACLE (test infrastructure): brute-force cosine top-K restated in numpy.

sklearn_topk   the reference's exact path, src/Evaluate/retrieval_overlap.py:84-90:
               sim = sklearn.metrics.pairwise.cosine_similarity(Q, G)  (f32: rows normalised by
               sklearn.preprocessing.normalize — zero rows stay zero — then Q_n @ G_n.T in f32),
               idx = np.argsort(sim[i])[::-1][:K].  Same idiom at retrieval.py:128-137.
exact_topk     the semantics the GPU path implements: cosine in f64 of the raw f32 rows (0 when a
               norm is 0), ranked by score desc then gallery index asc (deterministic ties).
"""
import numpy as np


def sklearn_cosine_f32(Q, G):
    """cosine_similarity(Q, G) as sklearn 1.7 computes it for f32 input (normalize + gemm)."""
    def _norm(X):
        X = np.asarray(X, np.float32)
        n = np.sqrt(np.einsum("ij,ij->i", X, X, dtype=np.float32))
        n[n == 0.0] = 1.0
        return X / n[:, None]
    return _norm(Q) @ _norm(G).T


def sklearn_topk(Q, G, K):
    sim = sklearn_cosine_f32(Q, G)
    idx = np.stack([np.argsort(sim[i])[::-1][:K] for i in range(sim.shape[0])])
    return idx.astype(np.int64), np.take_along_axis(sim, idx, 1).astype(np.float32)


def exact_scores(Q, G):
    Q = np.asarray(Q, np.float64)
    G = np.asarray(G, np.float64)
    qn = np.linalg.norm(Q, axis=1)
    gn = np.linalg.norm(G, axis=1)
    dots = Q @ G.T
    den = qn[:, None] * gn[None, :]
    with np.errstate(invalid="ignore", divide="ignore"):
        s = np.where(den > 0, dots / np.where(den > 0, den, 1.0), 0.0)
    return s


def exact_topk(Q, G, K, chunk=256):
    """(idx int64 (B,K'), score f64 (B,K')), K' = min(K, N); score desc, index asc."""
    N = np.asarray(G).shape[0]
    K = min(K, N)
    outs_i, outs_s = [], []
    for c0 in range(0, np.asarray(Q).shape[0], chunk):
        s = exact_scores(np.asarray(Q)[c0:c0 + chunk], G)
        for row in s:
            if K < N:
                part = np.argpartition(-row, K - 1)[:K]
                # include every element tied with the K-th so the index tie-break is exact
                kth = row[part].min()
                part = np.nonzero(row >= kth)[0]
            else:
                part = np.arange(N)
            order = np.lexsort((part, -row[part]))[:K]
            sel = part[order]
            outs_i.append(sel)
            outs_s.append(row[sel])
    return np.asarray(outs_i, np.int64).reshape(-1, K), np.asarray(outs_s, np.float64).reshape(-1, K)


def topk_equivalent(idx_ref, score_ref, idx_got, score_got, tie_tol=1e-6, score_tol=1e-4):
    """Parity criterion of BASELINE.md §3: identical indices, except that positions whose reference
    scores are within tie_tol of each other are compared as sets; scores within score_tol.
    Returns (ok, message)."""
    idx_ref = np.asarray(idx_ref)
    idx_got = np.asarray(idx_got)
    if idx_ref.shape != idx_got.shape:
        return False, f"shape {idx_got.shape} != {idx_ref.shape}"
    err = np.max(np.abs(np.asarray(score_ref, np.float64) - np.asarray(score_got, np.float64))) if idx_ref.size else 0.0
    if err > score_tol:
        return False, f"score error {err:.3e} > {score_tol}"
    for q in range(idx_ref.shape[0]):
        if np.array_equal(idx_ref[q], idx_got[q]):
            continue
        s = np.asarray(score_ref[q], np.float64)
        K = len(s)
        # group positions into tie runs; the last run may extend past K (compare as sets within
        # the run only where the run is internal; a boundary run only needs membership slack)
        i = 0
        while i < K:
            j = i
            while j + 1 < K and abs(s[j + 1] - s[i]) <= tie_tol:
                j += 1
            a, b = set(idx_ref[q, i:j + 1].tolist()), set(idx_got[q, i:j + 1].tolist())
            boundary = (j == K - 1)
            if a != b and not boundary:
                return False, f"query {q}: positions {i}..{j} differ {sorted(a)} vs {sorted(b)}"
            if a != b and boundary:
                # near-tied at the cut: the swapped-in rows must have a score within tie_tol
                sg = np.asarray(score_got[q], np.float64)
                if np.max(np.abs(sg[i:j + 1] - s[i])) > tie_tol + 1e-6:
                    return False, f"query {q}: boundary run {i}..{j} differs beyond the tie tolerance"
            i = j + 1
    return True, f"ok (max score err {err:.2e})"


def boundary_gaps(score_f64_sorted):
    """Per query: the smallest gap between consecutive exact scores in the list (diagnostic)."""
    s = np.asarray(score_f64_sorted, np.float64)
    if s.shape[1] < 2:
        return np.full(s.shape[0], np.inf)
    return np.min(s[:, :-1] - s[:, 1:], axis=1)
