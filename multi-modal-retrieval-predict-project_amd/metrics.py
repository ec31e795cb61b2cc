"""Retrieval metrics on id lists — same definitions as src/Helpers/retrieval_metrics.py.

precision_at_k  retrieval_metrics.py:4-11
recall_at_k     retrieval_metrics.py:74-79 (the module redefines it; the later, set-based one wins)
average_precision / mean_average_precision  :24-54
mean_reciprocal_rank  :56-72
ndcg_at_k  :81-89 (binary gains, ideal = the same gains sorted, i.e. normalised within the top-k)
Plus `ranking_metrics`, the exact brute-force evaluation of
src/Evaluate/retrieval_overlap.py:84-115 (first-relevant rank -> MRR, hit@k, recall@k over the whole
gallery), computed from top-k indices and label bitsets instead of a Python loop over N.
"""
import math

import numpy as np


def precision_at_k(retrieved_ids, relevant_ids, k=5):
    rel = set(relevant_ids)
    return sum(1 for r in retrieved_ids[:k] if r in rel) / k


def recall_at_k(retrieved, relevant, k=5):
    if len(relevant) == 0:
        return 0.0
    return len(set(retrieved[:k]) & set(relevant)) / len(set(relevant))


def average_precision(retrieved, relevant, k=None):
    if k is None:
        k = len(retrieved)
    hits, score = 0, 0.0
    for i, r in enumerate(retrieved[:k], start=1):
        if r in relevant:
            hits += 1
            score += hits / i
    return score / len(relevant) if relevant else 0.0


def mean_average_precision(all_retrieved, all_relevant, k=None):
    return float(np.mean([average_precision(r, s, k) for r, s in zip(all_retrieved, all_relevant)]))


def mean_reciprocal_rank(all_retrieved, all_relevant):
    rr = []
    for retrieved, relevant in zip(all_retrieved, all_relevant):
        v = 0.0
        for i, r in enumerate(retrieved, start=1):
            if r in relevant:
                v = 1.0 / i
                break
        rr.append(v)
    return float(np.mean(rr))


def ndcg_at_k(retrieved, relevant, k=5):
    gains = [1 if r in relevant else 0 for r in retrieved[:k]]
    dcg = sum(g / math.log2(i + 2) for i, g in enumerate(gains))
    idcg = sum(g / math.log2(i + 2) for i, g in enumerate(sorted(gains, reverse=True)))
    return dcg / idcg if idcg > 0 else 0.0


def _popcount_nonzero(a):
    return a != 0


def ranking_metrics(topk_idx, query_bits, gallery_bits, k, first_rank=None):
    """retrieval_overlap.py:84-115 from top-k indices.

    topk_idx (Q, >=k) int gallery indices in rank order; query_bits (Q,) / gallery_bits (N,) uint64
    label bitsets (relevance = any shared label).  `first_rank` (Q,) optional: 1-based rank of the
    first relevant gallery item in the full ranking (0 = none); when None it is taken from topk_idx
    (exact when the first relevant item is inside the returned list, else MRR counts 0 for it).
    Returns (mrr, hit@k, recall@k) like compute_ranking_metrics.
    """
    topk_idx = np.asarray(topk_idx)
    qb = np.asarray(query_bits, np.uint64)
    gb = np.asarray(gallery_bits, np.uint64)
    rel_top = _popcount_nonzero(gb[topk_idx] & qb[:, None])             # (Q, K')
    total_rel = _popcount_nonzero(gb[None, :] & qb[:, None]).sum(axis=1)  # (Q,)
    if first_rank is None:
        any_rel = rel_top.any(axis=1)
        first_rank = np.where(any_rel, rel_top.argmax(axis=1) + 1, 0)
    first_rank = np.asarray(first_rank)
    rr = np.where(first_rank > 0, 1.0 / np.maximum(first_rank, 1), 0.0)
    hits = ((first_rank > 0) & (first_rank <= k)).sum()
    rel_k = rel_top[:, :k].sum(axis=1)
    recalls = np.where(total_rel > 0, rel_k / np.maximum(total_rel, 1), 0.0)
    return float(np.mean(rr)), hits / len(qb), float(np.mean(recalls))
