"""ORACLE (test infrastructure): the DLS link graph, its greedy walk and the Reranker, restated.

link_graph     DLSRetrievalEngine._build_link_graph (src/Retrieval/retrieval.py:121-138):
               sim = cosine_similarity(embs) with the diagonal set to -1; per row the neighbours in
               descending similarity with sim >= threshold, first max_links.  Restated on the exact
               f64 cosine (0 for zero rows, like sklearn's normalize) with ties broken by the lower
               index (np.argsort is unstable there: the reference's tie order is unspecified).
walk_retrieve  DLSRetrievalEngine.retrieve (retrieval.py:140-271) without reranking: explicit seed ->
               np.random.seed(seed); np.random.choice seeds; (-sim, idx) heap; greedy expansion with
               the visited set, heap bounded to max(candidate_multiplier*K, seed_size) by
               heapq.nsmallest, stop at the first pop that adds nothing; top-K by (-sim, idx).
               The walk is the reference's host algorithm; sims follow retrieval.py:203-206,225.
rerank         Reranker.rerank (src/Retrieval/reranker.py:240-333): min-max scaled embedding cosine,
               label Jaccard and KG-vector cosine, alpha/beta/gamma mix, np.argsort(final)[::-1][:topk]
               (small lists: numpy's sort is an insertion sort, stable ascending, so equal finals come
               out with the later candidate first — restated explicitly).
record tables  Reranker.get_record_label_set / get_record_kg_vec (reranker.py:161-220): label sets
               from the labels CSV (columns whose value int()s to 1), KG vector = report node, else
               mean (or LabelAttention-pooled) label-node vectors, else zeros.
"""
import heapq

import numpy as np

from . import knn as oknn


def link_graph(embs, threshold, max_links, chunk=512):
    """-> list of neighbour lists (python ints)."""
    E = np.asarray(embs, np.float32)
    N = E.shape[0]
    graph = []
    for c0 in range(0, N, chunk):
        s = oknn.exact_scores(E[c0:c0 + chunk], E)
        for r, row in enumerate(s):
            i = c0 + r
            row = row.copy()
            row[i] = -1.0
            cand = np.nonzero(row >= threshold)[0]
            order = np.lexsort((cand, -row[cand]))[:max_links]
            graph.append([int(j) for j in cand[order]])
    return graph


def walk_retrieve(embs, graph, q, K=5, seed_size=5, max_steps=100, candidate_multiplier=10, seed=None):
    """Greedy graph walk of retrieval.py:187-244 -> (indices, scores)."""
    embs = np.asarray(embs, np.float32)
    q = np.asarray(q, np.float32).reshape(-1)
    N = embs.shape[0]
    np.random.seed(seed)
    seeds = np.random.choice(N, size=min(seed_size, N), replace=False).tolist()
    visited = set(seeds)
    q_norm = np.linalg.norm(q) + 1e-6

    def sim(i):
        e = embs[i]
        return float(e @ q / (np.linalg.norm(e) * q_norm + 1e-12))
    heap = []
    for i in seeds:
        heapq.heappush(heap, (-sim(i), i))
    R = max(candidate_multiplier * K, seed_size)
    steps = 0
    while steps < max_steps and heap:
        _, best = heapq.heappop(heap)
        improved = False
        for nbr in graph[best]:
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
    return [i for _, i in top], [s for s, _ in top]


def label_sets(labels01, names):
    """Per record: the set of label column names whose value int()s to 1 (reranker.py:161-179)."""
    out = []
    for row in np.asarray(labels01):
        out.append({n for n, v in zip(names, row) if int(v) == 1})
    return out


def record_kg_vectors(ids, lsets, node2id, node_emb, attn=None):
    """Reranker._load_kg normalisation (reranker.py:119-120) + get_record_kg_vec (:181-220)."""
    ne = np.asarray(node_emb, np.float32)
    ne = ne / (np.linalg.norm(ne, axis=1, keepdims=True) + 1e-12)
    out = np.zeros((len(ids), ne.shape[1]), np.float64)
    for i, rid in enumerate(ids):
        for key in (f"report:{rid}", str(rid)):
            if key in node2id:
                out[i] = ne[node2id[key]]
                break
        else:
            vecs = []
            for lab in sorted(lsets[i]):
                for ck in (f"label:{lab}", lab, lab.lower(), lab.replace(" ", "_")):
                    if ck in node2id:
                        vecs.append(ne[node2id[ck]])
                        break
            if vecs:
                L = np.stack(vecs).astype(np.float64)
                if attn is None:
                    out[i] = L.mean(0)
                else:  # LabelAttention (KnowledgeGraph/label_attention.py:19-27)
                    w1, b1, w2, b2 = attn
                    s = np.tanh(L @ w1.T + b1) @ w2.T + b2
                    s = np.exp(s[:, 0] - s[:, 0].max())
                    out[i] = (s / s.sum()) @ L
    return out


def _cos(a, b):
    na, nb = np.linalg.norm(a), np.linalg.norm(b)
    if na == 0 or nb == 0:
        return 0.0
    return float(np.dot(a, b) / (na * nb))


def _jac(a, b):
    if not a and not b:
        return 0.0
    u = len(a | b)
    return 0.0 if u == 0 else len(a & b) / u


def _minmax(x):
    x = np.asarray(x, np.float64)
    if x.size == 0:
        return x
    lo, hi = np.nanmin(x), np.nanmax(x)
    return np.zeros_like(x) if hi - lo == 0 else (x - lo) / (hi - lo)


def rerank(q_emb, cand_embs, q_lset, cand_lsets, q_kg, cand_kg, alpha=0.6, beta=0.25, gamma=0.15, topk=None):
    """-> (order (positions into the candidate list), final, emb_n, lab_n, kg_n) per reranker.py:298-333."""
    q_emb = np.asarray(q_emb, np.float64)
    emb = [_cos(q_emb, np.asarray(c, np.float64)) for c in cand_embs]
    lab = [_jac(q_lset, c) for c in cand_lsets]
    kg = [_cos(q_kg, c) for c in cand_kg]
    e, l, k = _minmax(emb), _minmax(lab), _minmax(kg)
    final = alpha * e + beta * l + gamma * k
    n = len(final)
    order = sorted(range(n), key=lambda i: (-final[i], -i))   # stable ascending argsort, reversed
    if topk:
        order = order[:topk]
    return order, final[order], e[order], l[order], k[order]
