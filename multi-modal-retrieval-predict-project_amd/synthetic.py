"""Synthetic inputs of the reference's shapes; no network, no datasets.

* images: one grey channel u ~ U[0,1) replicated x3 (DataHandler/tensorDICOM.py:150), normalised
  with the eval-path mean/std 0.5/0.25 (Evaluate/retrieval_eval.py:105-111).  u is quantised to
  k/256 so every pixel (k/64 - 2) is exact in f32 and bf16.
* reports: (B, L) int64 ids, length L_i ~ U[16, L], [CLS]=101 at 0, [SEP]=102 at L_i-1, body ids
  ~ U[999, vocab), PAD 0 after; mask = 1[pos < L_i]  (DataHandler/ChestXRDataset.py:10-33,
  padding='max_length').
* galleries: N(0,1) rows (throughput) or a 43-label multi-hot gallery (1-3 labels per row, row =
  sum of label centres + 0.6 N(0,1)) for P@10 / R@10, relevance = shares >= 1 label
  (Helpers/contructGT.py:69-81).
"""
import numpy as np

SEED = 2709  # configs/config.yaml:6
NUM_LABELS = 43  # LabelData/labeledData.py: disease 19 + finding 19 + symptom 4 + normal 1


def gauss_gallery(n, d, seed=SEED):
    return np.random.default_rng(seed).standard_normal((n, d), dtype=np.float32)


def label_centres(d, seed=SEED):
    return np.random.default_rng(seed + 1000003).standard_normal((NUM_LABELS, d), dtype=np.float32)


def labelled_gallery(n, d, seed=SEED, noise=0.6, centre_seed=SEED):
    """(rows f32 (n,d), labels uint8 (n,43)). Label centres are shared across calls."""
    rng = np.random.default_rng(seed)
    c = label_centres(d, centre_seed)
    labels = np.zeros((n, NUM_LABELS), np.uint8)
    nl = rng.integers(1, 4, size=n)
    for i in range(n):
        labels[i, rng.choice(NUM_LABELS, size=int(nl[i]), replace=False)] = 1
    x = labels.astype(np.float32) @ c + noise * rng.standard_normal((n, d), dtype=np.float32)
    return x.astype(np.float32), labels


DLS_N, DLS_D, DLS_Q = 1200, 128, 24
DLS_ZERO, DLS_DUP = [5, 77], (10, 20)      # zero rows; row DUP[1] := row DUP[0] (exact ties)
LABEL_NAMES = [f"Finding {i}" if i % 5 == 0 else f"L{i}" for i in range(NUM_LABELS)]  # some with spaces


def dls_gallery():
    """Labelled gallery of the DLS / reranker fixture (tests/golden/dls_rerank.npz): two zero rows,
    one exact duplicate pair, one record with no labels."""
    G, gl = labelled_gallery(DLS_N, DLS_D, SEED + 11)
    G[DLS_ZERO] = 0.0
    G[DLS_DUP[1]] = G[DLS_DUP[0]]
    gl[DLS_DUP[1]] = gl[DLS_DUP[0]]
    gl[DLS_ZERO[0]] = 0
    return G, gl


def kg_node2id(n_records=DLS_N):
    """Synthetic KG node table: report nodes for every 3rd record ("report:r<i>"), label nodes under
    the key forms the reference's Reranker.get_record_kg_vec tries (reranker.py:190-207), one label
    without a node."""
    node2id = {}
    for i in range(0, n_records, 3):
        node2id[f"report:r{i}"] = len(node2id)
    for j, name in enumerate(LABEL_NAMES):
        if j == 42:
            continue
        key = [f"label:{name}", name, name.lower(), name.replace(" ", "_")][j % 4]
        node2id[key] = len(node2id)
    return node2id


def image_u8(b, seed=SEED, hw=224):
    return np.random.default_rng(seed).integers(0, 256, size=(b, hw, hw), dtype=np.uint8)


def image_from_u8(u8):
    """(B,H,W) uint8 -> (B,3,H,W) f32, ((k/256) - 0.5) / 0.25 replicated over 3 channels."""
    x = (u8.astype(np.float32) / 256.0 - 0.5) / 0.25
    return np.ascontiguousarray(np.repeat(x[:, None], 3, axis=1))


def reports(b, l=128, seed=SEED, vocab=28996, min_len=16):
    rng = np.random.default_rng(seed)
    ids = np.zeros((b, l), np.int64)
    mask = np.zeros((b, l), np.int64)
    lens = rng.integers(min(min_len, l), l + 1, size=b)
    for i in range(b):
        n = int(lens[i])
        ids[i, 0] = 101
        ids[i, 1:n - 1] = rng.integers(min(999, vocab - 1), vocab, size=max(n - 2, 0))
        ids[i, n - 1] = 102
        mask[i, :n] = 1
    return ids, mask


def labels_to_bits(labels):
    """(n,43) multi-hot -> (n,) uint64 bitsets (relevance = popcount(a & b) > 0)."""
    w = (np.uint64(1) << np.arange(NUM_LABELS, dtype=np.uint64))
    return (labels.astype(np.uint64) * w).sum(axis=1).astype(np.uint64)


def f32_to_bf16_bits(x):
    """Round-to-nearest-even f32 -> bf16 bit pattern (uint16); inputs here are finite."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return r.astype(np.uint16)


def bf16_bits_to_f32(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)
