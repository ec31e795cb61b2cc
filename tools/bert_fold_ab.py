"""BERT-base tower (random init) at the cfg2 shape (B = 256 x 128 tokens), the LayerNorm-folded layer stack
(O-proj / FFN2 with the LNM = 2 + statistics epilogue, QKV / FFN1 folding the coefficients) against the
unfolded one (plain residual epilogues + the add-LayerNorm passes), interleaved in one process: tower time
per forward (HIP events, min of 3 x 5).  usage: python tools/bert_fold_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd.towers import BERT_BASE, BertTower, init_bert_state  # noqa: E402

B, L = 256, 128
bt = BertTower(init_bert_state(BERT_BASE, seed=3), BERT_BASE, "cuda")
ids = torch.randint(0, BERT_BASE["vocab_size"], (B, L), generator=torch.Generator().manual_seed(1)).cuda()
mask = torch.ones(B, L, dtype=torch.int64).cuda()


def timeit(it=5):
    bt.forward(ids, mask)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        bt.forward(ids, mask)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for rnd in range(2):
    for fold in (True, False):
        bt.ln_fold = fold
        t = min(timeit() for _ in range(3))
        print(f"round {rnd} ln_fold={fold}: {t:.3f} ms per BERT-base forward (B={B}, L={L})", flush=True)
