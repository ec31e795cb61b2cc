"""x3 BERT tower (B = 256, L = 128): the residual adds in the O-proj / FFN2 split-GEMM epilogues vs in the
LayerNorm passes (BertTowerX3.res_in_gemm), interleaved on one box: ms per tower call and bitwise equality of
the outputs.  Diagnostic only: python tools/x3_res_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.towers import BERT_BASE, init_bert_state  # noqa: E402
from mmr_amd.towers_x3 import BertTowerX3  # noqa: E402

dev = torch.device("cuda:0")
B = 256
ids, mask = (torch.from_numpy(a).to(dev) for a in synthetic.reports(B, 128, 72))
tw = BertTowerX3(init_bert_state(BERT_BASE, 2710), BERT_BASE, dev)


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


outs, res = {}, {True: [], False: []}
for rep in range(3):
    for rg in (False, True):
        tw.res_in_gemm = rg
        res[rg].append(timeit(lambda: tw.forward(ids, mask)))
        outs[rg] = tw.forward(ids, mask).clone()
torch.cuda.synchronize()
print("residual in the LayerNorm:", " ".join(f"{v:.3f}" for v in res[False]), "ms | in the GEMM epilogue:",
      " ".join(f"{v:.3f}" for v in res[True]), "ms   bitwise equal:", bool(torch.equal(outs[True], outs[False])))
