"""ORACLE — test infrastructure only (CPU restatement of the reference's hot path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker / the timed CPU baseline, never as the product path.

Pinned by tests/golden/* (generated from the reference itself by tests/golden/make_golden.py):
  knn.py     sklearn cosine_similarity + np.argsort[::-1] (retrieval_overlap.py:84-90) and the
             exact f64 form the GPU path implements.
  towers.py  timm Swin-v1 forward_features + HF BertModel + the reference heads (fusion.py:255-327,
             model.py:330-489, MultiHeadMLP model.py:61-75), plain torch fp32 on CPU.
"""
