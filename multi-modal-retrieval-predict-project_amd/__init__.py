"""mmr_amd — MI355X-native joint-embedding extraction + brute-force cosine kNN retrieval.

Drop-in for the reference's hot path:
  * `make_retrieval_engine(..., method="mi355x")` / `MI355XRetrievalEngine` mirror
    src/Retrieval/retrieval.py (RetrievalEngine ABC + factory) and run the batched-cosine top-K on
    the GPU through libmmr.so (hand-written gfx950 HIP kernels behind a C ABI, include/mmr.h);
    `method="dls"` / `DLSRetrievalEngine` builds the DLS link graph as a GPU self-join.
  * `Reranker` mirrors src/Retrieval/reranker.py on a fused device rerank kernel.
  * `Backbones` / `MultiModalRetrievalModel` mirror src/Model/fusion.py / model.py for the
    Swin-Tiny + ClinicalBERT towers, the projection / text / image heads and the multimodal fusion
    stack (model.py, mmr_amd.fusion).
  * `gallery.build_gallery` writes the reference's `.npy` + ids `.json` embedding galleries.
  * `metrics` mirrors src/Helpers/retrieval_metrics.py.
Import is cheap: the native library is loaded on first use and fails loudly if it is missing.
"""
from . import metrics, synthetic  # noqa: F401
from .rerank import Reranker  # noqa: F401
from .retrieval import DLSRetrievalEngine, MI355XRetrievalEngine, RetrievalEngine, make_retrieval_engine  # noqa: F401

__all__ = ["RetrievalEngine", "MI355XRetrievalEngine", "DLSRetrievalEngine", "Reranker", "make_retrieval_engine",
           "metrics", "synthetic"]
