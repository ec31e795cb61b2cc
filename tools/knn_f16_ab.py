"""Native fp16 index search time (the p8 scan's raw-row 1/|g| path) for whichever libmmr MMR_LIBMMR selects:
1M x 1024 fp16 gallery, Q = 2048, K = 10 (cfg5) and 100k x 768 fp16, Q = 256 (HIP events, min of 3 x 10).
Run once per library, interleaved, for a same-box A/B.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.retrieval import GalleryIndex  # noqa: E402


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("MMR_LIBMMR", "libmmr.so"))
for N, D, Q in ((1_000_000, 1024, 2048), (100_000, 768, 256)):
    G16 = synthetic.gauss_gallery(N, D, synthetic.SEED + 5).astype(np.float16)
    ix = GalleryIndex(G16)
    q = torch.from_numpy(synthetic.gauss_gallery(Q, D, synthetic.SEED + 6)).cuda()
    t = min(timeit(lambda: ix.search(q, 10)) for _ in range(3))
    i, _, s64 = ix.search(q, 10, want_f64=True)
    torch.cuda.synchronize()
    print(f"{tag:16s} N={N} D={D} Q={Q}: {t:8.1f} us  checksum {int(i.sum())} {float(s64.sum()):.12f}", flush=True)
    ix.close()
    del G16
