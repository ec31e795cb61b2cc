"""Cost of the sharded (RCCL) search path at one rank vs the direct index search, cfg2 kNN shape
(256 queries x 100k x 768 fp16 index, top-10): host time per call (perf_counter, no sync) and GPU time
(events around 20 back-to-back calls behind a device spin).  Diagnostic only: python tools/rccl_overhead.py"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mmr_amd import synthetic  # noqa: E402
from mmr_amd.parallel import ShardedIndex  # noqa: E402
from mmr_amd.retrieval import GalleryIndex  # noqa: E402

with socket.socket() as so:
    so.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]), RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
dev = torch.device("cuda:0")
n, d, B, K = 100_000, 768, 256, 10
ix = GalleryIndex(synthetic.gauss_gallery(n, d, synthetic.SEED), device=0, mode="f16")
st = torch.zeros((), dtype=torch.int32, device=dev)


def local(q, k):
    i, _, s64, s = ix.search(q, k, want_f64=True, want_status=True)
    return i, s64, s


sh = ShardedIndex(None, n, 0, local_search=local, status_out=st)
q = torch.from_numpy(synthetic.gauss_gallery(B, d, 9)).to(dev)
calls = {"direct": lambda: ix.search(q, K, want_f64=True, want_status=True),
         "sharded (RCCL)": lambda: sh.search(q, K),
         "pack+merge only": lambda: __import__("mmr_amd.parallel", fromlist=["x"]).merge_gathered(
             __import__("mmr_amd.parallel", fromlist=["x"]).pack_lists(*local(q, K)[:2]).unsqueeze(0), 0, B, K)}
for name, fn in calls.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    host = (time.perf_counter() - t0) / 20 * 1e6
    torch.cuda.synchronize()
    torch.cuda._sleep(50_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:18s} host {host:8.1f} us/call   GPU {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us/call", flush=True)
dist.destroy_process_group()
