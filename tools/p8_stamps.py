"""Per-tile time breakdown of the 8-phase GEMM from the diagnostic stamp build
(tools/ab/libmmr_stamps.so = libmmr built with -DMMR_P8_STAMPS; run with MMR_LIBMMR pointing at it):
per workgroup / wave / tile the shader clock at the tile start, the end of its K loop and the end of
its epilogue.  Prints medians over workgroups of: K loop, epilogue, gap to the next tile's start,
for waves 0 (m-group 0) and 4 (m-group 1), and the in-kernel clock.  Diagnostic only."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmr_amd  # noqa: E402,F401
from mmr_amd import _lib, ops  # noqa: E402

L = _lib.lib()
assert hasattr(L, "mmr_diag_p8_stamps"), "needs the stamp build (MMR_LIBMMR=tools/ab/libmmr_stamps.so)"
L.mmr_diag_p8_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]


def read():
    buf = np.zeros(1024 * 256, np.uint64)
    assert L.mmr_diag_p8_stamps(buf.ctypes.data, buf.size) == 0
    return buf.reshape(1024, 8, 8, 4).astype(np.int64)  # [wg][wave][tile][k]


def report(name, fn, nwg):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    fn()
    t1.record()
    torch.cuda.synchronize()
    st = read()[:nwg]
    print(f"{name}: {t0.elapsed_time(t1) * 1e3:.1f} us", flush=True)
    clk = []
    for w in (0, 4):
        s = st[:, w]
        kl = s[:, :, 1] - s[:, :, 0]
        ep = s[:, :, 2] - s[:, :, 1]
        gap = s[:, 1:, 0] - s[:, :-1, 2]
        v = (s[:, :, 0] > 0) & (s[:, :, 2] > 0)
        vg = v[:, 1:] & v[:, :-1]
        full = s[:, 6, 3] - s[:, 1, 3]
        cyc = s[:, 6, 0] - s[:, 1, 0]
        ok = (full > 0) & (cyc > 0)
        if ok.any():
            clk.append(np.median(cyc[ok] / (full[ok] * 10e-9)) / 1e9)
        print(f"  wave {w}: K loop median {np.median(kl[v]):7.0f} cyc  epilogue {np.median(ep[v]):6.0f}  "
              f"gap to next tile {np.median(gap[vg]):5.0f}  (tile 0: K loop {np.median(kl[:, 0]):7.0f})", flush=True)
    if clk:
        print(f"  in-kernel clock ~{np.mean(clk):.2f} GHz", flush=True)


for M, N, K, act in [(262144, 2304, 768, 0), (262144, 3072, 768, 1), (262144, 768, 3072, 0)]:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    report(f"bf16 M={M} N={N} K={K} act={act} (variant {L.mmr_linear_bf16_variant(M, N, K, act, 1, 0)})",
           lambda: ops.linear(x, w, b, act=act, out=y), 256)
    w8 = ops.quantize_mxfp8(w, layout=2 if (N % 256 == 0 and not act) else 1)
    x8 = ops.quantize_mxfp8(x, layout=0)
    report(f"fp8  M={M} N={N} K={K} act={act}", lambda: ops.linear_mxfp8(x8, w8, b, act=act, out=y), 256)
    if N % 256 == 0:
        w8b = ops.quantize_mxfp8(w, layout=2)
        report(f"fp8 q8-out M={M} N={N} K={K} act={act}", lambda: ops.linear_mxfp8_q8(x8, w8b, b, act=act), 256)
    del x, w, x8, w8, y
