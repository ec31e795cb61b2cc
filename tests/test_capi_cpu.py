"""CPU: libmmr.so (the drop-in C ABI) loads and exports every symbol include/mmr.h declares; the
Python binding declares a signature for each; error reporting works without a GPU."""
import ctypes
import os
import subprocess

import pytest

import __graft_entry__ as ge

LIB = os.path.join(ge.PKG, "libmmr.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-j8"], cwd=os.path.join(ge.PKG, "csrc"), check=True)
    import torch  # noqa: F401  (same HIP runtime as the product path)
    return ctypes.CDLL(LIB)


def test_exports_every_header_symbol(lib):
    syms = ge.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from mmr_amd import _lib
    assert sorted(_lib.SIGNATURES) == ge.header_symbols()


def test_errors_without_gpu(lib):
    from mmr_amd import _lib
    L = _lib.lib()
    assert L.mmr_version() >= 1 and L.mmr_max_k() >= 50
    # invalid arguments are rejected before touching the device
    st = L.mmr_index_search(None, None, 1, 10, None, None, None, None, None)
    assert st == 1 and b"NULL" in L.mmr_last_error()
    st = L.mmr_linear_bf16(None, None, None, None, None, 4, 8, 8, 0, None)
    assert st == 1
    st = L.mmr_bert_attention(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 100, 12, 60, None)
    assert st == 1 and b"head_dim 60" in L.mmr_last_error()
    assert L.mmr_linear_bf16_variant(32768, 3072, 768, 1, 1, 0) == -1  # nothing tuned in this process
