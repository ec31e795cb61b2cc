"""ctypes binding of libmmr.so (include/mmr.h).  The product path has no CPU fallback: if the
library is missing or no GPU is visible, the first call raises.

torch is imported first on purpose: torch's wheel ships its own libamdhip64.so.7, and loading it
before libmmr.so makes both share ONE HIP runtime (same soname), so torch device pointers and
streams are valid inside the library.
"""
import ctypes
import os

import torch  # noqa: F401  (see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMR_LIBMMR", os.path.join(_HERE, "libmmr.so"))  # override: diagnostic builds

c_i32, c_i64, c_f32, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p

# name -> argtypes (restype is always int status unless listed in _RESTYPES)
SIGNATURES = {
    "mmr_last_error": [],
    "mmr_version": [],
    "mmr_max_k": [],
    "mmr_index_create": [c_vp, c_i64, c_i32, c_i32, ctypes.c_int, c_i64, ctypes.c_int, ctypes.POINTER(c_vp)],
    "mmr_index_destroy": [c_vp],
    "mmr_index_info": [c_vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i32), ctypes.POINTER(c_i64)],
    "mmr_index_reserve": [c_vp, c_i64],
    "mmr_index_device_bytes": [c_vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)],
    "mmr_index_set_mode": [c_vp, c_i32],
    "mmr_index_search": [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "mmr_index_link_graph": [c_vp, ctypes.c_double, c_i32, c_i64, c_i64, c_vp, c_vp, c_vp],
    "mmr_index_rerank": [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, ctypes.c_double,
                         ctypes.c_double, ctypes.c_double, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "mmr_merge_topk": [c_vp, c_vp, c_i32, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp],
    "mmr_merge_topk_payload": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp,
                               c_vp, c_vp],
    "mmr_merge_topk_packed": [c_vp, c_i32, c_i32, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "mmr_index_rerank_components": [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp],
    "mmr_rerank_mix": [c_vp, c_vp, c_i64, c_i32, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_i32, c_vp, c_vp,
                       c_vp, c_vp, c_vp, c_vp],
    "mmr_linear_bf16": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp],
    "mmr_linear_bf16_variant": [c_i64, c_i32, c_i32, c_i32, c_i32, c_i32],
    "mmr_linear_bf16_n_variants": [],
    "mmr_linear_bf16_ln_parts": [c_i64, c_i32, c_i32],
    "mmr_linear_bf16_ln": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                           c_vp],
    "mmr_ln_row_coef": [c_vp, c_i64, c_i32, c_i32, c_f32, c_vp, c_vp],
    "mmr_pin_variant": [c_i32, c_i32],
    "mmr_linear_rw_parts": [c_i32, c_i32],
    "mmr_linear_rw_pack": [c_vp, c_i32, c_i32, c_vp, c_vp],
    "mmr_linear_rw": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp],
    "mmr_linear_x3": [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                      c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_quantize_mxfp8": [c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp],
    "mmr_linear_mxfp8": [c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp],
    "mmr_linear_mxfp8_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp],
    "mmr_layernorm_bf16": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_add_layernorm_bf16": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_layernorm_bf16_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_layernorm_bf16_q8p": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_vp],
    "mmr_scaled_add_layernorm_bf16": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_scaled_add_layernorm_bf16_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_bert_embed": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_bert_embed_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_bert_attention": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_bert_attention_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_swin_window_attention": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_swin_window_attention_q8": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_swin_attn_bias": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_swin_attn_block_pack_bytes": [c_i32],
    "mmr_swin_attn_block_pack": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp],
    "mmr_swin_attn_block": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_swin_mlp_pack_elems": [c_i32],
    "mmr_swin_mlp_pack": [c_vp, c_vp, c_vp, c_i32, c_vp],
    "mmr_swin_mlp": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_patch_im2col": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_patch_merge_ln": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_patch_merge_ln_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_swin_head": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_mean_tokens": [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "mmr_proj_head": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_linear_f32": [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_mha": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32,
                c_vp],
    "mmr_mha_q8": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32,
                   c_i32, c_f32, c_vp],
    "mmr_add_pos_bf16": [c_vp, c_i32, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp],
    "mmr_add_pos_bf16_q8": [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp],
    "mmr_ln_rows_split": [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_ln_rows": [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_i32, c_f32,
                    c_i32, c_i32, c_i64, c_vp],
    "mmr_linear_f32_batched": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                               c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_assemble_seq": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "mmr_assemble_seq_q8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "mmr_rows_to_f32": [c_vp, c_i64, c_vp, c_i32, c_i32, c_vp],
    "mmr_x3_linear": [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_p8_kpad": [c_i32],
    "mmr_x3_p8_npad": [c_i32],
    "mmr_x3_split_rows": [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp],
    "mmr_x3_linear_p8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_attention": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32,
                         c_i32, c_f32, c_vp],
    "mmr_x3_attention_xs": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32,
                            c_f32, c_vp],
    "mmr_x3_swin_window_attention_xs": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_swin_window_attention": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_patch_im2col": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_patch_merge_ln": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_x3_patch_merge_ln_xs": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_x3_bert_embed": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_x3_add_pos": [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp],
    "mmr_x3_add_pos_split": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp],
    "mmr_x3_swin_mlp_pack_elems": [c_i32],
    "mmr_x3_rowlin_pack_elems": [c_i32, c_i32],
    "mmr_x3_rowlin_pack": [c_vp, c_vp, c_i32, c_i32, c_vp],
    "mmr_x3_rowlin": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_vp],
    "mmr_x3_swin_mlp_pack": [c_vp, c_vp, c_vp, c_i32, c_vp],
    "mmr_x3_swin_attn_block_pack_bytes": [c_i32],
    "mmr_x3_swin_attn_block_pack": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp],
    "mmr_x3_swin_attn_block": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp],
    "mmr_x3_swin_mlp": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "mmr_x3_assemble_seq": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_assemble_seq_split": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_mean_rows": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "mmr_x3_gather_rows": [c_vp, c_i64, c_vp, c_i32, c_i32, c_vp],
    "mmr_x3_patch_embed_pack_elems": [],
    "mmr_x3_patch_embed_pack": [c_vp, c_vp, c_vp],
    "mmr_x3_patch_embed_ln": [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp],
    "mmr_patch_embed_ln_bf16": [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp],
}
_RESTYPES = {"mmr_last_error": ctypes.c_char_p, "mmr_version": ctypes.c_int, "mmr_max_k": ctypes.c_int,
             "mmr_linear_bf16_variant": ctypes.c_int32, "mmr_linear_bf16_n_variants": ctypes.c_int32,
             "mmr_linear_bf16_ln_parts": ctypes.c_int32,
             "mmr_linear_rw_parts": ctypes.c_int32,
             "mmr_swin_mlp_pack_elems": ctypes.c_int64, "mmr_swin_attn_block_pack_bytes": ctypes.c_int64,
             "mmr_x3_swin_mlp_pack_elems": ctypes.c_int64, "mmr_x3_rowlin_pack_elems": ctypes.c_int64,
             "mmr_x3_patch_embed_pack_elems": ctypes.c_int64,
             "mmr_x3_swin_attn_block_pack_bytes": ctypes.c_int64}

_lib = None


class MMRError(RuntimeError):
    pass


def lib():
    """Load libmmr.so once; raise (never fall back) if it is absent or incomplete."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MMRError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            if not hasattr(L, name):  # a call to a missing export raises AttributeError
                continue
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
    return _lib


def check(status, what):
    if status != 0:
        msg = lib().mmr_last_error().decode(errors="replace")
        raise MMRError(f"{what} failed (status {status}): {msg}")


def require_gpu(t=None):
    if not torch.cuda.is_available():
        raise MMRError("libmmr needs a ROCm GPU (torch.cuda.is_available() is False); no CPU fallback")
    if t is not None and not t.is_cuda:
        raise MMRError("libmmr ops take device tensors")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
