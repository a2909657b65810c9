"""ctypes binding of libtmae.so (include/tmae.h).

The library is the product: if it is missing or fails to load, every op raises — there is no
PyTorch or CPU fallback anywhere on the hot path.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libtmae.so")

TMAE_F32, TMAE_BF16 = 0, 1
ACT_NONE, ACT_GELU = 0, 1

P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


LL = ctypes.c_longlong


class ConvArgs(ctypes.Structure):
    """mirror of tmae_conv_args (include/tmae.h)"""
    _fields_ = [
        ("x1", P), ("c1", I), ("ld1", I), ("x1_s1", LL), ("x1_s2", LL),
        ("x2", P), ("c2", I), ("ld2", I), ("x2_s1", LL), ("x2_s2", LL),
        ("n", I), ("H", I), ("W", I), ("stride", I),
        ("w", P), ("w_s1", LL), ("w_s2", LL),
        ("bias", P), ("b_s1", LL), ("b_s2", LL),
        ("cout", I), ("act", I), ("pixel_shuffle", I),
        ("y", P), ("y_f32", I), ("ldy", I), ("y_s1", LL), ("y_s2", LL),
        ("y32", P), ("ld32", I), ("y32_s1", LL), ("y32_s2", LL),
        ("addend", P), ("ld_add", I), ("a_s1", LL), ("a_s2", LL),
        ("lrp_src", P), ("ld_src", I), ("src_s1", LL), ("src_s2", LL),
        ("y2", P), ("ldy2", I), ("y2_s1", LL), ("y2_s2", LL),
        ("nb1", I), ("nb2", I),
    ]


class EBParams(ctypes.Structure):
    _fields_ = [("matrix", ctypes.c_void_p * 5), ("bias", ctypes.c_void_p * 5), ("factor", ctypes.c_void_p * 4),
                ("quantiles", ctypes.c_void_p)]


# name -> argtypes (all return int status except where noted)
SIGNATURES = {
    "tmae_abi_version": [],
    "tmae_ids_shuffle": [P, P, P, I, I, I, I, P],
    "tmae_layernorm_fwd": [P, P, P, P, I, I, I, I, I, F, I, P],
    "tmae_linear_fwd": [P, I, I, I, I, I, P, P, P, I, I, P, I, I, I, I, I, I, P],
    "tmae_linear_residual_fwd": [P, I, P, P, P, I, I, I, I, I, P],
    "tmae_patch_embed_fwd": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "tmae_cls_rows": [P, P, P, I, I, I, P],
    "tmae_mha_fwd": [P, P, I, I, I, I, F, I, P],
    "tmae_decoder_embed_fwd": [P, I, P, P, P, P, P, I, I, I, I, I, I, P],
    "tmae_mask_rows": [P, P, P, P, I, I, I, I, P],
    "tmae_decoder_pred_fwd": [P, P, P, P, I, I, I, I, I, I, I, I, P],
    "tmae_conv3x3": [ctypes.POINTER(ConvArgs), I, P],
    "tmae_gc_slices_fwd": [P, I, I, P, P, LL, I, P, P, I, P, I, I, P, I, I, I, I, I, P],
    "tmae_eb_likelihood_fwd": [P, ctypes.POINTER(EBParams), P, P, P, I, P, I, I, I, P],
    "tmae_eb_aux_loss": [ctypes.POINTER(EBParams), P, P, P, I, P],
    "tmae_gc_likelihood_fwd": [P, P, P, P, P, P, I, F, P],
    "tmae_nhwc_to_nchw": [P, I, P, I, I, I, P],
    "tmae_bpp_sum": [P, LL, P, LL, P, P, ctypes.c_double, P],
    "tmae_gemm_plan": [I, I, I, I, I, ctypes.c_char_p, I],
    "tmae_mae_masking": [P, P, P, P, I, I, I, P],
    "tmae_mae_loss": [P, P, P, I, I, I, I, I, I, I, P, P, P],
    "tmae_gc_slices_code": [P, I, I, P, P, LL, I, P, I, P, I, I, P, I, I, I, I, I, P, P, P, I, P],
    "tmae_gc_indexes": [P, LL, I, I, I, I, I, P, I, F, P, P],
    "tmae_gc_dequantize": [P, P, LL, I, I, I, I, I, I, P, I, I, P, I, P],
    "tmae_gc_pmf": [P, P, I, I, P, P, P],
    "tmae_eb_pmf": [ctypes.POINTER(EBParams), P, P, I, I, P, P, P],
    "tmae_eb_symbols": [P, ctypes.POINTER(EBParams), P, I, I, I, P, P],
    "tmae_eb_dequantize": [P, ctypes.POINTER(EBParams), P, I, I, I, P, I, P],
    "tmae_invert_permutation": [P, P, I, I, P],
    "tmae_pmf_to_quantized_cdf": [P, I, I, P],
    "tmae_rans_encoder_create": [ctypes.POINTER(ctypes.c_void_p)],
    "tmae_rans_encode_with_indexes": [P, P, P, LL, P, I, P, P, I],
    "tmae_rans_encoder_flush": [P, ctypes.POINTER(ctypes.c_longlong)],
    "tmae_rans_encoder_take": [P, P, LL],
    "tmae_rans_encoder_destroy": [P],
    "tmae_rans_decoder_create": [P, LL, ctypes.POINTER(ctypes.c_void_p)],
    "tmae_rans_decode_with_indexes": [P, P, LL, P, I, P, P, I, P],
    "tmae_rans_decoder_destroy": [P],
}

_lib = None


class TmaeError(RuntimeError):
    pass


def load():
    """Load libtmae.so (raises if it has not been built — run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TmaeError(f"{LIB_PATH} is missing: build it with `python __graft_entry__.py` or build.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        lib.tmae_last_error_string.argtypes = []
        lib.tmae_last_error_string.restype = ctypes.c_char_p
        _lib = lib
    return _lib


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.tmae_last_error_string().decode(errors="replace")
        if rc == 1:
            raise ValueError(f"{name}: {msg}")
        raise TmaeError(f"{name} failed (status {rc}): {msg}")
    return rc
