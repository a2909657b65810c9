"""ctypes binding of libtmae.so (include/tmae.h).

The library is the product: if it is missing or fails to load, every op raises — there is no
PyTorch or CPU fallback anywhere on the hot path.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TMAE_LIB") or os.path.join(PKG_DIR, "lib", "libtmae.so")  # TMAE_LIB: A/B builds

TMAE_F32, TMAE_BF16 = 0, 1
ACT_NONE, ACT_GELU, ACT_RELU = 0, 1, 2

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
        ("pre", P), ("ldp", I), ("pre_s1", LL), ("pre_s2", LL),
    ]


class WgradArgs(ctypes.Structure):
    """mirror of tmae_wgrad_args"""
    _fields_ = [
        ("a", P), ("lda", I), ("a_G", I), ("a_Gs", I), ("a_off", I),
        ("b", P), ("ldb", I), ("b_G", I), ("b_Gs", I), ("b_off", I),
        ("b_conv", I), ("b2", P), ("b_c1", I), ("b_ld2", I), ("b_H", I), ("b_W", I), ("b_stride", I), ("b_Cin", I),
        ("M", I), ("N", I), ("K", I),
        ("work", P), ("work_elems", LL),
        ("out", P), ("o_base", LL), ("o_sm", LL), ("o_sc", LL), ("o_st", LL), ("o_cp", I), ("accumulate", I),
        ("bias_out", P), ("bias_accumulate", I),
        ("slot_div", I),
        ("nb", I), ("s_a", LL), ("s_b", LL), ("s_b2", LL), ("s_out", LL), ("s_bias", LL),
    ]


class ConvDgradArgs(ctypes.Structure):
    """mirror of tmae_conv_dgrad_args"""
    _fields_ = [
        ("dy", P), ("ldy", I),
        ("n", I), ("H", I), ("W", I), ("stride", I), ("cout", I), ("cin", I),
        ("wd", P),
        ("out", P), ("out_f32", I), ("ldo", I), ("pre", P), ("ldp", I),
        ("acc", P * 3), ("ld_acc", I * 3), ("lim", I * 3),
        ("nb", I), ("s_dy", LL), ("s_wd", LL), ("s_out", LL), ("s_pre", LL),
    ]


LSTK_MAXL = 5


class LicStackArgs(ctypes.Structure):
    """mirror of tmae_lic_stack_args"""
    _fields_ = [
        ("n", I), ("G", I), ("nb1", I), ("nb2", I), ("nlayers", I),
        ("x1", P), ("c1", I), ("ld1", I), ("x1_s", LL * 2),
        ("x2", P), ("c2", I), ("ld2", I), ("x2_s", LL * 2),
        ("w", P * LSTK_MAXL), ("w_s", (LL * 2) * LSTK_MAXL),
        ("bias", P * LSTK_MAXL), ("b_s", (LL * 2) * LSTK_MAXL),
        ("cout", I * LSTK_MAXL),
        ("addend", P), ("ld_add", I), ("a_s", LL * 2),
        ("y", P), ("y_f32", I), ("ldy", I), ("y_s", LL * 2),
        ("lrp_src", P), ("ld_src", I), ("src_s", LL * 2),
        ("y2", P), ("ldy2", I), ("y2_s", LL * 2),
        ("flags", I),
        ("cn", I), ("cw", P * LSTK_MAXL), ("cb", P * LSTK_MAXL), ("ccout", I * LSTK_MAXL),
        ("cx1", P), ("cc1", I), ("cld1", I),
        ("yv", P), ("ldyv", I),
        ("cadd", P), ("cld_add", I),
        ("csrc", P), ("cld_src", I),
        ("cy", P), ("cldy", I),
        ("cy2", P), ("cldy2", I),
        ("cs_x1", LL), ("cs_yv", LL), ("cs_src", LL), ("cs_add", LL), ("cs_y", LL), ("cs_y2", LL),
        ("cs_w", LL * LSTK_MAXL), ("cs_b", LL * LSTK_MAXL),
        ("sv_pre", P * LSTK_MAXL), ("sv_act", P * LSTK_MAXL), ("sv_s", (LL * 2) * LSTK_MAXL),
        ("sv_t", P), ("sv_t_s", LL * 2),
        ("csv_pre", P * LSTK_MAXL), ("csv_act", P * LSTK_MAXL), ("cs_sv", LL * LSTK_MAXL),
        ("csv_t", P), ("cs_t", LL),
        ("racc", P * 3), ("rld", I * 3), ("rlim", I * 3), ("rs", LL * 3),
    ]


class LicLatentArgs(ctypes.Structure):
    """mirror of tmae_lic_latent_args"""
    _fields_ = [
        ("n", I), ("G", I), ("cin", I), ("nb", I),
        ("x", P * 4), ("ldx", I),
        ("w", P), ("nfr", I), ("blk", LL),
        ("f_off", I * 4), ("f_lo", I), ("f_hi", I),
        ("y", P), ("ldy", I),
        ("y_s", LL * 4), ("bias", P * 4), ("act", I), ("y_bf16", I),
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
    "tmae_patch_embed_gathered": [P, P, P, P, P, P, I, I, I, I, I, I, P],
    "tmae_cls_rows": [P, P, P, I, I, I, P],
    "tmae_mha_fwd": [P, P, I, I, I, I, F, I, P],
    "tmae_qkv_attn_fwd": [P, P, P, P, I, I, I, I, F, I, P],
    "tmae_decoder_embed_fwd": [P, I, P, P, P, P, P, I, I, I, I, I, I, P],
    "tmae_mask_rows": [P, P, P, P, I, I, I, I, P],
    "tmae_decoder_pred_fwd": [P, P, P, P, I, I, I, I, I, I, I, I, P],
    "tmae_decoder_pred_cp_fwd": [P, P, P, P, I, I, I, I, I, I, I, I, P],
    "tmae_conv3x3": [ctypes.POINTER(ConvArgs), I, P],
    "tmae_lic_stack": [ctypes.POINTER(LicStackArgs), P],
    "tmae_lic_latent": [ctypes.POINTER(LicLatentArgs), P],
    "tmae_gc_slices_fwd": [P, I, I, P, P, LL, I, P, P, I, P, I, I, P, I, I, I, I, I, P],
    "tmae_eb_likelihood_fwd": [P, ctypes.POINTER(EBParams), P, P, P, I, P, I, I, I, P],
    "tmae_eb_aux_loss": [ctypes.POINTER(EBParams), P, P, P, I, P],
    "tmae_gc_likelihood_fwd": [P, P, P, P, P, P, I, F, P],
    "tmae_nhwc_to_nchw": [P, I, P, I, I, I, P],
    "tmae_crop_normalize_u8": [P, I, I, I, P, I, I, ctypes.POINTER(F), ctypes.POINTER(F), P, P],
    "tmae_bpp_sum": [P, LL, P, LL, P, P, ctypes.c_double, P],
    "tmae_gemm_plan": [I, I, I, I, I, ctypes.c_char_p, I],
    "tmae_mae_masking": [P, P, P, P, I, I, I, P],
    "tmae_mae_loss": [P, P, P, I, I, I, I, I, I, I, P, P, P],
    "tmae_mae_loss_bwd": [P, P, P, I, I, I, I, I, I, I, P, P, P, I, P],
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
    # Kodak eval harness: Huffman side info (host), metrics and the score-map producer (device)
    "tmae_huffman_build": [P, LL, P, P, P, I, ctypes.POINTER(I)],
    "tmae_huffman_encode": [P, LL, P, P, P, I, P, LL, ctypes.POINTER(LL)],
    "tmae_huffman_decode": [ctypes.c_char_p, LL, P, P, P, I, P, LL, ctypes.POINTER(LL)],
    "tmae_image_metrics": [P, P, I, I, I, I, P, LL, P, P],
    "tmae_image_scores": [P, I, I, I, I, I, P, LL, P, P],
    # VGG16 feature loss glue
    "tmae_vgg_prep": [P, I, I, I, I, I, P, I, P],
    "tmae_vgg_prep_bwd": [P, I, I, I, I, I, P, I, P],
    "tmae_maxpool2": [P, I, I, I, I, P, P, I, P],
    "tmae_maxpool2_bwd": [P, P, I, I, I, I, P, P, I, P],
    "tmae_relu_mask": [P, P, LL, I, P],
    "tmae_mse": [P, P, LL, P, P, I, I, P],
    "tmae_mse_bwd": [P, P, LL, P, P, I, P],
    # training
    "tmae_linear_fwd_pre": [P, I, I, I, I, I, P, P, P, I, I, P, I, I, I, I, I, I, P],
    "tmae_linear_residual_out": [P, I, P, P, P, P, I, I, I, I, I, P],
    "tmae_mha_fwd_lse": [P, P, P, I, I, I, I, F, I, P],
    "tmae_mha_bwd": [P, P, P, P, P, I, I, I, I, F, I, P],
    "tmae_patch_gather": [P, P, P, I, I, I, I, I, I, I, I, P],
    "tmae_wgrad": [ctypes.POINTER(WgradArgs), I, P],
    "tmae_dgrad_linear": [P, I, I, I, I, P, I, I, I, P, I, I, P, I, P, I, I, P],
    "tmae_conv_dgrad": [ctypes.POINTER(ConvDgradArgs), I, P],
    "tmae_relayout": [P, P, I, I, I, I, I, LL, LL, LL, LL, P],
    "tmae_relayout_multi": [P, I, LL, P],
    "tmae_colsum": [P, I, I, I, I, I, I, I, P, LL, P, I, P],
    "tmae_layernorm_bwd": [P, P, P, P, P, P, I, I, I, I, I, I, F, P, LL, P, P, P, I, P],
    "tmae_unshuffle_bwd": [P, I, I, P, I, P, I, I, I, I, I, P],
    "tmae_gelu_bwd": [P, I, P, P, LL, I, P],
    "tmae_lrp_bwd": [P, I, P, I, P, I, P, I, P, I, P, I, I, I, I, P],
    "tmae_copy2d": [P, I, P, I, I, I, I, P],
    "tmae_gc_bwd": [P, I, I, P, P, I, P, I, P, P, I, P, I, P, P, I, I, I, I, I, P],
    "tmae_eb_bwd": [ctypes.POINTER(EBParams), P, P, P, P, P, I, I, I, ctypes.POINTER(EBParams), I, P],
    "tmae_eb_aux_bwd": [ctypes.POINTER(EBParams), P, P, P, I, I, P],
    "tmae_bpp_bwd": [P, P, P, LL, ctypes.c_double, P],
    "tmae_patchify": [P, P, I, I, I, I, I, I, P],
    "tmae_decoder_embed_bwd_gather": [P, P, P, I, I, I, I, I, P, P, I, P],
    "tmae_add": [P, P, P, LL, P],
    "tmae_adam": [P, P, P, P, LL, F, F, F, F, F, I, P, P],
    "tmae_adam_multi": [P, I, LL, F, F, F, F, F, P, P],
    "tmae_grad_norm": [P, LL, P, F, P, P],
    "tmae_scale": [P, LL, P, P],
    "tmae_distortion_fwd": [P, P, I, I, I, P, P, P, P, P],
    "tmae_distortion_bwd": [P, P, I, I, I, P, P, P, P, P],
}

# entry points that return a value rather than a status
VALUE_FUNCS = {"tmae_wgrad_workspace": ([I, I, I, I], ctypes.c_longlong),
               "tmae_wgrad_workspace_nb": ([I, I, I, I, I, I], ctypes.c_longlong),
               "tmae_metrics_workspace": ([I, I, I, I], ctypes.c_longlong),
               "tmae_image_scores_workspace": ([I, I, I, I], ctypes.c_longlong),
               "tmae_qkv_attn_supported": ([I, I, I], ctypes.c_int)}

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
        for name, (args, res) in VALUE_FUNCS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        lib.tmae_last_error_string.argtypes = []
        lib.tmae_last_error_string.restype = ctypes.c_char_p
        _lib = lib
    return _lib


def value(name: str, *args):
    """call an entry point of VALUE_FUNCS and return its result"""
    return getattr(load(), name)(*args)


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.tmae_last_error_string().decode(errors="replace")
        if rc == 1:
            raise ValueError(f"{name}: {msg}")
        raise TmaeError(f"{name} failed (status {rc}): {msg}")
    return rc
