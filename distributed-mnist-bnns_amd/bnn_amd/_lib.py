"""ctypes binding of libbnn.so (C ABI declared in include/bnn.h).

The library is the product: there is no CPU fallback.  Loading fails loudly when the .so is
missing, and every op raises when handed a non-ROCm tensor.
"""
import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so libbnn binds to the same one

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libbnn.so")

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int32
F32 = ctypes.c_float
U64 = ctypes.c_uint64

# name -> (restype, argtypes); must match include/bnn.h
SIGNATURES = {
    "bnn_version": (I32, []),
    "bnn_last_error": (ctypes.c_char_p, []),
    "bnn_sign_pack_i8": (I32, [P, I64, I64, I64, P, I64, P, I64, P]),
    "bnn_sign_pack_fp4": (I32, [P, I64, I64, I64, P, I64, P, I64, I32, P]),
    "bnn_sign_pack_fp4_out": (I32, [P, I64, I64, P, I64, P, I64, I32, P, P]),
    "bnn_sign_f32": (I32, [P, P, I64, P]),
    "bnn_sign_pack_bits": (I32, [P, I64, I64, I64, P, P, I64, P]),
    "bnn_quant_rows": (I32, [P, I64, I64, I64, P, I64, I64, P, P]),
    "bnn_quant_cols_workspace": (I64, [I64, I64]),
    "bnn_quant_cols_t": (I32, [P, I64, I64, I64, P, I64, I64, P, P, P, P]),
    "bnn_quant_cols_t_dsum": (I32, [P, I64, I64, I64, P, I64, I64, P, P, P, P, P]),
    "bnn_gemm_i8": (I32, [P, I64, I64, I32, P, I64, I64, I32, P, P, P, P, I64, I64, I64, I64, P]),
    "bnn_gemm_i8_affine": (I32, [P, I64, I64, I32, P, I64, I64, I32, P, P, P, P, P, ctypes.c_double, P, I64,
                                 I64, I64, I64, P]),
    "bnn_gemm_i8_bnstats_chunk": (I64, [I64, I64]),
    "bnn_gemm_fp4_bnstats_chunk": (I64, [I64, I64, I64]),
    "bnn_gemm_fp4_bnstats": (I32, [P, I64, P, I64, P, P, P, I64, P, I64, I64, I64, F32, ctypes.c_uint64, P, I64,
                                   P]),
    "bnn_gemm_i8_bnstats_ok": (I32, [I64, I64, I64, I64, I64]),
    "bnn_gemm_i8_s20_ok": (I32, [I64, I64, I64, I64, ctypes.c_double]),
    "bnn_gemm_i8_affine_bnstats_s20": (I32, [P, I64, P, I64, P, ctypes.c_double, I64, P, P, I64, I64, I64, I64, P,
                                             I64, P, P, P]),
    "bnn_bn_apply_pack_s20": (I32, [P, P, P, F32, I64, I64, P, P, P, P, P, P, I64, P, I64, I32, P]),
    "bnn_bn_bwd_i8cols_s20": (I32, [P, P, P, F32, P, I64, I64, P, P, P, P, P, I32, P, P, P, I64, I64, P, P, P, P,
                                    P]),
    "bnn_bn_bwd_i8cols_s20_pre": (I32, [P, P, P, F32, P, I64, I64, P, P, P, P, P, I32, P, P, P, I64, I64, P, P, P,
                                        P, P]),
    "bnn_gemm_i8_affine_bnstats": (I32, [P, I64, P, I64, P, P, P, ctypes.c_double, P, I64, I64, I64, I64, P, I64,
                                         P]),
    "bnn_linear_nsmall_workspace": (I64, [I64, I64, I64]),
    "bnn_linear_nsmall_fwd": (I32, [P, I64, I64, P, P, I64, P, P]),
    "bnn_linear_nsmall_bwd": (I32, [P, P, P, I64, I64, I64, P, P, P, P, I64, P]),
    "bnn_col_sums_narrow": (I32, [P, I64, I64, I64, P, P]),
    "bnn_cross_entropy_ok": (I32, [I64]),
    "bnn_cross_entropy_workspace": (I64, [I64]),
    "bnn_cross_entropy_fwd": (I32, [P, P, I64, I64, I64, P, P, I64, P]),
    "bnn_cross_entropy_bwd": (I32, [P, P, I64, I64, I64, P, P, P, P]),
    "bnn_unit_to_pixels": (I32, [P, I64, P, P, P]),
    "bnn_pixels_pack": (I32, [P, I64, I64, I64, P, I64, P, I64, P]),
    "bnn_row_sums": (I32, [P, I64, I64, I64, P, P]),
    "bnn_gemm_fp4": (I32, [P, I64, P, I64, P, P, I64, I64, I64, I64, P]),
    "bnn_gemm_fp4_i16": (I32, [P, I64, P, I64, P, I64, I64, I64, I64, P]),
    "bnn_gemm_set_variant": (I32, [I32]),
    "bnn_gemm_set_raster": (I32, [I32]),
    "bnn_adam_pack_set_tile256": (I32, [I32]),
    "bnn_gemm_i8_kernel": (ctypes.c_char_p, [I32, I32, I64, I64, I64]),
    "bnn_gemm_xnor": (I32, [P, P, I64, P, P, I64, P, P, I64, I64, I64, I64, P]),
    "bnn_conv2d_fwd": (I32, [P, I32, P, P, P, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32, P]),
    "bnn_conv2d_bwd_data": (I32, [P, P, P, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32, P]),
    "bnn_conv2d_bwd_filter_workspace": (I64, [I64, I64, I64, I64, I64, I32]),
    "bnn_conv2d_bwd_filter": (I32, [P, P, I32, P, P, P, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32,
                                    I32, P]),
    "bnn_conv_set_mfma": (I32, [I32]),
    "bnn_conv_set_c1_filter": (I32, [I32]),
    "bnn_conv_set_popc": (I32, [I32]),
    "bnn_bn2d_set_rows": (I32, [I32]),
    "bnn_bn2d_bwd_stats_q": (I32, [P, P, I32, P, I64, I64, I64, I64, P, P, P, P, I32, I32, P, P, P, P, P, P]),
    "bnn_conv2d_bwd_filter_bn_ok": (I32, [I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32]),
    "bnn_conv2d_bwd_filter_bn": (I32, [P, P, I32, P, P, P, P, P, P, P, F32, I32, P, I32, P, P, P, I64, I64, I64, I64,
                                       I64, I64, I64, I32, I32, I32, I32, P]),
    "bnn_conv_bf3_plan": (I32, [I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32, P]),
    "bnn_bn_workspace": (I64, [I64, I64]),
    "bnn_bn_fwd_train": (I32, [P, I64, I64, P, P, P, P, F32, F32, P, P, P, P, I32, P, P]),
    "bnn_bn_fwd_final_parts": (I32, [P, I64, I64, I64, I64, P, P, F32, F32, P, P, P, P]),
    "bnn_bn_fwd_eval": (I32, [P, I64, I64, P, P, P, P, F32, P, I32, P, P]),
    "bnn_bn_bwd": (I32, [P, P, I64, I64, P, P, P, P, P, I32, P, P, P, P, P]),
    "bnn_bn_bwd_eval": (I32, [P, P, I64, I64, P, P, P, P, I32, P, P, P, P, P]),
    "bnn_bn2d_workspace": (I64, [I64, I64]),
    "bnn_bn2d_fwd_train": (I32, [P, I64, I64, I64, I64, P, P, P, P, F32, F32, P, P, P, I32, I32, P, P]),
    "bnn_bn2d_fwd_eval": (I32, [P, I64, I64, I64, I64, P, P, P, P, F32, P, I32, I32, P, P]),
    "bnn_bn2d_bwd": (I32, [P, P, I64, I64, I64, I64, P, P, P, P, I32, I32, P, P, P, P, P]),
    "bnn_bn2d_bwd_eval": (I32, [P, P, I64, I64, I64, I64, P, P, P, P, I32, I32, P, P, P, P, P]),
    "bnn_bn2d_fwd_train_q": (I32, [P, P, I32, I64, I64, I64, I64, P, P, P, P, F32, F32, P, P, P, I32, I32, P, P]),
    "bnn_bn2d_bwd_q": (I32, [P, P, I32, P, I64, I64, I64, I64, P, P, P, P, I32, I32, P, P, P, P, P]),
    "bnn_conv2d_fwd_q": (I32, [P, P, P, I32, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32, P]),
    "bnn_conv2d_fwd_q_ok": (I32, [I32, I64, I64, I64, I64, I64, I64, I64, I32, I32, I32, I32]),
    "bnn_bn_dropout_fwd_train": (I32, [P, I64, I64, P, P, P, P, F32, F32, P, P, P, P, I32, F32, U64, P, P, P]),
    "bnn_dropout_keep_bits_bytes": (I64, [I64, I64]),
    "bnn_bn_set_head_reduce_cols": (I32, [I32]),
    "bnn_gemm_i8_bnstats_set_tile": (I32, [I32]),
    "bnn_bn_dropout_bwd": (I32, [P, P, I64, I64, P, P, P, P, P, I32, F32, U64, P, P, P, P, P]),
    "bnn_bn_bwd_q6": (I32, [P, P, I64, I64, P, P, P, P, P, I32, F32, U64, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "bnn_dropout_mask": (I32, [I64, F32, U64, P, P]),
    "bnn_bn_head_workspace": (I64, [I64, I64, I32]),
    "bnn_bn_head_fwd": (I32, [P, I64, I64, P, P, P, P, P, F32, U64, P, P, I32, P, P, P]),
    "bnn_bn_head_bwd_q6": (I32, [P, P, P, I32, I64, I64, P, P, P, P, P, F32, U64, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "bnn_bn_apply_pack": (I32, [P, I64, I64, P, P, P, P, P, I32, P, I64, P, I64, I32, P]),
    "bnn_bn_fwd_train_i16": (I32, [P, P, I64, I64, P, P, P, P, F32, F32, P, P, P, F32, U64, P, P, P]),
    "bnn_bn_apply_pack_i16": (I32, [P, P, I64, I64, P, P, P, P, P, P, I64, P, I64, I32, P]),
    "bnn_bn_bwd_q6_i16": (I32, [P, P, P, I64, I64, P, P, P, P, P, I32, F32, U64, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "bnn_bn_head_fwd_i16": (I32, [P, P, I64, I64, P, P, P, P, P, F32, U64, P, P, I32, P, P, P]),
    "bnn_bn_head_bwd_q6_i16": (I32, [P, P, P, P, I32, I64, I64, P, P, P, P, P, F32, U64, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "bnn_bn_bwd_i8cols_workspace": (I64, [I64, I64]),
    "bnn_bn_bwd_i8cols": (I32, [P, P, I64, I64, P, P, P, P, P, I32, P, P, P, I64, I64, P, P, P, P, P]),
    "bnn_bn_bwd_i8cols_pre": (I32, [P, P, I64, I64, P, P, P, P, P, I32, P, P, P, I64, I64, P, P, P, P, P]),
    "bnn_bn_bwd_stats_pre": (I32, [P, I64, I64, I64, I32, P, P, P, P, P, P, P, P]),
    "bnn_bn_bwd_q6_pre": (I32, [P, P, I64, I64, P, P, P, P, P, I32, F32, U64, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "bnn_bn_bwd_q6_i16_pre": (I32, [P, P, P, I64, I64, P, P, P, P, P, I32, F32, U64, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "bnn_gemm_fp6_bnstats_rows": (I64, [I64]),
    "bnn_gemm_fp6_bnstats": (I32, [P, P, P, I64, P, P, I64, P, I64, I64, I64, I64, P, P, I32, P, P, P, P, P, I32, I32, P, P]),
    "bnn_hardtanh_bwd": (I32, [P, P, P, I64, P]),
    "bnn_adam_clamp": (I32, [P, P, P, P, I64, F32, F32, F32, F32, I64, F32, I32, P]),
    "bnn_adam_clamp_pack": (I32, [P, P, P, P, I64, I64, F32, F32, F32, F32, I64, F32, I32, I32, P, I64, P, I64, I32,
                                  P]),
    "bnn_adam_schedule": (I32, [F32, F32, F32, I64, I64, P]),
    "bnn_adam_clamp_multi": (I32, [I32, P, P, P, P, P, P, P, F32, F32, F32, F32, P, P, F32, P]),
    "bnn_adam_clamp_sched": (I32, [P, P, P, P, I64, F32, F32, F32, P, P, F32, I32, P]),
    "bnn_adam_clamp_pack_sched": (I32, [P, P, P, P, I64, I64, F32, F32, F32, P, P, F32, I32, I32, P, I64, P, I64,
                                        I32, P]),
    "bnn_counter_add": (I32, [P, I64, P]),
    "bnn_set_seed_counter": (I32, [P]),
    "bnn_quant6_scale_rows": (I64, [I64]),
    "bnn_quant6_rows": (I32, [P, I64, I64, I64, I64, P, P, P, P, P]),
    "bnn_quant6_cols_workspace": (I64, [I64, I64]),
    "bnn_quant6_cols_t": (I32, [P, I64, I64, I64, I64, P, P, P, P, P, P]),
    "bnn_gemm_fp6": (I32, [P, P, P, I64, P, P, I64, P, P, I64, I64, I64, I64, P]),
    "bnn_gemm_fp6_workspace": (I64, [I64, I64, I64]),
    "bnn_gemm_fp6_ws": (I32, [P, P, P, I64, P, P, I64, P, P, I64, I64, I64, I64, P, I64, P]),
    "bnn_fp4_panel_bytes": (I64, [I64, I64]),
    "bnn_fp4_panelize": (I32, [P, I64, I64, I64, P, P]),
    "bnn_gemm_fp6_panel_ws": (I32, [P, P, P, I64, P, P, I64, P, P, I64, I64, I64, I64, P, I64, P]),
    "bnn_gemm_fp6_kernel": (ctypes.c_char_p, [I64, I64]),
    "bnn_gemm_fp6_kernel_k": (ctypes.c_char_p, [I64, I64, I64]),
    "bnn_gemm_fp6_kernel_kr": (ctypes.c_char_p, [I64, I64, I64, I32]),
    "bnn_gemm_fp6_set_variant": (I32, [I32]),
    "bnn_gemm_fp6_set_persistent": (I32, [I32]),
    "bnn_gemm_fp6_set_half": (I32, [I32, ctypes.c_double]),
    "bnn_gemm_fp6_set_half_group": (I32, [I32]),
}

_lib = None


def library_path():
    return os.environ.get("BNN_LIB", DEFAULT_PATH)


def lib():
    """Load libbnn.so once.  Raises RuntimeError (no fallback) if it is missing."""
    global _lib
    if _lib is None:
        path = library_path()
        if not os.path.exists(path):
            raise RuntimeError(
                f"libbnn.so not found at {path}: build it with "
                "`make -C distributed-mnist-bnns_amd/csrc` (or __graft_entry__.build()). "
                "The BNN hot path has no CPU fallback.")
        L = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class BnnError(RuntimeError):
    pass


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().bnn_last_error().decode(errors="replace")
        raise BnnError(f"{name} failed (code {rc}): {msg}")
    return rc


def ptr(t):
    """Device pointer of a tensor (or NULL for None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
