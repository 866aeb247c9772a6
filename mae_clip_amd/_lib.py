"""ctypes binding of libmaeclip.so (include/maeclip.h).

The product path has no fallback: if the shared library is missing, fails to
load, or no gfx950 device is visible, every op raises. (The CPU restatement in
/oracle is test infrastructure and is never imported from here.)
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MAECLIP_LIB", os.path.join(_HERE, "libmaeclip.so"))

F32, BF16 = 0, 1
# plan options (include/maeclip.h MAECLIP_OPT_*), by name without the prefix
OPTIONS = ("GEMM_BM", "GEMM_SK", "GEMM_SPLIT", "GEMM_SPLIT_D", "GEMM_SPLIT_MINK", "GEMM_BM128", "GEMM_GRID",
           "WG_SK", "ATTN_TWO", "ATTN_ROWS", "ATTN_DIAG", "ATTN_BW16", "ATTN_FW16")
ABI_VERSION = 11

c_i32, c_i64, c_f32, c_u64, c_vp, c_sz = C.c_int32, C.c_int64, C.c_float, C.c_uint64, C.c_void_p, C.c_size_t


class GemmArgs(C.Structure):
    _fields_ = [("A", c_vp), ("B", c_vp), ("C", c_vp),
                ("M", c_i64), ("N", c_i64), ("K", c_i64),
                ("lda", c_i64), ("ldb", c_i64), ("ldc", c_i64),
                ("batch", c_i64), ("strideA", c_i64), ("strideB", c_i64), ("strideC", c_i64),
                ("dtype", c_i32), ("out_dtype", c_i32), ("a_layout", c_i32), ("b_layout", c_i32),
                ("epilogue", c_i32), ("alpha", c_f32), ("beta", c_f32),
                ("bias", c_vp), ("aux", c_vp), ("aux_out", c_vp), ("ldaux", c_i64),
                ("resid", c_vp), ("ldr", c_i64), ("colsum_partial", c_vp),
                ("splitk", c_i32), ("workspace", c_vp),
                ("q8", c_vp), ("ldq8", c_i64), ("q8_scale", c_vp), ("q8_fmt", c_i32)]


class AttnArgs(C.Structure):
    _fields_ = [("qkv", c_vp), ("o", c_vp), ("lse", c_vp), ("dout", c_vp), ("dqkv", c_vp),
                ("key_mask", c_vp), ("colsum_partial", c_vp),
                ("ld_qkv", c_i64), ("ld_o", c_i64), ("ld_dqkv", c_i64),
                ("B", c_i32), ("n", c_i32), ("H", c_i32), ("head_dim", c_i32), ("dtype", c_i32),
                ("scale", c_f32), ("dropout_p", c_f32), ("seed", c_u64), ("step_ptr", c_vp),
                ("q8", c_vp), ("ldq8", c_i64), ("q8_scale", c_vp), ("q8_fmt", c_i32)]


class LnFwdArgs(C.Structure):
    _fields_ = [("x", c_vp), ("x_dtype", c_i32), ("res", c_vp), ("ldres", c_i64), ("in_dropout_p", c_f32),
                ("gamma", c_vp), ("beta", c_vp), ("y", c_vp), ("y_dtype", c_i32), ("y2", c_vp), ("ldy2", c_i64),
                ("xsum_out", c_vp), ("ldxs", c_i64), ("mean", c_vp), ("rstd", c_vp), ("out_dropout_p", c_f32),
                ("seed_in", c_u64), ("seed_out", c_u64), ("step_ptr", c_vp),
                ("M", c_i64), ("D", c_i64), ("ldx", c_i64), ("ldy", c_i64), ("eps", c_f32),
                ("q8", c_vp), ("ldq8", c_i64), ("q8_scale", c_vp), ("q8_fmt", c_i32)]


class LnBwdArgs(C.Structure):
    _fields_ = [("dy", c_vp), ("dy_dtype", c_i32), ("x", c_vp), ("x_dtype", c_i32),
                ("mean", c_vp), ("rstd", c_vp), ("gamma", c_vp), ("dres", c_vp),
                ("dx", c_vp), ("dx_bf", c_vp), ("lddx_bf", c_i64),
                ("dgamma_partial", c_vp), ("dbeta_partial", c_vp), ("dx_colsum_partial", c_vp),
                ("M", c_i64), ("D", c_i64), ("ldx", c_i64), ("lddy", c_i64), ("lddx", c_i64),
                ("dres_pool", c_vp), ("pool_n", c_i64),
                ("q8", c_vp), ("ldq8", c_i64), ("q8_scale", c_vp), ("q8_fmt", c_i32)]


class MtEntry(C.Structure):
    _fields_ = [("p0", c_vp), ("p1", c_vp), ("p2", c_vp), ("p3", c_vp), ("p4", c_vp),
                ("n", c_i64), ("chunk_start", c_i64)]


class ColsumEntry(C.Structure):
    _fields_ = [("partial", c_vp), ("out", c_vp), ("P", c_i64), ("N", c_i64), ("scale", c_f32), ("accumulate", c_i32),
                ("block_start", c_i64)]


class AdamwHparams(C.Structure):
    _fields_ = [("lr", c_f32), ("beta1", c_f32), ("beta2", c_f32), ("eps", c_f32), ("weight_decay", c_f32),
                ("step_size", c_f32), ("bc2_sqrt", c_f32), ("grad_scale", c_f32), ("step_ptr", c_vp)]


class MaskArgs(C.Structure):
    _fields_ = [("ids_shuffle", c_vp), ("ids_restore", c_vp), ("mask", c_vp), ("noise", c_vp),
                ("B", c_i32), ("L", c_i32), ("len_keep", c_i32),
                ("seed", c_u64), ("step", c_u64), ("sample_offset", c_u64), ("step_ptr", c_vp)]


_U8_FIELDS = [("img_u8", c_vp), ("u8_mean", c_f32 * 3), ("u8_std", c_f32 * 3), ("u8_max_pixel", c_f32)]


class PatchArgs(C.Structure):
    _fields_ = [("img", c_vp), ("ids_shuffle", c_vp), ("out", c_vp), ("ld_out", c_i64),
                ("B", c_i32), ("C", c_i32), ("S", c_i32), ("p", c_i32), ("keep", c_i32), ("dtype", c_i32)] + _U8_FIELDS


class TokensArgs(C.Structure):
    _fields_ = [("y", c_vp), ("ldy", c_i64), ("ids_shuffle", c_vp), ("ids_restore", c_vp),
                ("pos", c_vp), ("cls", c_vp), ("x", c_vp), ("dx", c_vp), ("dy", c_vp), ("dpos", c_vp), ("dcls", c_vp),
                ("B", c_i32), ("L", c_i32), ("keep", c_i32), ("D", c_i32), ("dtype", c_i32)]


class UnshuffleArgs(C.Structure):
    _fields_ = [("y", c_vp), ("ldy", c_i64), ("ids_shuffle", c_vp), ("ids_restore", c_vp),
                ("mask_token", c_vp), ("pos", c_vp), ("out", c_vp), ("dout", c_vp), ("dy", c_vp),
                ("dmask_partial", c_vp), ("colsum_partial", c_vp),
                ("B", c_i32), ("L", c_i32), ("keep", c_i32), ("D", c_i32), ("dtype", c_i32)]


class MaeLossArgs(C.Structure):
    _fields_ = [("pred", c_vp), ("ldp", c_i64), ("img", c_vp), ("mask", c_vp), ("row_loss", c_vp),
                ("dpred", c_vp), ("lddp", c_i64), ("grad_out", c_vp), ("colsum_partial", c_vp),
                ("loss_scale", c_f32), ("mask_count", c_f32),
                ("B", c_i32), ("C", c_i32), ("S", c_i32), ("p", c_i32), ("L", c_i32), ("norm_pix", c_i32),
                ("dtype", c_i32)] + _U8_FIELDS


class ClipArgs(C.Structure):
    _fields_ = [("I", c_vp), ("T", c_vp), ("ld_I", c_i64), ("ld_T", c_i64), ("N", c_i64), ("P", c_i64),
                ("temperature", c_f32), ("loss", c_vp), ("row_loss_out", c_vp), ("dI", c_vp), ("dT", c_vp),
                ("ld_dI", c_i64), ("ld_dT", c_i64), ("grad_row0", c_i64), ("grad_rows", c_i64),
                ("workspace", c_vp), ("ws_bytes", c_sz)]


class WgradProblem(C.Structure):
    _fields_ = [("dy", c_vp), ("x", c_vp), ("dw", c_vp), ("N", c_i64), ("K", c_i64), ("ldy", c_i64), ("ldx", c_i64)]


class Fp8wEntry(C.Structure):
    _fields_ = [("w", c_vp), ("q", c_vp), ("sq", c_vp), ("qt", c_vp), ("sqt", c_vp),
                ("rows", c_i32), ("cols", c_i32), ("ld", c_i32), ("ldqt", c_i32),
                ("row_begin", c_i64), ("unit_begin", c_i64), ("part_begin", c_i64)]


class ImageSrc(C.Structure):
    _fields_ = [("src", c_vp), ("H", c_i32), ("W", c_i32), ("row_stride", c_i64)]


class PreprocessArgs(C.Structure):
    _fields_ = [("images", c_vp), ("dst", c_vp), ("B", c_i64), ("S", c_i64),
                ("mean", c_f32 * 3), ("std", c_f32 * 3), ("max_pixel", c_f32)]


class ImageU8Args(C.Structure):
    _fields_ = [("src", c_vp), ("dst", c_vp), ("B", c_i64), ("H", c_i64), ("W", c_i64),
                ("mean", c_f32 * 3), ("std", c_f32 * 3), ("max_pixel", c_f32)]


# name -> (restype, argtypes)
_SIGS = {
    "maeclip_abi_version": (c_i32, []),
    "maeclip_last_error": (C.c_char_p, []),
    "maeclip_device_count": (c_i32, []),
    "maeclip_set_option": (c_i32, [c_i32, c_i32]),
    "maeclip_get_option": (c_i32, [c_i32]),
    "maeclip_gemm": (c_i32, [C.POINTER(GemmArgs), c_vp]),
    "maeclip_gemm_colsum_rows": (c_i64, [c_i64]),
    "maeclip_gemm_workspace": (c_i64, [C.POINTER(GemmArgs)]),
    "maeclip_gemm_splitk": (c_i32, [c_i64, c_i64, c_i64]),
    "maeclip_gemm_fp8": (c_i32, [C.POINTER(GemmArgs), c_vp, c_vp, c_vp]),
    "maeclip_quant_rows_fp8": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "maeclip_fp8b_scale_bytes": (c_i64, [c_i64, c_i64]),
    "maeclip_quant_blocks_fp8": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "maeclip_gemm_fp8_blocks": (c_i32, [C.POINTER(GemmArgs), c_vp, c_vp, c_vp]),
    "maeclip_quant_cols_fp8_workspace": (c_i64, [c_i64, c_i64]),
    "maeclip_quant_weights_fp8_prepare": (c_i64, [C.POINTER(Fp8wEntry), c_i32]),
    "maeclip_quant_weights_fp8": (c_i32, [c_vp, C.POINTER(Fp8wEntry), c_i32, c_vp, c_i64, c_vp]),
    "maeclip_quant_cols_fp8": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "maeclip_wgrad_grouped_workspace": (c_i64, [C.POINTER(WgradProblem), c_i32, c_i64, c_i32]),
    "maeclip_wgrad_grouped": (c_i32, [C.POINTER(WgradProblem), c_i32, c_i64, c_i32, c_f32, c_vp, c_i64, c_vp]),
    "maeclip_image_normalize_u8": (c_i32, [C.POINTER(ImageU8Args), c_vp]),
    "maeclip_image_preprocess_u8": (c_i32, [C.POINTER(PreprocessArgs), c_vp]),
    "maeclip_l2_normalize": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_vp]),
    "maeclip_topk_rows": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp]),
    "maeclip_attn_fwd": (c_i32, [C.POINTER(AttnArgs), c_vp]),
    "maeclip_attn_bwd": (c_i32, [C.POINTER(AttnArgs), c_vp]),
    "maeclip_ln_fwd": (c_i32, [C.POINTER(LnFwdArgs), c_vp]),
    "maeclip_ln_bwd": (c_i32, [C.POINTER(LnBwdArgs), c_vp]),
    "maeclip_ln_bwd_partial_rows": (c_i32, [c_i64, c_i64]),
    "maeclip_colsum_reduce": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_f32, c_vp, c_vp]),
    "maeclip_rows_colsum": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "maeclip_rows_colsum_partial_rows": (c_i32, [c_i64]),
    "maeclip_rows_colsum_q8": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "maeclip_colsum_scratch": (c_i64, [c_i64, c_i64]),
    "maeclip_cast_flat": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_i64, c_f32, c_vp]),
    "maeclip_pool_fwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "maeclip_pool_bwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp]),
    "maeclip_dropout": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i64, c_f32, c_u64, c_vp, c_vp]),
    "maeclip_embed_fwd": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "maeclip_mt_chunk": (c_i64, []),
    "maeclip_colsum_multi": (c_i32, [c_vp, C.POINTER(ColsumEntry), c_i32, c_vp]),
    "maeclip_cast_multi": (c_i32, [c_vp, C.POINTER(MtEntry), c_i32, c_vp]),
    "maeclip_adamw_multi": (c_i32, [c_vp, C.POINTER(MtEntry), c_i32, C.POINTER(AdamwHparams), c_vp]),
    "maeclip_mask_ids": (c_i32, [C.POINTER(MaskArgs), c_vp]),
    "maeclip_patch_gather": (c_i32, [C.POINTER(PatchArgs), c_vp]),
    "maeclip_tokens_fwd": (c_i32, [C.POINTER(TokensArgs), c_vp]),
    "maeclip_tokens_bwd": (c_i32, [C.POINTER(TokensArgs), c_vp]),
    "maeclip_unshuffle_fwd": (c_i32, [C.POINTER(UnshuffleArgs), c_vp]),
    "maeclip_unshuffle_bwd": (c_i32, [C.POINTER(UnshuffleArgs), c_vp]),
    "maeclip_unshuffle_bwd_partial_rows": (c_i32, [c_i32]),
    "maeclip_mae_loss_fwd": (c_i32, [C.POINTER(MaeLossArgs), c_vp]),
    "maeclip_mae_loss_bwd": (c_i32, [C.POINTER(MaeLossArgs), c_vp]),
    "maeclip_mae_loss_bwd_partial_rows": (c_i32, [c_i32, c_i32]),
    "maeclip_clip_loss_workspace": (c_sz, [c_i64, c_i64, c_i64]),
    "maeclip_clip_loss": (c_i32, [C.POINTER(ClipArgs), c_vp]),
    "maeclip_counter_add": (c_i32, [c_vp, c_i64, c_vp]),
    "maeclip_counter_add_snap": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "maeclip_scalar_axpy": (c_i32, [c_vp, c_vp, C.c_float, c_vp, c_vp]),
    "maeclip_host_mapped_alloc": (c_i32, [C.c_int64, C.POINTER(c_vp), C.POINTER(c_vp)]),
    "maeclip_host_mapped_free": (c_i32, [c_vp]),
    "maeclip_copy_f32": (c_i32, [c_vp, c_vp, C.c_int64, c_vp]),
    "maeclip_copy_f32_slot": (c_i32, [c_vp, c_vp, C.c_int64, c_vp, c_vp]),
    "maeclip_gemm_impl": (c_i32, [C.POINTER(GemmArgs)]),
    "maeclip_scale_by_scalar2": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, C.c_float, c_vp]),
    "maeclip_memcpy_h2d": (c_i32, [c_vp, c_vp, c_sz, c_vp]),
    "maeclip_timestamp": (c_i32, [c_vp, c_vp]),
    "maeclip_wallclock_khz": (c_i64, []),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


class MaeClipNativeError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libmaeclip.so (no GPU needed to load; ops need a GPU)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MaeClipNativeError(
            f"libmaeclip.so not found at {path}: build it with `make` (or __graft_entry__.build()); "
            "mae_clip_amd has no CPU fallback")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.maeclip_abi_version() != ABI_VERSION:
        raise MaeClipNativeError("libmaeclip ABI mismatch")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.maeclip_last_error().decode(errors="replace")
        raise MaeClipNativeError(f"{what} failed ({rc}): {msg}")


def lib():
    return _lib if _lib is not None else load()
