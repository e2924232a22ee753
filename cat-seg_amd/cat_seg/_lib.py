"""ctypes binding of libcatseg_hip.so (include/catseg_hip.h).

The library is the product: there is no fallback.  Loading fails loudly when the
shared object is missing, and `require_gpu()` fails when no HIP device is
visible, so nothing on the path can silently run elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CATSEG_HIP_LIB", os.path.join(_HERE, "libcatseg_hip.so"))

F32, BF16, FP8 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_GELU, ACT_QUICKGELU, ACT_SIGMOID = 0, 1, 2, 3, 4
BIG = 1 << 62

i64, i32, f32, vp = C.c_int64, C.c_int, C.c_float, C.c_void_p


class RowMap(C.Structure):
    _fields_ = [(n, i64) for n in ("d1", "m1", "s1", "d2", "m2", "s2", "off")]


def rowmap(d1=1, m1=BIG, s1=1, d2=1, m2=1, s2=0, off=0) -> RowMap:
    return RowMap(d1, m1, s1, d2, m2, s2, off)


IDENTITY = rowmap()


class SwinAttnArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("ld_x", i64),
        ("ln_g", vp), ("ln_b", vp), ("eps", f32),
        ("w_qkv", vp), ("b_qkv", vp),
        ("gqk", vp), ("ld_g", i64), ("gmap", RowMap),
        ("out", vp), ("ld_out", i64),
        ("S", i64), ("img_h", i32), ("img_w", i32), ("window", i32), ("shift", i32), ("n_heads", i32),
        ("head_dim", i32), ("scale", f32),
        ("dtype", i32),
    ]


class GemmArgs(C.Structure):
    _fields_ = [
        ("A", vp), ("lda", i64), ("amap", RowMap),
        ("W", vp), ("ldw", i64),
        ("M", i64), ("N", i64), ("K", i64),
        ("bias", vp),
        ("add", vp), ("ld_add", i64), ("addmap", RowMap), ("add_ncols", i64),
        ("act", i32), ("alpha", f32),
        ("res", vp), ("ld_res", i64),
        ("res2", vp), ("ld_res2", i64),
        ("out", vp), ("ldo", i64),
        ("store_mode", i32), ("cvt_k", i32), ("cvt_hin", i32), ("cvt_win", i32), ("cvt_cout", i32),
        ("dtype_a", i32), ("dtype_out", i32),
    ]


class AttnArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("ld_qkv", i64),
        ("out", vp), ("ld_out", i64),
        ("n_seq", i64), ("seq_len", i32), ("n_heads", i32), ("head_dim", i32),
        ("scale", f32), ("causal", i32),
        ("mode", i32), ("img_h", i32), ("img_w", i32), ("window", i32), ("shift", i32),
        ("dtype", i32),
    ]


class ClassAttnArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("ld_x", i64),
        ("ln_g", vp), ("ln_b", vp), ("eps", f32),
        ("w_qkv", vp), ("b_qkv", vp),
        ("tg", vp), ("ld_tg", i64), ("tg_bstride", i64),
        ("n_pad", i32), ("k_pad", vp), ("v_pad", vp), ("attn_eps", f32),
        ("y", vp), ("ld_y", i64),
        ("B", i64), ("T", i32), ("HW", i32), ("n_heads", i32), ("head_dim", i32),
        ("dtype", i32),
        ("tgk_t", vp), ("ld_tgk_t", i64), ("tgk_t_bstride", i64),
    ]


class LinAttnArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("ld_qkv", i64),
        ("x", vp), ("y", vp), ("ld_xy", i64),
        ("B", i64), ("T", i32), ("HW", i32), ("n_heads", i32), ("head_dim", i32),
        ("n_pad", i32), ("k_pad", vp), ("v_pad", vp), ("eps", f32),
        ("dtype", i32),
    ]


class ClassSeqArgs(C.Structure):
    _fields_ = [
        ("qkv", vp), ("ld_qkv", i64), ("packed", vp), ("ld_packed", i64),
        ("o", vp), ("ld_o", i64), ("x", vp), ("y", vp), ("ld_xy", i64),
        ("B", i64), ("T", i32), ("HW", i32), ("C", i32),
        ("n_pad", i32), ("k_pad", vp), ("v_pad", vp),
        ("dtype", i32),
    ]


class RowsEpi(C.Structure):
    _fields_ = [
        ("bias", vp),
        ("add", vp), ("ld_add", i64), ("addmap", RowMap), ("add_ncols", i64),
        ("act", i32),
        ("res", vp), ("ld_res", i64),
        ("res2", vp), ("ld_res2", i64),
        ("out", vp), ("ldo", i64),
        ("store_mode", i32), ("cvt_k", i32), ("cvt_hin", i32), ("cvt_win", i32), ("cvt_cout", i32),
    ]


class ConvArgs(C.Structure):
    _fields_ = [
        ("src1", vp), ("s1_slice_stride", i64), ("s1_offset", i64), ("c1", i32),
        ("src2", vp), ("s2_slice_stride", i64), ("s2_offset", i64), ("c2", i32), ("src2_div", i64),
        ("S", i64), ("H", i32), ("W", i32),
        ("weight", vp), ("c_out", i32),
        ("bias", vp), ("act", i32),
        ("gn_mean", vp), ("gn_rstd", vp), ("gn_gamma", vp), ("gn_beta", vp), ("gn_cpg", i32),
        ("out", vp), ("stats", vp), ("stats_cpg", i32),
        ("dtype", i32),
        ("addend", vp), ("addend_slice_stride", i64), ("addend_div", i64),
        ("workspace", vp), ("workspace_bytes", i64),
    ]


class GemmExArgs(C.Structure):
    _fields_ = [
        ("A", vp), ("a_sm", i64), ("a_sk", i64),
        ("B", vp), ("b_sk", i64), ("b_sn", i64),
        ("M", i64), ("N", i64), ("K", i64),
        ("C", vp), ("ldc", i64),
        ("alpha", f32), ("beta", i32),
        ("workspace", vp), ("workspace_bytes", i64),
        ("act_u", vp), ("ld_u", i64), ("act", i32),
    ]


class WinAttnBwdArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("ld_qkv", i64),
        ("o", vp), ("ld_o", i64),
        ("dout", vp), ("ld_dout", i64),
        ("dq", vp), ("dk", vp), ("dv", vp), ("ld_dqkv", i64),
        ("S", i64), ("img_h", i32), ("img_w", i32), ("window", i32), ("shift", i32), ("n_heads", i32),
        ("head_dim", i32), ("scale", f32),
    ]


class AttnBwdArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("ld_qkv", i64),
        ("o", vp), ("ld_o", i64),
        ("dout", vp), ("ld_dout", i64),
        ("dq", vp), ("dk", vp), ("dv", vp), ("ld_dqkv", i64),
        ("n_seq", i64), ("seq_len", i32), ("n_heads", i32), ("head_dim", i32), ("scale", f32), ("causal", i32),
        ("workspace", vp), ("workspace_bytes", i64),
    ]


class LinAttnBwdArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("ld_qkv", i64),
        ("dy", vp), ("ld_dy", i64),
        ("dq", vp), ("dk", vp), ("dv", vp), ("ld_dqkv", i64),
        ("B", i64), ("T", i32), ("HW", i32), ("n_heads", i32), ("head_dim", i32),
        ("n_pad", i32), ("k_pad", vp), ("v_pad", vp), ("eps", f32),
        ("dk_pad", vp), ("dv_pad", vp),
        ("workspace", vp), ("workspace_bytes", i64),
    ]


class Conv2dArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("ld_x", i64),
        ("S", i64), ("H", i32), ("W", i32), ("cin", i32),
        ("w", vp), ("ld_w", i64),
        ("cout", i32), ("ksize", i32), ("pad", i32),
        ("bias", vp), ("act", i32),
        ("y", vp), ("ld_y", i64),
        ("alpha", f32), ("beta", i32),
        ("dw", vp),
        ("workspace", vp), ("workspace_bytes", i64),
    ]


# name -> (argtypes); every entry returns int
_SIGS = {
    "catseg_gemm": [C.POINTER(GemmArgs), vp],
    "catseg_gemm_fp8": [C.POINTER(GemmArgs), vp, vp, vp],
    "catseg_quant_fp8_rows": [vp, i32, i64, i64, i64, vp, i64, vp, vp],
    "catseg_layernorm_fp8": [vp, i64, RowMap, i32, vp, i64, vp, vp, vp, i64, i64, f32, vp],
    "catseg_semseg_confusion": [vp, i64, i64, i64, vp, i32, i32, i32, vp, vp, vp],
    "catseg_rows_gemm": [vp, i64, i64, vp, vp, f32, vp, i64, C.POINTER(RowsEpi), i32, vp],
    "catseg_rows_mlp": [vp, i64, i64, vp, vp, f32, vp, vp, i64, i32, vp, C.POINTER(RowsEpi), i32, vp],
    "catseg_layernorm": [vp, i64, RowMap, i32, vp, i64, i32, vp, vp, i64, i64, f32, vp],
    "catseg_l2normalize": [vp, i64, RowMap, i32, vp, i64, i32, i64, i64, f32, vp],
    "catseg_attention": [C.POINTER(AttnArgs), vp],
    "catseg_linear_attention": [C.POINTER(LinAttnArgs), vp],
    "catseg_class_seq_pack": [C.POINTER(ClassSeqArgs), vp],
    "catseg_class_seq_unpack_add": [C.POINTER(ClassSeqArgs), vp],
    "catseg_conv3x3": [C.POINTER(ConvArgs), vp],
    "catseg_conv3x3_partial": [vp, i64, i32, i32, i32, vp, i32, vp, i32, vp],
    "catseg_upconv3x3": [C.POINTER(ConvArgs), vp],
    "catseg_bce_onehot_loss": [vp, i64, i32, i32, i32, vp, i32, i32, i32, vp, vp, vp],
    "catseg_bce_onehot_loss_backward": [vp, i64, i32, i32, i32, vp, i32, i32, i32, vp, vp, vp, vp],
    "catseg_swin_proj_mlp": [vp, i64, vp, i64, i64, vp, vp, vp, vp, C.c_float, vp, vp, i64, vp, vp, vp, i64, vp],
    "catseg_upconv3x3_stats_tile": [],
    "catseg_upconv_addend": [vp, i64, i32, i32, i32, vp, vp, i32, vp, i32, vp],
    "catseg_conv_tile_rows": [],
    "catseg_conv3x3_stats_tile": [C.POINTER(ConvArgs)],
    "catseg_conv3x3_workspace": [C.POINTER(ConvArgs)],
    "catseg_groupnorm_stats": [vp, i64, i32, i32, i64, f32, vp, vp, vp],
    "catseg_groupnorm_relu": [vp, vp, i64, i64, i32, i32, vp, vp, vp, vp, i32, vp],
    "catseg_conv3x3_head": [vp, i64, i32, i32, i32, i32, vp, f32, vp, i32, vp, i32, vp],
    "catseg_conv3x3_head_gn": [vp, i64, i32, i32, i32, i32, vp, f32, vp, vp, vp, vp, i32, vp, i32, vp, i32, vp],
    "catseg_corr_embed": [vp, i64, i64, vp, i64, i32, i32, i32, vp, vp, i32, vp, i32, vp],
    "catseg_topk_classes": [vp, i64, i64, i64, i32, i32, i32, vp, vp, vp],
    "catseg_gather_rows": [vp, i64, vp, i64, i64, vp, i64, i32, vp],
    "catseg_transpose_rows": [vp, i64, i64, i64, i64, i64, vp, i64, i32, vp],
    "catseg_convert": [vp, i64, RowMap, i32, vp, i64, i32, i64, i64, vp],
    "catseg_fill_f32": [vp, i64, f32, vp],
    "catseg_preprocess_im2col": [vp, vp, i64, i32, i32, vp, vp, i32, i32, vp, i64, i32, vp],
    "catseg_vit_embed": [vp, vp, vp, vp, vp, i64, i32, i32, vp, vp],
    "catseg_bicubic_resize": [vp, i32, i32, vp, i32, vp],
    "catseg_postprocess": [vp, i64, i32, i32, i32, i32, i32, vp, i32, i32, vp],
    "catseg_swin_window_attention": [C.POINTER(SwinAttnArgs), vp],
    "catseg_class_attention": [C.POINTER(ClassAttnArgs), vp],
    "catseg_resize_bilinear": [vp, i64, i32, i32, i32, i32, i32, vp, i32, i32, vp],
    "catseg_avgpool_rows": [vp, i64, i32, i32, i32, i32, i32, vp, i32, vp],
    "catseg_upsample_add_rows": [vp, i64, i32, i32, i32, vp, i32, i32, i32, vp],
    "catseg_sliding_crops": [vp, vp, i64, i32, i32, i32, i32, i32, vp, vp],
    "catseg_sliding_merge": [vp, i64, i32, i32, i32, i32, i32, i32, vp, vp],
    "catseg_token_embed": [vp, i64, i32, vp, vp, i32, vp, vp],
    "catseg_eot_gather": [vp, vp, i64, i32, i32, vp, vp],
    "catseg_convt64_gn": [vp, i64, i64, vp, vp, vp, vp, i32, vp, i64, C.POINTER(RowsEpi), vp],
    # training-side entry points (include/catseg_hip_train.h)
    "catseg_gemm_ex": [C.POINTER(GemmExArgs), vp],
    "catseg_gemm_ex_workspace": [i64, i64, i64],
    "catseg_colsum": [vp, i64, i64, i64, vp, f32, i32, vp, i64, vp],
    "catseg_colsum_workspace": [i64, i64],
    "catseg_layernorm_backward": [vp, i64, vp, vp, i64, vp, i64, i32, i64, i64, f32, vp, vp, i32, vp, i64, vp],
    "catseg_layernorm_backward_workspace": [i64, i64],
    "catseg_act_forward": [vp, vp, i64, i32, vp],
    "catseg_act_backward": [vp, vp, vp, i64, i32, vp],
    "catseg_groupnorm_stats_rows": [vp, i64, i64, i32, i32, f32, vp, vp, vp, i64, vp],
    "catseg_groupnorm_stats_rows_workspace": [i64, i64, i32, i32],
    "catseg_groupnorm_relu_backward": [vp, vp, vp, i64, i64, i32, i32, vp, vp, vp, vp, vp, vp, i32, vp, i64, vp],
    "catseg_groupnorm_relu_backward_workspace": [i64, i64, i32],
    "catseg_l2normalize_backward": [vp, i64, RowMap, vp, i64, vp, i64, RowMap, i32, i64, i64, f32, vp],
    "catseg_axpby": [vp, vp, vp, i64, f32, f32, vp],
    "catseg_add_dev_scalar": [vp, i64, vp, vp],
    "catseg_scatter_rows": [vp, i64, vp, i64, i64, vp, i64, vp],
    "catseg_adamw_chunks": [vp, i32],
    "catseg_adamw_chunk_table": [vp, i32, vp],
    "catseg_adamw_step": [vp, vp, i64, f32, f32, f32, f32, vp, vp, i64, vp],
    "catseg_corr_embed_backward_input": [vp, vp, vp, i64, i32, i32, i32, i32, vp],
    "catseg_sum_classes": [vp, i64, i64, i32, i64, i32, vp, i64, i32, vp],
    "catseg_sum_pixels": [vp, i64, i64, i32, i64, i32, vp, i64, i32, vp],
    "catseg_avgpool_backward_rows": [vp, i64, i32, i32, i32, i32, i32, vp, i32, vp],
    "catseg_upsample_ac_backward_rows": [vp, i64, i32, i32, i32, i32, i32, vp, i32, vp],
    "catseg_convt_gather": [vp, i64, i64, i32, i32, i32, i32, vp, vp],
    "catseg_window_attention_backward": [C.POINTER(WinAttnBwdArgs), vp],
    "catseg_attention_backward": [C.POINTER(AttnBwdArgs), vp],
    "catseg_attention_backward_workspace": [i64, i32, i32],
    "catseg_linear_attention_backward": [C.POINTER(LinAttnBwdArgs), vp],
    "catseg_linear_attention_backward_workspace": [i64, i32],
    "catseg_conv2d_nhwc": [C.POINTER(Conv2dArgs), vp],
    "catseg_conv2d_wgrad": [C.POINTER(Conv2dArgs), vp],
    "catseg_conv2d_wgrad_workspace": [C.POINTER(Conv2dArgs)],
    "catseg_head_conv_backward": [vp, vp, vp, vp, vp, i64, i32, i32, i32, vp, i64, vp],
    "catseg_head_conv_backward_workspace": [i64, i32, i32, i32],
    "catseg_abi_version": [],
    "catseg_last_error": [],
}
# diagnostics entry (include/catseg_hip_tuning.h), not part of the product ABI
_TUNING = {
    "catseg_tuning_set": [C.c_char_p, i32],
    "catseg_tuning_get": [C.c_char_p, C.POINTER(C.c_int)],
    "catseg_tuning_list": [],
}

EXPORTED = tuple(_SIGS)

_lib = None


def load() -> C.CDLL:
    """Load libcatseg_hip.so (raises if it is missing — there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libcatseg_hip.so not found at {LIB_PATH}: build it with "
            "`make -C cat-seg_amd/csrc` (or __graft_entry__.build()); the CAT-Seg HIP path has no fallback")
    lib = C.CDLL(LIB_PATH)
    for name, args in list(_SIGS.items()) + list(_TUNING.items()):
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = (C.c_char_p if name in ("catseg_last_error", "catseg_tuning_list") else
                      C.c_int64 if name.endswith("_workspace") or name == "catseg_adamw_chunks" else C.c_int)
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.catseg_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def tune(name: str, value: int) -> None:
    """Force an A/B knob (include/catseg_hip_tuning.h; tests / tools only): process-wide, read at
    launch.  Raises on an unknown name."""
    call("catseg_tuning_set", name.encode(), int(value))


def tuning(name: str) -> int:
    v = C.c_int(0)
    call("catseg_tuning_get", name.encode(), C.byref(v))
    return v.value


def tuning_knobs():
    return load().catseg_tuning_list().decode().split(",")


def require_gpu():
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError("the CAT-Seg HIP path needs a visible MI355X (torch.cuda.is_available() is False)")
    load()
