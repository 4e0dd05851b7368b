"""ctypes binding of libdfu_hip.so — the C ABI declared in include/dfu_hip.h.

This is the only place the host touches the native library.  Loading fails loudly: there is
no CPU or ATen fallback for any op on the hot path (SURVEY.md §7 design stance).
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# DFU_HIP_LIB: another build of the library (A/B timing of two builds); default: in-tree
LIB_PATH = os.environ.get("DFU_HIP_LIB") or os.path.join(_HERE, "libdfu_hip.so")
HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "include", "dfu_hip.h"))

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_float = ctypes.c_float
c_uint64 = ctypes.c_uint64
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p

# enum dfu_operand_mode
OPND_KMAJOR, OPND_MNMAJOR, OPND_CONV_FWD, OPND_CONV_DGRAD, OPND_CONV_DGRAD_W, OPND_CONV_WGRAD_X = range(6)
# enum dfu_epilogue
(EPI_BF16, EPI_BF16_RELU, EPI_BF16_GELU, EPI_F32, EPI_F32_RESID, EPI_BF16_DGELU, EPI_BF16_ADD,
 EPI_F32_ACC, EPI_F32_ACC_CONVW, EPI_BF16_STATS, EPI_PATCH, EPI_F32_STATS,
 EPI_BF16_DSTATS, EPI_X3_GELU, EPI_F16_DUAL, EPI_F16_GELU) = range(16)
# dfu_gemm_desc.operand_type
OPERAND_BF16, OPERAND_F16 = 0, 1

DFU_E_INVALID = 1001
DFU_E_UNSUPPORTED = 1002


class GemmDesc(ctypes.Structure):
    """Mirror of `dfu_gemm_desc` (include/dfu_hip.h)."""
    _fields_ = [
        ("M", c_int32), ("N", c_int32), ("K", c_int32),
        ("a_mode", c_int32), ("b_mode", c_int32),
        ("A", c_void_p), ("lda", c_int64),
        ("B", c_void_p), ("ldb", c_int64),
        ("C", c_void_p), ("ldc", c_int64),
        ("epilogue", c_int32), ("alpha", c_float),
        ("bias", c_void_p),
        ("aux", c_void_p), ("ldaux", c_int64),
        ("aux_out", c_void_p), ("ldaux_out", c_int64),
        ("stats", c_void_p),
        ("split_k", c_int32),
        ("ep_tokens", c_int32),
        ("conv_n", c_int32), ("conv_h", c_int32), ("conv_w", c_int32), ("conv_c", c_int32),
        ("conv_k", c_int32), ("conv_r", c_int32), ("conv_s", c_int32),
        ("conv_stride", c_int32), ("conv_pad", c_int32),
        ("conv_p", c_int32), ("conv_q", c_int32),
        ("tile", c_int32),
        ("workspace", c_void_p), ("workspace_bytes", c_int64),
        ("tile_counters", c_void_p), ("tile_counters_len", c_int32),
        ("operand_type", c_int32),
        ("a_seg", c_int32), ("a_lo", c_void_p),
        ("x3_pairs", c_int32),
    ]


class ReduceEntry(ctypes.Structure):
    """Mirror of `dfu_reduce_entry` (include/dfu_hip.h)."""
    _fields_ = [("partial", c_void_p), ("stride", c_int64), ("out", c_void_p),
                ("blocks", c_int32), ("D", c_int32)]


REDUCE_BATCH = 8
P = c_void_p
I32 = c_int32
I64 = c_int64
F = c_float

# name -> argtypes (restype is always int32 unless listed in _RESTYPE)
PROTOTYPES = {
    "dfu_last_error_string": [],
    "dfu_version": [],
    "dfu_zero": [P, I64, P],
    "dfu_streams_abort_capture": [P, I32, P],
    "dfu_stream_capture_status": [P, P],
    "dfu_stream_create": [I32, P],
    "dfu_stream_destroy": [P],
    "dfu_stream_wait": [P, P],
    "dfu_gemm": [ctypes.POINTER(GemmDesc), P],
    "dfu_gemm_stats_tiles": [I32],
    "dfu_gemm_workspace_bytes": [ctypes.POINTER(GemmDesc)],
    "dfu_gemm_plan": [ctypes.POINTER(GemmDesc), ctypes.POINTER(c_int32), ctypes.POINTER(c_int32)],
    "dfu_gemm_set_persistent": [I32],
    "dfu_gemm_set_inkernel_reduce": [I32],
    "dfu_gemm_set_tail_split": [I32],
    "dfu_gemm_f32": [I32, I32, I32, P, I64, I64, P, I64, I64, P, I64, P, I32, I32, P, I64, P],
    "dfu_gemm_f32_workspace_bytes": [I32, I32, I32],
    "dfu_pack_conv_weight": [P, P, I32, I32, I32, I32, P],
    "dfu_conv_grad_krsc_to_oihw": [P, P, I32, I32, I32, I32, P],
    "dfu_cast_rows_bf16": [P, I64, P, I64, I32, I32, P],
    "dfu_transpose_bf16": [P, I32, I32, P],
    "dfu_cast_rows_f32": [P, I64, P, I64, I32, I32, P],
    "dfu_cast_rows_f16": [P, I64, P, I64, I32, I32, P],
    "dfu_im2col_f32": [P, I64, I64, I64, I64, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, I32, P],
    "dfu_patchify_f32": [P, I64, I64, I64, I64, I32, I32, I32, I32, I32, P, P],
    "dfu_col2im_f32": [P, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, P],
    "dfu_unpatchify_f32": [P, I32, I32, I32, I32, I32, P, P],
    "dfu_gradcam": [P, I32, I64, I64, I64, P, I32, I64, I64, I64, I32, I32, I32, P, P],
    "dfu_saliency": [P, I32, I32, I32, P, P],
    "dfu_bn_finalize": [P, I32, I32, I32, P, P, F, F, P, P, P, P, P, P, P, P, P, I32, P],
    "dfu_bn_finalize_ws_bytes": [I32, I32],
    "dfu_bn_bwd_finalize_ws_bytes": [I32, I32],
    "dfu_bn_eval_coeffs": [P, P, P, P, F, I32, P, P, P],
    "dfu_bn_apply": [P, P, P, P, I32, P, I64, I32, P],
    "dfu_bn_tile_stats": [P, I64, I32, P, P],
    "dfu_bn_apply_mask": [P, P, P, P, I32, P, P, I64, I32, P],
    "dfu_bn_bwd_blocks": [I64, I32],
    "dfu_bn_bwd_reduce": [P, P, P, I32, P, P, P, P, I64, I32, P, P],
    "dfu_bn_bwd_finalize": [P, I32, I64, I32, P, P, I32, P, P, P, P, P, I32, P],
    "dfu_bn_bwd_apply": [P, P, P, I32, P, P, P, P, P, I64, I32, P, P, P],
    "dfu_bn_bwd_ws_bytes": [I64, I32],
    "dfu_bn_bwd": [P, P, P, I32, P, P, P, P, P, I64, I32, I32, P, P, P, P, P, I64, P, I32, P],
    "dfu_maxpool_fwd": [P, I32, I32, I32, I32, P, P, I32, I32, P],
    "dfu_maxpool_bn_fwd": [P, P, P, I32, I32, I32, I32, P, P, I32, I32, P],
    "dfu_maxpool_bwd": [P, P, I32, I32, I32, I32, I32, I32, P, P],
    "dfu_avgpool_fwd": [P, I32, I32, I32, P, P],
    "dfu_avgpool_bwd": [P, I32, I32, I32, P, P],
    "dfu_layernorm_fwd": [P, I64, I32, I32, P, P, F, P, I64, I32, P, P, P],
    "dfu_ln_bwd_blocks": [I32],
    "dfu_layernorm_bwd": [P, I64, I32, P, I64, P, P, P, I32, I32, P, I64, P, P, P, P],
    "dfu_reduce_partials": [P, I32, I32, I32, P, P, P],
    "dfu_reduce_partials_batch": [ctypes.POINTER(ReduceEntry), I32, P],
    "dfu_attention_fwd": [P, I32, I32, I32, I32, F, P, P, P],
    "dfu_attention_fwd_f16": [P, I32, I32, I32, I32, F, P, P, P, P],
    "dfu_attention_bwd": [P, P, P, P, I32, I32, I32, I32, F, P, P, P],
    "dfu_attention_bwd_qkv16": [P, P, P, P, I32, I32, I32, I32, F, P, P, P],
    "dfu_attention_npad": [I32],
    "dfu_vit_cls_rows": [P, P, P, I32, I32, I32, P],
    "dfu_vit_embed_bwd": [P, I32, I32, I32, P, P, P, P, P, P],
    "dfu_colsum": [P, I32, I64, I32, I32, P, P, P],
    "dfu_colsum_blocks": [I32],
    "dfu_gather_rows_f32": [P, I64, I32, I32, I32, I32, P, I64, P],
    "dfu_scatter_rows_f32": [P, I64, I32, I32, I32, I32, P, I64, P],
    "dfu_relu_fwd": [P, P, I64, I32, P],
    "dfu_relu_bwd": [P, P, P, I64, I32, P],
    "dfu_dropout_fwd": [P, P, P, I64, F, c_uint64, P, I32, P],
    "dfu_dropout_bwd": [P, P, P, I64, F, I32, P],
    "dfu_concat2_bf16": [P, I32, I32, P, I32, I32, I32, P, P],
    "dfu_split2_f32": [P, I32, I32, I32, I32, P, P, P],
    "dfu_ce_weighted_fwd": [P, P, P, I32, I32, P, P, P],
    "dfu_ce_weighted_bwd": [P, P, I32, I32, P, P],
    "dfu_adamw": [P, P, P, P, P, I32, P, I32, F, F, F, F, F, P, P],
    "dfu_adamw_flat": [P, P, P, P, I64, F, F, F, F, F, P, P, P, P, I64, I64, P],
    "dfu_step_increment": [P, P],
    "dfu_argmax_rows": [P, I32, I32, P, P],
    "dfu_softmax_rows": [P, I32, I32, P, P],
    "dfu_metrics_accumulate": [P, P, I32, I32, P, P, P, P, P],
    "dfu_split_x3": [P, I64, I32, I32, I32, P, I32, P, I64, P],
    "dfu_pack_conv_weight_x3": [P, P, I32, I32, I32, I32, I32, P],
    "dfu_stem_conv_x3": [P, I64, I64, I64, I64, I32, I32, I32, I32, P, I32, I32, I32, I32, I32,
                         P, P, P, P, P],
    "dfu_stem_wgrad_ws_bytes": [I32, I32, I32],
    "dfu_stem_wgrad_x3": [P, I64, I64, I64, I64, I32, I32, I32, I32, P, I32, I32, I32, I32, I32,
                          P, P, I64, P],
    "dfu_maxpool_bn_fwd_x3": [P, P, P, P, I32, I32, I32, I32, P, P, P, P, I32, I32, P],
    "dfu_im2col_f32_x3": [P, I64, I64, I64, I64, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, P, I32, P],
    "dfu_patchify_f32_x3": [P, I64, I64, I64, I64, I32, I32, I32, I32, I32, P, P],
    "dfu_bn_apply_x3": [P, P, P, P, P, P, I32, I32, P, P, P, P, P, I64, I32, P],
    "dfu_maxpool_fwd_x3": [P, I32, I32, I32, I32, P, P, P, I32, I32, P],
    "dfu_avgpool_fwd_x3": [P, P, I32, I32, I32, P, P],
    "dfu_layernorm_fwd_x3": [P, I64, I32, I32, P, P, F, P, P, P, P, P],
    "dfu_layernorm_fwd_h16": [P, I64, I32, I32, P, P, F, P, P, P, P, P],
    "dfu_gelu_x3": [P, I64, I32, P, P, P, P],
    "dfu_attention_fwd_f32": [P, I32, I32, I32, I32, F, I32, P, P, P, P, P],
    "dfu_resize_ksize": [I32, I32],
    "dfu_resize_coeffs": [I32, I32, P, P],
    "dfu_resize_batch": [P, P, P, I32, I32, I32, P, P, P],
    "dfu_augment_normalize": [P, P, I32, I32, I32, P, P, P, P, P],
}
_RESTYPE = {"dfu_last_error_string": c_char_p, "dfu_gemm_workspace_bytes": c_int64,
            "dfu_gemm_f32_workspace_bytes": c_int64, "dfu_bn_finalize_ws_bytes": c_int64,
            "dfu_bn_bwd_finalize_ws_bytes": c_int64, "dfu_stem_wgrad_ws_bytes": c_int64,
            "dfu_bn_bwd_ws_bytes": c_int64}


def header_symbols(path=HEADER_PATH):
    """Every function name declared in include/dfu_hip.h (used by the symbol-export test)."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(dfu_\w+)\s*\(", text, re.M)))


class DfuError(RuntimeError):
    def __init__(self, msg, code=0):
        super().__init__(msg)
        self.code = code


_lib = None


def load():
    """Load libdfu_hip.so once; raise if it is missing (never fall back)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DfuError(
            f"libdfu_hip.so not found at {LIB_PATH}; build it with "
            f"`make -C dfu-multimodal_amd` (or __graft_entry__.build()). There is no fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPE.get(name, c_int32)
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().dfu_last_error_string()
        msg = msg.decode() if msg else ""
        raise DfuError(f"{what or 'dfu call'} failed (rc={rc}): {msg}", rc)
