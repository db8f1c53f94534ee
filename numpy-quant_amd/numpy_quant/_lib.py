"""ctypes binding of libnqk.so (include/nqk.h).

The library is built in-tree by `__graft_entry__.build()` (csrc/Makefile) and
sits next to this file.  There is no fallback: if it is missing or fails to load,
every entry point raises, so a silent CPU path can never stand in for the kernels.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnqk.so")

NQK_I8, NQK_I16, NQK_I32, NQK_I64, NQK_F32 = 1, 2, 3, 4, 5
ZP_NONE, ZP_SCALAR, ZP_ROW, ZP_COL, ZP_KCONST, ZP_FULL = 0, 1, 2, 4, 8, 16
ADD, SUB, MUL, DIV = 0, 1, 2, 3
NEG, EXP, ERF, SQRT, RELU, SIGMOID, RECIP, TANH = range(8)

_p = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_int64
_f = ctypes.c_float
_lp = ctypes.POINTER(ctypes.c_int64)

class Epilogue(ctypes.Structure):
    """Mirror of `nqk_epilogue` (include/nqk.h)."""
    _fields_ = [("zp_flags", ctypes.c_int32), ("bit_width", ctypes.c_int32), ("group_cols", ctypes.c_int32),
                ("tokens", ctypes.c_int32), ("heads", ctypes.c_int32), ("hdim", ctypes.c_int32),
                ("ld_out", ctypes.c_int32), ("col_absmax", ctypes.c_int32),
                ("zpa", ctypes.c_int64), ("zpb", ctypes.c_int64), ("kdim", ctypes.c_int64),
                ("row", ctypes.c_void_p), ("col", ctypes.c_void_p),
                ("s_acc", ctypes.c_float * 3), ("s_out", ctypes.c_float * 3), ("zp_out", ctypes.c_int64 * 3),
                ("out", ctypes.c_void_p * 3), ("bias", ctypes.c_void_p), ("resid", ctypes.c_void_p),
                ("div", ctypes.c_float), ("add1", ctypes.c_float), ("mul2", ctypes.c_float),
                ("b_packed", ctypes.c_int32), ("colterm", ctypes.c_void_p), ("bt_pg", ctypes.c_void_p),
                ("gelu_lut", ctypes.c_void_p), ("lut_k", ctypes.c_float * 5), ("lut_n", ctypes.c_int32),
                ("col_l1max", ctypes.c_int32),
                ("ln_gamma", ctypes.c_void_p), ("ln_beta", ctypes.c_void_p), ("ln_out", ctypes.c_void_p),
                ("ln_eps", ctypes.c_float), ("ln_scale", ctypes.c_float), ("ln_zp", ctypes.c_int64)]


class Attention(ctypes.Structure):
    """Mirror of `nqk_attention` (include/nqk.h)."""
    _fields_ = [("heads", ctypes.c_int32), ("tokens", ctypes.c_int32), ("hdim", ctypes.c_int32),
                ("ld_out", ctypes.c_int32), ("bit_width", ctypes.c_int32), ("pad0", ctypes.c_int32),
                ("zq", ctypes.c_int64), ("zk", ctypes.c_int64),
                ("s_qk", ctypes.c_float), ("div", ctypes.c_float), ("s_p", ctypes.c_float), ("s_pv", ctypes.c_float),
                ("zp_p", ctypes.c_int64), ("zv", ctypes.c_int64),
                ("s_ctx", ctypes.c_float), ("pad1", ctypes.c_float), ("zp_ctx", ctypes.c_int64)]


SIGNATURES = {
    "nqk_init": [_i],
    "nqk_device_count": [ctypes.POINTER(_i)],
    "nqk_malloc": [ctypes.POINTER(_p), ctypes.c_size_t],
    "nqk_free": [_p],
    "nqk_memcpy_h2d": [_p, _p, ctypes.c_size_t],
    "nqk_memcpy_d2h": [_p, _p, ctypes.c_size_t],
    "nqk_memcpy_d2d": [_p, _p, ctypes.c_size_t],
    "nqk_memset": [_p, _i, ctypes.c_size_t],
    "nqk_sync": [],
    "nqk_stream": [ctypes.POINTER(_p)],
    "nqk_set_stream": [_i],
    "nqk_stream_fork": [],
    "nqk_stream_join": [],
    "nqk_timer_start": [],
    "nqk_timer_stop": [],
    "nqk_timer_ms": [ctypes.POINTER(_f)],
    "nqk_event_create": [ctypes.POINTER(_p)],
    "nqk_event_record": [_p],
    "nqk_event_elapsed": [_p, _p, ctypes.POINTER(_f)],
    "nqk_event_destroy": [_p],
    "nqk_event_wait": [_p],
    "nqk_graph_begin": [],
    "nqk_graph_end": [ctypes.POINTER(_p)],
    "nqk_graph_abort": [],
    "nqk_graph_launch": [_p],
    "nqk_graph_destroy": [_p],
    "nqk_quantize": [_p, _p, _i, _l, _f, _l, _i, _i, _p, _l],
    "nqk_dequantize": [_p, _i, _p, _l, _l, _l, _f, _i, _l, _l, _l, _l, _p, _p, _lp],
    "nqk_requantize": [_p, _i, _p, _i, _p, _i, _l, _l, _l, _f, _i, _l, _l, _l, _l, _p, _p, _lp, _f, _l, _i, _i],
    "nqk_rowsum": [_p, _i, _p, _l, _l, _l, _l, _l],
    "nqk_relu_q": [_p, _i, _p, _i, _l, _l],
    "nqk_qgemm_i8": [_p, _p, _p, _l, _l, _l, _l, _l, _l, _l, _lp, _l, _l, _l],
    "nqk_qgemm_generic": [_p, _i, _p, _i, _p, _l, _l, _l, _l, _l, _l, _l, _l, _l, _lp, _l, _l, _l],
    "nqk_sgemm": [_p, _p, _p, _l, _l, _l, _l, _l, _l, _l, _l, _l, _lp, _l, _l, _l],
    "nqk_sgemv_t": [_p, _p, _p, _l, _l, _l, _l],
    "nqk_sgemv_small": [_p, _p, _p, _l, _l, _l],
    "nqk_sgemv_n": [_p, _p, _p, _l, _l, _l, _l],
    "nqk_im2col": [_p, _p] + [_l] * 12,
    "nqk_binary_f32": [_i, _p, _p, _p, _i, _lp, _lp, _lp],
    "nqk_unary_f32": [_i, _p, _p, _l],
    "nqk_add_scalar_f32": [_p, _f, _p, _l],
    "nqk_softmax_lastdim": [_p, _p, _l, _l],
    "nqk_layernorm_lastdim": [_p, _p, _p, _p, _l, _l, _f],
    "nqk_mean_lastdim": [_p, _p, _l, _l],
    "nqk_minmax_f32": [_p, _l, _p, _p, _l],
    "nqk_copy_strided": [_p, _p, _i, _i, _lp, _lp, _lp],
    "nqk_where_f32": [_p, _p, _p, _p, _i, _lp, _lp, _lp, _lp],
    "nqk_pack_b": [_p, _p, _l, _l, _l],
    "nqk_pack_b4": [_p, _p, _l, _l, _l],
    "nqk_pack_pg": [_p, _p, _l, _l, _l, _i],
    "nqk_qgemm_fused": [_i, _p, _p, _l, _l, _l, _l, _l, _l, _lp, _l, _l, ctypes.POINTER(Epilogue)],
    "nqk_qgemm_last_kernel": [],
    "nqk_pack_pg4": [_p, _p, _l, _l, _l, _i],
    "nqk_gelu_lut_build": [_f, _l, _i, _f, _f, _f, _p, ctypes.POINTER(_f), ctypes.POINTER(ctypes.c_int32)],
    "nqk_gelu_lut_capacity": [],
    "nqk_gelu_lut_check": [_f, _l, _i, _f, _f, _f, _p, ctypes.POINTER(_f), ctypes.c_int32,
                           ctypes.POINTER(ctypes.c_uint64)],
    "nqk_ln_quant": [_p, _p, _p, _p, _l, _l, _f, _f, _l, _i],
    "nqk_softmax_quant": [_p, _p, _p, _l, _l, _l, _f, _l, _i],
    "nqk_transpose_pad_i8": [_p, _p, _p, _l, _l, _l, _l],
    "nqk_attention_fused": [_p, _p, _p, _p, _l, _p],
    "nqk_selftest_fastmath": [_p, _p],
    "nqk_selftest_gelu_filter": [_p],
    "nqk_sgemm_embed": [_p, _p, _p, _p, _p, _p, _l, _l, _l, _l],
    "nqk_patchify_dequant": [_p, _p, _l, _l, _l, _l, _l, _l, _f, _l],
    "nqk_embed_weight_order": [],
    "nqk_embed_q": [_p, _f, _l, _p, _p, _p, _p, _p, _l, _l, _l, _l, _l, _l, _l],
    "nqk_comm_unique_id": [_p],
    "nqk_comm_init": [_p, _i, _i],
    "nqk_comm_bcast": [_p, ctypes.c_size_t, _i],
    "nqk_comm_gather": [_p, _p, ctypes.c_size_t, _i],
    "nqk_comm_barrier": [],
    "nqk_comm_destroy": [],
}


class NQKError(RuntimeError):
    pass


_lib = None


_ROUND4 = {"nqk_gelu_lut_build", "nqk_gelu_lut_check", "nqk_pack_pg4"}  # absent from round-3 builds


def load() -> ctypes.CDLL:
    """Load libnqk.so once and declare every exported signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NQKError(f"libnqk.so not built ({LIB_PATH}); run __graft_entry__.build() — "
                       "there is no CPU fallback for the hot path")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if name in _ROUND4:  # a previous round's build (same-box A/B runs, tools/ab.sh)
                continue
            raise NQKError(f"libnqk.so lacks {name}: rebuild it (__graft_entry__.build())")
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.nqk_last_error.argtypes = []
    lib.nqk_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise NQKError(f"{name}: {lib.nqk_last_error().decode(errors='replace')}")


def i64arr(values) -> ctypes.Array:
    vals = [int(v) for v in values]
    return (ctypes.c_int64 * max(1, len(vals)))(*vals)


_initialised = -1


def ensure_init(device: int | None = None) -> None:
    global _initialised
    if device is None:
        device = int(os.environ.get("NQK_DEVICE", os.environ.get("LOCAL_RANK", "0")) or 0)
        if _initialised >= 0:
            return
    if _initialised == device:
        return
    call("nqk_init", device)
    _initialised = device


def device_count() -> int:
    n = ctypes.c_int(0)
    call("nqk_device_count", ctypes.byref(n))
    return n.value
