#!/usr/bin/env python
"""Per-kernel timing of the int8 GEMMs at the ViT-Base B=256 shapes (stream events,
interleaved repetitions in one process).  Prints one line per (kernel, shape)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import DeviceArray  # noqa: E402

if os.environ.get("GM_LIB"):  # a diagnostic build (tools/gemm_diag.sh)
    _lib.LIB_PATH = os.environ["GM_LIB"]
_lib.ensure_init()
M = int(os.environ.get("GM_M", 256 * 197))
shapes = {"qkv": (2304, 768, 0), "out": (768, 768, 3), "up": (3072, 768, 4), "down": (768, 3072, 3)}
rng = np.random.default_rng(0)


def ev():
    e = ctypes.c_void_p()
    _lib.call("nqk_event_create", ctypes.byref(e))
    return e


def timeit(fn, reps=10):
    a, b = ev(), ev()
    fn()
    _lib.call("nqk_event_record", a)
    for _ in range(reps):
        fn()
    _lib.call("nqk_event_record", b)
    ms = ctypes.c_float()
    _lib.call("nqk_event_elapsed", a, b, ctypes.byref(ms))
    return ms.value / reps


A = {}
for name, (N, K, epi) in shapes.items():
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt0 = DeviceArray.from_host(rng.integers(-128, 128, size=(N, K), dtype=np.int8))
    from numpy_quant.plan import _pack_b
    bt, kind = _pack_b(bt0, 8)  # the plan's tile-packed weight image
    col = DeviceArray.from_host(np.zeros(N, np.int64))
    colterm = DeviceArray.from_host(np.zeros(N, np.int32))
    bias = DeviceArray.from_host(np.zeros(N, np.float32))
    resid = DeviceArray((M, N), np.float32)
    out = DeviceArray((M, N), np.float32)
    c32 = DeviceArray((M, N), np.int32)
    outs = [DeviceArray((M, 768), np.int8) for _ in range(3)] if epi == 0 else [out]
    e = _lib.Epilogue()
    e.zp_flags = _lib.ZP_COL
    e.bit_width = 8
    e.group_cols = 768 if epi == 0 else (1 << 30)
    e.tokens, e.heads, e.hdim = 197, 12, 64
    e.zpa = 3
    e.col = col.ptr
    e.colterm = colterm.ptr
    # realistic magnitudes: uniform int8 operands give |acc| ~ 150e3 * sqrt(K / 768), so
    # s_acc puts the dequantized values near N(0, 1) (GELU outputs in [-0.17, ~4])
    for g in range(3):
        e.s_acc[g] = 7e-6 * (768 / K) ** 0.5
        e.s_out[g] = 0.0165 if epi == 4 else 0.03
        e.zp_out[g] = -118 if epi == 4 else -2
        e.out[g] = outs[min(g, len(outs) - 1)].ptr
    if epi == 4:
        h = DeviceArray((M, N), np.int8)
        e.out[0] = h.ptr
    e.bias = bias.ptr
    e.resid = resid.ptr
    e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
    e.b_packed = kind
    ops = 2.0 * M * N * K

    def fused():
        _lib.call("nqk_qgemm_fused", epi, a.vp, bt.vp, 1, M, N, K, K, K, None, 0, 0, ctypes.byref(e))

    def plain():
        _lib.call("nqk_qgemm_i8", a.vp, bt0.vp, c32.vp, 1, M, N, K, K, K, N, None, 0, 0, 0)

    def oldk():
        os.environ["NQK_NO_PROJ"] = "1"
        try:
            fused()
        finally:
            del os.environ["NQK_NO_PROJ"]

    def null():
        _lib.call("nqk_qgemm_fused", 5, a.vp, bt.vp, 1, M, N, K, K, K, None, 0, 0, ctypes.byref(e))

    only = os.environ.get("GM_ONLY")  # e.g. "down:null_epi" (profiling one variant)
    for tag, fn in (("fused", fused), ("old_big", oldk), ("null_epi", null)):
        if only and only != f"{name}:{tag}":
            continue
        ms = timeit(fn)
        print(f"{name:5s} {tag:9s} M={M} N={N} K={K}: {ms * 1e3:8.1f} us  {ops / ms / 1e9:8.1f} TOPS  "
              f"({100 * ops / ms / 1e9 / 5033.2:5.1f}% of int8 peak)", flush=True)
