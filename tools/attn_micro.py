#!/usr/bin/env python
"""Timing of nqk_attention_fused at the ViT-Base B=256 shape (stream events)."""
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
B, H, T, Dh = int(os.environ.get("AM_B", 256)), 12, 197, 64
rng = np.random.default_rng(0)
q, k, v = (DeviceArray.from_host(rng.integers(-128, 128, size=(B * H * T, Dh), dtype=np.int8)) for _ in range(3))
ctx = DeviceArray((B, T, H * Dh), np.int8)
a = _lib.Attention()
a.heads, a.tokens, a.hdim, a.ld_out, a.bit_width = H, T, Dh, H * Dh, 8
a.zq, a.zk, a.s_qk, a.div = -3, 4, 0.0008, 8.0
a.s_p, a.zp_p, a.s_pv, a.zv = 1 / 255, -128, 0.0001, -1
a.s_ctx, a.zp_ctx = 0.02, 2


def ev():
    e = ctypes.c_void_p()
    _lib.call("nqk_event_create", ctypes.byref(e))
    return e


def run():
    _lib.call("nqk_attention_fused", q.vp, k.vp, v.vp, ctx.vp, B * H, ctypes.byref(a))


run()
e0, e1 = ev(), ev()
reps = 20
_lib.call("nqk_event_record", e0)
for _ in range(reps):
    run()
_lib.call("nqk_event_record", e1)
ms = ctypes.c_float()
_lib.call("nqk_event_elapsed", e0, e1, ctypes.byref(ms))
us = 1e3 * ms.value / reps
elems = B * H * T * T
byts = 3 * B * H * T * Dh + B * T * H * Dh
print(f"attention B={B} H={H} T={T}: {us:8.1f} us/launch  {elems / us / 1e3:7.2f} G score elems/s  "
      f"{byts / us / 1e3:7.1f} GB/s algorithmic HBM", flush=True)
