#!/usr/bin/env python
"""Timing of nqk_attention_fused at the ViT-Base B=256 shape (stream events), for the main
build and, side by side in ONE process (interleaved rounds; MI355X_MICROARCH.md: never rank
builds timed in different processes), any diagnostic builds:

  AM_LIBS=name=path,...   extra builds (tools/gemm_diag.sh with SRC=nqk_attn)
  AM_ROUNDS, AM_REPS      interleaved rounds, launches per timing"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import DeviceArray  # noqa: E402

if os.environ.get("GM_LIB"):  # replace the main build
    _lib.LIB_PATH = os.environ["GM_LIB"]
_lib.ensure_init()
libs = {"main": _lib.load()}
for item in filter(None, os.environ.get("AM_LIBS", "").split(",")):
    name, path = item.split("=", 1)
    lib = ctypes.CDLL(os.path.abspath(path))
    for fname, argt in _lib.SIGNATURES.items():
        fn = getattr(lib, fname)
        fn.argtypes = argt
        fn.restype = ctypes.c_int
    assert lib.nqk_init(0) == 0
    libs[name] = lib
B, H, T, Dh = int(os.environ.get("AM_B", 256)), 12, 197, 64
ROUNDS, REPS = int(os.environ.get("AM_ROUNDS", 3)), int(os.environ.get("AM_REPS", 20))
rng = np.random.default_rng(0)
q, k, v = (DeviceArray.from_host(rng.integers(-128, 128, size=(B * H * T, Dh), dtype=np.int8)) for _ in range(3))
ctx = DeviceArray((B, T, H * Dh), np.int8)
a = _lib.Attention()
a.heads, a.tokens, a.hdim, a.ld_out, a.bit_width = H, T, Dh, H * Dh, 8
a.zq, a.zk, a.s_qk, a.div = -3, 4, 0.0008, 8.0
a.s_p, a.zp_p, a.s_pv, a.zv = 1 / 255, -128, 0.0001, -1
a.s_ctx, a.zp_ctx = 0.02, 2


def timed(lib):
    def run():
        rc = lib.nqk_attention_fused(q.vp, k.vp, v.vp, ctx.vp, B * H, ctypes.byref(a))
        assert rc == 0, rc
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.nqk_event_create(ctypes.byref(e0))
    lib.nqk_event_create(ctypes.byref(e1))
    run()
    lib.nqk_event_record(e0)
    for _ in range(REPS):
        run()
    lib.nqk_event_record(e1)
    ms = ctypes.c_float()
    lib.nqk_event_elapsed(e0, e1, ctypes.byref(ms))
    lib.nqk_sync()
    return 1e3 * ms.value / REPS


outs = {}
res = {n: [] for n in libs}
for _ in range(ROUNDS):
    for n, lib in libs.items():
        res[n].append(timed(lib))
        if n not in outs:
            outs[n] = ctx.to_host()
elems = B * H * T * T
byts = 3 * B * H * T * Dh + B * T * H * Dh
for n, ts in res.items():
    us = min(ts)
    same = "same ctx as main" if np.array_equal(outs[n], outs["main"]) else "ctx DIFFERS from main"
    print(f"attention[{n}] B={B} H={H} T={T}: min {us:8.1f} us  med {sorted(ts)[len(ts) // 2]:8.1f} us  "
          f"{elems / us / 1e3:7.2f} G score elems/s  {byts / us / 1e3:7.1f} GB/s algorithmic HBM  ({same})", flush=True)
