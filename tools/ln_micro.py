#!/usr/bin/env python
"""Timing of nqk_ln_quant at the ViT-Base B=256 shape (50432 x 768), stream events, with
environment variants of the main build interleaved in one process (LNM_ENV="name:VAR=val;...");
GM_LIB selects a diagnostic build (tools/gemm_diag.sh)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import DeviceArray  # noqa: E402

if os.environ.get("GM_LIB"):
    _lib.LIB_PATH = os.environ["GM_LIB"]
_lib.ensure_init()
rows, cols = 256 * 197, int(os.environ.get("LN_COLS", 768))
rng = np.random.default_rng(0)
x = DeviceArray.from_host(rng.standard_normal((rows, cols), dtype=np.float32))
g = DeviceArray.from_host(np.ones(cols, np.float32))
b = DeviceArray.from_host(np.zeros(cols, np.float32))
out = DeviceArray((rows, cols), np.int8)


def ev():
    e = ctypes.c_void_p()
    _lib.call("nqk_event_create", ctypes.byref(e))
    return e


def run():
    _lib.call("nqk_ln_quant", x.vp, g.vp, b.vp, out.vp, rows, cols, 1e-12, 0.03, -3, 8)


def timed(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        run()
        a, c = ev(), ev()
        _lib.call("nqk_event_record", a)
        for _ in range(20):
            run()
        _lib.call("nqk_event_record", c)
        ms = ctypes.c_float()
        _lib.call("nqk_event_elapsed", a, c, ctypes.byref(ms))
        return ms.value / 20 * 1e3
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


# variants of the main build by environment, interleaved (LNM_ENV="name:VAR=val,...;...")
variants = {"main": {}}
for item in filter(None, os.environ.get("LNM_ENV", "").split(";")):
    name, kv = item.split(":", 1)
    variants[name] = dict(x.split("=", 1) for x in kv.split(","))
res = {n: [] for n in variants}
for _ in range(int(os.environ.get("LNM_ROUNDS", 5))):
    for n, env in variants.items():
        res[n].append(timed(env))
for n, ts in res.items():
    us = min(ts)
    print(f"ln_quant[{n}] {rows}x{cols}: min {us:.1f} us  med {sorted(ts)[len(ts) // 2]:.1f} us  "
          f"{rows * cols * 5 / us / 1e3:.0f} GB/s", flush=True)
