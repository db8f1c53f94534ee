#!/usr/bin/env python
"""Timing of nqk_ln_quant at the ViT-Base B=256 shape (50432 x 768), stream events, with
environment variants of the main build interleaved in one process (LNM_ENV="name:VAR=val;...") and
variant builds loaded next to the main one (LNM_LIBS="name=path,...", tools/diag_build.sh), each
checked byte for byte against the main build's output; GM_LIB replaces the main build."""
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
libs = {"main": _lib.load()}
for item in filter(None, os.environ.get("LNM_LIBS", "").split(",")):
    name, path = item.split("=", 1)
    lib = ctypes.CDLL(os.path.abspath(path))
    for fname, argt in _lib.SIGNATURES.items():
        fn = getattr(lib, fname)
        fn.argtypes = argt
        fn.restype = ctypes.c_int
    assert lib.nqk_init(0) == 0
    libs[name] = lib
rows, cols = 256 * 197, int(os.environ.get("LN_COLS", 768))
rng = np.random.default_rng(0)
x = DeviceArray.from_host(rng.standard_normal((rows, cols), dtype=np.float32))
g = DeviceArray.from_host(np.ones(cols, np.float32))
b = DeviceArray.from_host(np.zeros(cols, np.float32))
out = DeviceArray((rows, cols), np.int8)


def call(lib, fn, *args):
    rc = getattr(lib, fn)(*args)
    assert rc == 0, (fn, rc)


def ev(lib):
    e = ctypes.c_void_p()
    call(lib, "nqk_event_create", ctypes.byref(e))
    return e


def run(lib, o=out):
    call(lib, "nqk_ln_quant", x.vp, g.vp, b.vp, o.vp, rows, cols, ctypes.c_float(1e-12), ctypes.c_float(0.03), -3, 8)


def timed(env, lib):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        run(lib)
        a, c = ev(lib), ev(lib)
        call(lib, "nqk_event_record", a)
        for _ in range(20):
            run(lib)
        call(lib, "nqk_event_record", c)
        ms = ctypes.c_float()
        call(lib, "nqk_event_elapsed", a, c, ctypes.byref(ms))
        return ms.value / 20 * 1e3
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


# variants of the main build by environment, interleaved (LNM_ENV="name:VAR=val,...;...")
variants = {n: ({}, lib) for n, lib in libs.items()}
for item in filter(None, os.environ.get("LNM_ENV", "").split(";")):
    name, kv = item.split(":", 1)
    variants[name] = (dict(x.split("=", 1) for x in kv.split(",")), libs["main"])
ref = DeviceArray((rows, cols), np.int8)
run(libs["main"], ref)
call(libs["main"], "nqk_sync")
want = ref.to_host()
for n, (env, lib) in variants.items():
    o = DeviceArray((rows, cols), np.int8)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    run(lib, o)
    call(lib, "nqk_sync")
    for k, v in old.items():
        os.environ.pop(k, None) if v is None else os.environ.__setitem__(k, v)
    assert np.array_equal(o.to_host(), want), f"ln_quant[{n}] differs from the main build"
res = {n: [] for n in variants}
for _ in range(int(os.environ.get("LNM_ROUNDS", 5))):
    for n, (env, lib) in variants.items():
        res[n].append(timed(env, lib))
for n, ts in res.items():
    us = min(ts)
    print(f"ln_quant[{n}] {rows}x{cols}: min {us:.1f} us  med {sorted(ts)[len(ts) // 2]:.1f} us  "
          f"{rows * cols * 5 / us / 1e3:.0f} GB/s", flush=True)
