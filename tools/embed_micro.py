#!/usr/bin/env python
"""Patch-embedding timing at ViT-Base B = 256 (round 6): nqk_embed_q of several builds of
libnqk.so side by side in ONE process, interleaved rounds (EMB_LIBS=name=path,... from
tools/diag_build.sh; EMB_ENV="name:VAR=val;..." per-variant environment of the main build)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import DeviceArray  # noqa: E402

_lib.ensure_init()
libs = {"main": _lib.load()}
for item in filter(None, os.environ.get("EMB_LIBS", "").split(",")):
    name, path = item.split("=", 1)
    lib = ctypes.CDLL(os.path.abspath(path))
    for fname, argt in _lib.SIGNATURES.items():
        getattr(lib, fname).argtypes = argt
        getattr(lib, fname).restype = ctypes.c_int
    assert lib.nqk_init(0) == 0
    libs[name] = lib
envs = {}
for item in filter(None, os.environ.get("EMB_ENV", "").split(";")):
    name, kv = item.split(":", 1)
    envs[name] = dict(x.split("=", 1) for x in kv.split(","))
B, N = int(os.environ.get("EMB_B", 256)), 768
rng = np.random.default_rng(0)
q = DeviceArray.from_host(rng.integers(-128, 128, size=(B, 3, 224, 224), dtype=np.int8))
wt = DeviceArray.from_host((0.02 * rng.standard_normal((N, 768))).astype(np.float32))
bias = DeviceArray.from_host(rng.standard_normal(N).astype(np.float32))
cls = DeviceArray.from_host(rng.standard_normal(N).astype(np.float32))
pos = DeviceArray.from_host(rng.standard_normal((197, N)).astype(np.float32))
out = DeviceArray((B, 197, N), np.float32)
REPS, ROUNDS = int(os.environ.get("EMB_REPS", 10)), int(os.environ.get("EMB_ROUNDS", 4))
variants = [(n, l, {}) for n, l in libs.items()] + [(n, libs["main"], e) for n, e in envs.items()]
res = {n: [] for n, _, _ in variants}
for _ in range(ROUNDS):
    for name, lib, env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        call = lambda: lib.nqk_embed_q(q.vp, 0.0125, -3, wt.vp, bias.vp, cls.vp, pos.vp, out.vp, B, 3, 224, 224, 16, 16, N)
        assert call() == 0
        lib.nqk_sync()
        t0 = time.perf_counter()
        for _ in range(REPS):
            call()
        lib.nqk_sync()
        res[name].append((time.perf_counter() - t0) / REPS * 1e6)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
flops = 2 * B * 196 * 768 * N
for name, ts in res.items():
    print(f"embed[{name}] B={B}: min {min(ts):7.1f} us  med {sorted(ts)[len(ts) // 2]:7.1f} us  "
          f"{flops / min(ts) / 1e6:6.1f} TFLOP/s", flush=True)
