#!/usr/bin/env python
"""Projection-GEMM timing at the ViT-Base B=256 shapes (round 3): the persistent 16x16x64
kernel (k_pg) of several builds of libnqk.so side by side in ONE process (interleaved
rounds; MI355X_MICROARCH.md: never rank builds timed in different processes), plus the
round-2 kernels (k_proj / k_qgemm_big) of the main build.

  PGM_LIBS=name=path,...   extra builds (tools/pg_diag.sh) loaded next to the main one
  PGM_SHAPES=qkv,out,up,down
  PGM_ENV="name:VAR=val;..." per-variant environment of the main build (e.g. stagger)
Timing: host wall clock over REPS back-to-back launches after a device sync (the kernels
run 50-250 us; the launch cost is hidden behind the queue)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import DeviceArray  # noqa: E402
from numpy_quant.plan import _pack_b, _pack_pg  # noqa: E402

_lib.ensure_init()
main = _lib.load()
M = int(os.environ.get("GM_M", 256 * 197))
REPS = int(os.environ.get("PGM_REPS", 20))
ROUNDS = int(os.environ.get("PGM_ROUNDS", 3))
shapes = {"qkv": (2304, 768, 0), "out": (768, 768, 3), "up": (3072, 768, 4), "down": (768, 3072, 3),
          "tqkv": (576, 192, 0), "tup": (768, 192, 4)}  # (t*: ViT-Ti, K = 192)
sel = os.environ.get("PGM_SHAPES", "qkv,out,up,down").split(",")
rng = np.random.default_rng(0)

libs = {"main": main}
for item in filter(None, os.environ.get("PGM_LIBS", "").split(",")):
    name, path = item.split("=", 1)
    lib = ctypes.CDLL(os.path.abspath(path))
    for fname, argt in _lib.SIGNATURES.items():
        fn = getattr(lib, fname)
        fn.argtypes = argt
        fn.restype = ctypes.c_int
    assert lib.nqk_init(0) == 0
    libs[name] = lib
envs = {}
for item in filter(None, os.environ.get("PGM_ENV", "").split(";")):
    name, kv = item.split(":", 1)
    envs[name] = dict(x.split("=", 1) for x in kv.split(","))


def sync_all():
    for lib in libs.values():
        lib.nqk_sync()


def setup(name):
    N, K, epi = shapes[name]
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt0 = DeviceArray.from_host(rng.integers(-128, 128, size=(N, K), dtype=np.int8))
    bt, kind = _pack_b(bt0, 8)
    pg = _pack_pg(bt0, 8, 1 if epi == 3 else 0)
    col = DeviceArray.from_host(np.zeros(N, np.int64))
    colterm = DeviceArray.from_host(np.zeros(N, np.int32))
    bias = DeviceArray.from_host((0.01 * rng.standard_normal(N)).astype(np.float32))
    resid = DeviceArray.from_host(rng.standard_normal((M, N)).astype(np.float32))
    out = DeviceArray((M, N), np.float32)
    D = N // 3 if epi == 0 else 768  # the model width (QKV: N = 3 D)
    # QKV writes the head layout of whole images: ceil(M / 197) of them
    outs = [DeviceArray((-(-M // 197) * 197, D), np.int8) for _ in range(3)] if epi == 0 else [out]
    e = _lib.Epilogue()
    e.zp_flags, e.bit_width = _lib.ZP_COL, 8
    e.group_cols = D if epi == 0 else (1 << 30)
    e.tokens, e.heads, e.hdim = 197, D // 64, 64
    e.zpa, e.col, e.colterm, e.col_absmax = 3, col.ptr, colterm.ptr, 1
    for g in range(3):
        e.s_acc[g] = 7e-6 * (768 / K) ** 0.5
        e.s_out[g] = 0.0165 if epi == 4 else 0.03
        e.zp_out[g] = -118 if epi == 4 else -2
        e.out[g] = outs[min(g, len(outs) - 1)].ptr
    if epi == 4:
        h = DeviceArray((M, N), np.int8)
        outs = [h]
        e.out[0] = h.ptr
    e.bias, e.resid = bias.ptr, resid.ptr
    e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
    e.b_packed = kind
    glut = None
    if epi == 4:  # the GELU table of these output parameters (round 4: the "glut" variant)
        lut = DeviceArray((8192,), np.uint8)
        kk = (ctypes.c_float * 5)()
        nn = ctypes.c_int32(0)
        _lib.call("nqk_gelu_lut_build", e.s_out[0], e.zp_out[0], 8, e.div, e.add1, e.mul2, lut.vp, kk, ctypes.byref(nn))
        print(f"  GELU table: {nn.value} entries", flush=True)
        if nn.value > 0:
            glut = (lut, kk, nn.value)
    keep = (a, bt0, bt, pg, col, colterm, bias, resid, out, outs, glut)
    return N, K, epi, a, bt, pg, e, keep


def timed(lib, epi, a, bt, N, K, e, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        args = (epi, a.vp, bt.vp, 1, M, N, K, K, K, None, 0, 0, ctypes.byref(e))
        rc = lib.nqk_qgemm_fused(*args)
        if rc != 0:
            lib.nqk_last_error.restype = ctypes.c_char_p
            raise RuntimeError(f"nqk_qgemm_fused rc={rc}: {lib.nqk_last_error().decode()}")
        sync_all()
        diag = getattr(lib, "nqk_pg_diag_slow", None) if hasattr(lib, "nqk_pg_diag_slow") else None
        if diag is not None:
            diag.restype = ctypes.c_ulonglong
            diag(1)
        t0 = time.perf_counter()
        for _ in range(REPS):
            lib.nqk_qgemm_fused(*args)
        lib.nqk_sync()
        dt = (time.perf_counter() - t0) / REPS * 1e6
        if diag is not None:
            steps = M * N / 1024
            print(f"  exact-path entries per launch: {diag(0) / REPS:.0f} of {steps:.0f} epilogue steps", flush=True)
        return dt
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


print("libs:", list(libs), "envs:", envs, flush=True)
for name in sel:
    N, K, epi, a, bt, pg, e, keep = setup(name)
    ops = 2.0 * M * N * K
    variants = []
    for lname, lib in libs.items():
        variants.append((f"pg:{lname}", lib, {}, True))
    for vname, env in envs.items():  # (PGM_ENV variants: of every build)
        for lname, lib in libs.items():
            variants.append((f"pg:{vname}" if lname == "main" else f"pg:{lname}:{vname}", lib, env, True))
    if keep[-1] is not None:
        for lname, lib in libs.items():
            variants.append(("glut" if lname == "main" else f"glut:{lname}", lib, {}, "glut"))
            for vname, env in envs.items():
                variants.append((f"glut:{vname}" if lname == "main" else f"glut:{lname}:{vname}", lib, env, "glut"))
    variants.append(("r02", main, {"NQK_PROJ_GELU": "1"} if epi == 4 else {}, False))
    res = {v[0]: [] for v in variants}
    for _ in range(ROUNDS):
        for vname, lib, env, use_pg in variants:
            e.bt_pg = pg.ptr if use_pg else None
            glut = keep[-1] if use_pg == "glut" else None
            e.gelu_lut, e.lut_n = (glut[0].ptr, glut[2]) if glut else (None, 0)
            if glut:
                for j in range(5):
                    e.lut_k[j] = glut[1][j]
            try:
                res[vname].append(timed(lib, epi, a, bt, N, K, e, env))
            except RuntimeError as ex:
                print(vname, ex, flush=True)
                res[vname].append(float("nan"))
    if os.environ.get("PGM_CHECK") and epi == 3:  # every build's residual output against the main build's
        out_arr, ref = keep[8], None
        for vname, lib, env, use_pg in variants:
            if use_pg is not True:
                continue
            e.bt_pg = pg.ptr
            out_arr.fill_zero()
            sync_all()
            args = (epi, a.vp, bt.vp, 1, M, N, K, K, K, None, 0, 0, ctypes.byref(e))
            assert lib.nqk_qgemm_fused(*args) == 0
            sync_all()
            h = out_arr.to_host()
            ref = h if ref is None else ref
            ok = np.array_equal(h.view(np.int32), ref.view(np.int32))
            print(f"check {name} {vname}: {'equal' if ok else 'DIFF %d' % int((h != ref).sum())}", flush=True)
    for vname, ts in res.items():
        t = min(ts)
        print(f"{name:5s} {vname:14s} M={M} N={N} K={K}: min {t:7.1f} us  med {sorted(ts)[len(ts) // 2]:7.1f} us  "
              f"{ops / t / 1e6:7.1f} TOPS ({100 * ops / t / 1e6 / 5033.2:5.1f}% of int8 peak)", flush=True)
