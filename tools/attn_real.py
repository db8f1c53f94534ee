#!/usr/bin/env python
"""The fused attention on the bench's own data (round 4): builds and calibrates the ViT-Base
model exactly as bench.py does, runs one B = 256 forward, then times nqk_attention_fused on
the last layer's Q / K / V (still in the plan's workspace) with that layer's quantization
parameters — for the main build and, side by side in one process, diagnostic builds
(AM_LIBS=name=path,...).  A build with NQK_ATTN_DIAG & 128 also reports how many wave-tiles
took each slow path (nqk_attn_diag_stats)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
import bench  # noqa: E402
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import DeviceArray  # noqa: E402
from numpy_quant.plan import FusedLayer, _f32, _zp  # noqa: E402
from numpy_quant.replicas import ReplicaGroup  # noqa: E402
from numpy_quant.tensor import FTensor  # noqa: E402

B = 256
_lib.ensure_init(0)
group = ReplicaGroup()
model, qmodel = bench.build_vit(B, 8, group)
x = np.random.default_rng(256).standard_normal((B, 3, 224, 224)).astype(np.float32)
qmodel([FTensor(x)])
plan = qmodel._plan
layer = [o for _, o in plan.steps if isinstance(o, FusedLayer)][-1]
w = plan.ws.bufs
m = layer.m
H, T, Dh, D = m.heads, m.tokens, m.hdim, layer.D
pq, pk, pv_ = layer.p_head["q"], layer.p_head["k"], layer.p_head["v"]
a = _lib.Attention()
a.heads, a.tokens, a.hdim, a.ld_out, a.bit_width = H, T, Dh, D, layer.bw
a.zq, a.zk = _zp(pq), _zp(pk)
a.s_qk, a.div = _f32(np.float32(pq.scale) * np.float32(pk.scale)), m.div
a.s_p, a.zp_p = _f32(layer.p_sm.scale), _zp(layer.p_sm)
a.s_pv, a.zv = _f32(np.float32(layer.p_sm.scale) * np.float32(pv_.scale)), _zp(pv_)
a.s_ctx, a.zp_ctx = _f32(layer.p_ctx.scale), _zp(layer.p_ctx)
print(f"last layer: zq {a.zq} zk {a.zk} s_qk {a.s_qk:.4g} div {a.div} s_p {a.s_p:.4g} zp_p {a.zp_p} "
      f"s_pv {a.s_pv:.4g} zv {a.zv} s_ctx {a.s_ctx:.4g} zp_ctx {a.zp_ctx}", flush=True)
q = w["q"].offset_view(0, (B * H * T, Dh))
k = w["k"].offset_view(0, (B * H * T, Dh))
v = w["v"].offset_view(0, (B * H * T, Dh))
ctx = DeviceArray((B, T, D), np.int8)
# scores of the first (image, head) on the host: the spread y - max the softmax sees
qh = q.to_host()[:T].astype(np.int64)
kh = k.to_host()[:T].astype(np.int64)
sc = ((qh - a.zq) @ (kh - a.zk).T).astype(np.float64) * a.s_qk / a.div
print(f"image 0 head 0: scores span {sc.min():.3f} .. {sc.max():.3f}; min over rows of (min - max) "
      f"{(sc.min(1) - sc.max(1)).min():.3f}", flush=True)

libs = {"main": _lib.load()}
# AM_ENV="name:VAR=val,...;..." environment variants of the main build (read by the launcher per call)
envs = {}
for item in filter(None, os.environ.get("AM_ENV", "").split(";")):
    name, kv = item.split(":", 1)
    envs[name] = dict(x.split("=", 1) for x in kv.split(","))
for item in filter(None, os.environ.get("AM_LIBS", "").split(",")):
    name, path = item.split("=", 1)
    lib = ctypes.CDLL(os.path.abspath(path))
    for fname, argt in _lib.SIGNATURES.items():
        fn = getattr(lib, fname, None)
        if fn is not None:
            fn.argtypes = argt
            fn.restype = ctypes.c_int
    assert lib.nqk_init(0) == 0
    libs[name] = lib
REPS, ROUNDS = 20, 5


def timed(lib):
    run = lambda: lib.nqk_attention_fused(q.vp, k.vp, v.vp, ctx.vp, B * H, ctypes.byref(a))  # noqa: E731
    assert run() == 0
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.nqk_event_create(ctypes.byref(e0))
    lib.nqk_event_create(ctypes.byref(e1))
    lib.nqk_event_record(e0)
    for _ in range(REPS):
        run()
    lib.nqk_event_record(e1)
    ms = ctypes.c_float()
    lib.nqk_event_elapsed(e0, e1, ctypes.byref(ms))
    lib.nqk_sync()
    return 1e3 * ms.value / REPS


variants = [(n, lib, {}) for n, lib in libs.items()] + [(f"main:{n}", libs["main"], e) for n, e in envs.items()]
res = {v[0]: [] for v in variants}
ref = None
for _ in range(ROUNDS):
    for n, lib, env in variants:
        old = {kk: os.environ.get(kk) for kk in env}
        os.environ.update(env)
        try:
            res[n].append(timed(lib))
        finally:
            for kk, vv in old.items():
                if vv is None:
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = vv
        out = ctx.to_host()
        ref = out if ref is None else ref
        if not np.array_equal(out, ref):
            print(f"{n}: context DIFFERS from main", flush=True)
for n, ts in res.items():
    print(f"attention[{n}] (bench data, last layer, B={B}): min {min(ts):.1f} us  med {sorted(ts)[len(ts) // 2]:.1f} us",
          flush=True)
    fn = getattr(libs.get(n), "nqk_attn_diag_stats", None)
    if fn is not None:
        st = (ctypes.c_ulonglong * 4)()
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fn(st, 1)
        libs[n].nqk_attention_fused(q.vp, k.vp, v.vp, ctx.vp, B * H, ctypes.byref(a))
        libs[n].nqk_sync()
        fn(st, 1)
        tiles = B * H * 7 * 7  # wave-tiles x score tiles per launch (P counters count per score tile)
        print(f"  one launch: clamped-exp wave-tiles {st[0]}, clamped-P {st[1]} (of {B * H * 7} wave row tiles); "
              f"P exact fallbacks {st[2]} (of {tiles} score tiles); context fallbacks {st[3]}", flush=True)
group.close()
