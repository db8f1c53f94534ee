#!/usr/bin/env python
"""Rounding-filter exact-path entries of the persistent projection GEMM in the bench's own
forward (ViT-Base int8 B=256, bench.py's calibration and inputs), with a diagnostic build
(-DNQK_PG_DIAG=64, tools/pg_diag.sh) copied over the library: entries per launch against
the epilogue steps (16 elements x 64 lanes) of each launch."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "numpy-quant_amd"), ROOT):
    sys.path.insert(0, p)
import bench  # noqa: E402
from numpy_quant import _lib  # noqa: E402
from numpy_quant import kernels as K  # noqa: E402
from numpy_quant.replicas import ReplicaGroup  # noqa: E402
from numpy_quant.tensor import FTensor  # noqa: E402

_lib.ensure_init(0)
lib = _lib.load()
fn = lib.nqk_pg_diag_slow
fn.restype = ctypes.c_ulonglong
group = ReplicaGroup()
model, qmodel = bench.build_vit(256, 8, group)
x = np.random.default_rng(256).standard_normal((256, 3, 224, 224)).astype(np.float32)
xd = FTensor(x)
qmodel([xd])
qmodel._plan.split = False
fn(1)
qmodel.set_inputs([xd])
qmodel.run()
_lib.call("nqk_sync")
n = fn(1)
M = 256 * 197
steps = 12 * (M * 2304 + M * 3072) / 1024  # QKV + GELU epilogue steps of one forward
print(f"exact-path entries per forward: {n} of {steps:.0f} QKV + GELU epilogue steps ({100 * n / steps:.2f} %)")
group.close()
