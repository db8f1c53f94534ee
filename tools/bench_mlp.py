#!/usr/bin/env python
"""BASELINE configs[1]: mlp.onnx int8 on one MI355X, batch 4096 synthetic float32 inputs
(U[-1.2, 1.2], seed 4096), calibrated on the reference's make_circles(100) X
(tests/golden/mlp.npz).  Prints one JSON line: samples/s of QModel.__call__ with the
inputs resident in HBM (the node loop: 4 nodes, launch-bound at this size)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "numpy-quant_amd"), ROOT):
    sys.path.insert(0, p)
from numpy_quant import _lib  # noqa: E402
from numpy_quant.device import sync  # noqa: E402
from numpy_quant.model import Model  # noqa: E402
from numpy_quant.tensor import FTensor  # noqa: E402

_lib.ensure_init()
B, steps, warmup = int(os.environ.get("MLP_B", 4096)), 200, 20
X = np.load(os.path.join(ROOT, "tests", "golden", "mlp.npz"))["X"]
x = np.random.default_rng(4096).uniform(-1.2, 1.2, size=(B, 2)).astype(np.float32)
qmodel = Model.from_onnx(os.path.join(ROOT, "numpy-quant_amd", "models", "mlp.onnx")).quantize([X], bit_width=8)
x_dev = FTensor(x)


def step():
    qmodel.set_inputs([x_dev])
    qmodel.run()


for _ in range(warmup):
    step()
sync()
t0 = time.perf_counter()
for _ in range(steps):
    step()
sync()
dt = time.perf_counter() - t0
print(json.dumps({"metric": "mlp.onnx int8 samples/s (BASELINE configs[1])", "value": round(B * steps / dt, 1),
                  "unit": "samples/s", "batch": B, "steps": steps, "ms_per_step": round(1e3 * dt / steps, 4),
                  "dtype": "int8", "data": "synthetic U[-1.2,1.2]", "executor": "node loop"}), flush=True)
