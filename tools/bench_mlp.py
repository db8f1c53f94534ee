#!/usr/bin/env python
"""BASELINE configs[1]: mlp.onnx int8 on one MI355X, batch 4096 synthetic float32 inputs
(U[-1.2, 1.2], seed 4096), calibrated on the reference's make_circles(100) X
(tests/golden/mlp.npz).  Prints one JSON line per executor: samples/s of one forward
with the inputs resident in HBM — the node loop of QModel.__call__ (4 nodes,
launch-bound at this size) and the same forward replayed as one hipGraph (graph.py)."""
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
bw = int(os.environ.get("MLP_BW", 8))
X = np.load(os.path.join(ROOT, "tests", "golden", "mlp.npz"))["X"]
x = np.random.default_rng(4096).uniform(-1.2, 1.2, size=(B, 2)).astype(np.float32)
qmodel = Model.from_onnx(os.path.join(ROOT, "numpy-quant_amd", "models", "mlp.onnx")).quantize([X], bit_width=bw)
x_dev = FTensor(x)


def node_loop():
    qmodel.set_inputs([x_dev])
    qmodel.run()


graph = qmodel.graph([x_dev])


def replay():
    graph.run_device([x_dev])


ref = qmodel([x])[0]
assert np.array_equal(graph([x])[0], ref), "graph replay differs from the node loop"
for name, step in (("node loop", node_loop), ("hipGraph replay", replay)):
    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": f"mlp.onnx int{bw} samples/s (BASELINE configs[1])", "value": round(B * steps / dt, 1),
                      "unit": "samples/s", "batch": B, "steps": steps, "ms_per_step": round(1e3 * dt / steps, 4),
                      "dtype": f"int{bw}", "data": "synthetic U[-1.2,1.2]", "executor": name}), flush=True)
