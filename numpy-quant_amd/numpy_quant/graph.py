"""One QModel forward captured as a hipGraph and replayed with a single launch.

Small graphs are launch-bound: BASELINE configs[1] (mlp.onnx, 4 nodes) spends its
time in the Python node loop and the per-kernel launch cost, not on the GPU.  The
reference has no counterpart (its forward is numpy, model.py:486-565); this is an
extension beside `QModel.__call__`, with the same results.

Lifetime rules (why replay is safe):
  * the forward is run once eagerly first, so weight packs, the dequantized-constant
    cache and the fused plan's workspaces exist before capture;
  * the graph owns a private fused plan when the model is compiled, so the model's own
    plan may later run other batch sizes without freeing buffers the graph reads;
  * every block allocated during capture is held by the graph (the pool's capture
    list), so no buffer the graph writes is handed to anyone else while it lives;
  * replay copies the new inputs into the captured input buffers and returns the
    captured output buffers, which the next replay overwrites.  The qmodel's own
    values alias the graph's buffers after capture: every replay overwrites them,
    until the model's next eager or plan run assigns fresh ones.
  * host state read while capturing (epilogue parameters, shapes, scales) is frozen
    into the graph; kernel timers (kernels.TIMER) would be too, so capture refuses
    to run while one is active.
Integer (int64) model inputs are host tensors in this design and would be baked into
the graph, so they are refused.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Union

import numpy as np

from . import _lib
from .device import POOL, DeviceArray, sync
from .tensor import FTensor


class DeviceGraph:
    """`DeviceGraph(qmodel, example_inputs)`; then `g(inputs)` (host arrays out, as
    `QModel.__call__`) or `g.run_device(inputs)` (the captured output tensors)."""

    def __init__(self, qmodel, example_inputs: Sequence[Union[np.ndarray, FTensor]]):
        _lib.ensure_init()
        from . import kernels as KM
        if KM.TIMER is not None:
            raise RuntimeError("DeviceGraph: kernels.TIMER is active; its events would be frozen into the graph")
        self.q = qmodel
        self.staging: List[FTensor] = []
        for a in example_inputs:
            if isinstance(a, FTensor):
                self.staging.append(FTensor(a.dev.copy()))
            elif isinstance(a, np.ndarray) and a.dtype == np.float32:
                self.staging.append(FTensor(np.ascontiguousarray(a)))
            else:
                raise ValueError("DeviceGraph: float32 inputs only (int64 inputs are host tensors)")
        self.plan = None
        if qmodel._plan is not None or (qmodel.fuse and not qmodel.keep_values):
            from .plan import compile_plan
            self.plan = compile_plan(qmodel)
        self.exec = ctypes.c_void_p()
        self.outs: List[FTensor] = []
        self.blocks = []
        saved = qmodel._plan
        qmodel._plan = self.plan
        try:
            self._forward()                # eager warm-up: workspaces, packs, caches
            sync()
            self.deq_cache = dict(qmodel._deq_cache)
            POOL.capture = []
            _lib.call("nqk_graph_begin")
            try:
                outs = self._forward()
            except BaseException:
                _lib.call("nqk_graph_abort")
                raise
            _lib.call("nqk_graph_end", ctypes.byref(self.exec))
            self.outs = outs
        finally:
            if POOL.capture is not None:
                self.blocks, POOL.capture = POOL.capture, None
            qmodel._plan = saved

    def _forward(self) -> List[FTensor]:
        self.q.set_inputs(self.staging)
        self.q.run(eager=self.plan is None)
        return self.q.outputs_device()

    def _load(self, inputs) -> None:
        if len(inputs) != len(self.staging):
            raise ValueError(f"DeviceGraph: {len(self.staging)} inputs expected, got {len(inputs)}")
        for a, s in zip(inputs, self.staging):
            shape = tuple(a.dev.shape) if isinstance(a, FTensor) else tuple(np.shape(a))
            if shape != s.dev.shape:
                raise ValueError(f"DeviceGraph: input shape {shape} differs from the captured {s.dev.shape}")
            if isinstance(a, FTensor):
                _lib.call("nqk_memcpy_d2d", s.dev.vp, a.dev.vp, s.dev.nbytes)
            else:
                a = np.ascontiguousarray(a, dtype=np.float32)
                _lib.call("nqk_memcpy_h2d", s.dev.vp, a.ctypes.data_as(ctypes.c_void_p), s.dev.nbytes)

    def run_device(self, inputs) -> List[FTensor]:
        """Replay on device-resident (or host) inputs; returns the captured outputs."""
        if not self.exec:
            raise RuntimeError("DeviceGraph: destroyed")
        self._load(inputs)
        _lib.call("nqk_graph_launch", self.exec)
        for o in self.outs:
            o._host = None
        return self.outs

    def __call__(self, inputs) -> List[np.ndarray]:
        return [o.dev.to_host() for o in self.run_device(inputs)]

    def destroy(self) -> None:
        if self.exec:
            sync()
            _lib.call("nqk_graph_destroy", self.exec)
            self.exec = ctypes.c_void_p()
        self.blocks, self.outs, self.plan, self.deq_cache = [], [], None, {}

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
