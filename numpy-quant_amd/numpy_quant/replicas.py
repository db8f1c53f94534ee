"""Independent replicas across GPUs: one process per GPU.

The quantized forward has no exchange step — images are independent — so N GPUs
run N replicas of the same QModel on their own batches (weak scaling).  What is
shared is set up once:

* calibration and quantization run on rank 0 only; its QModel — every quantized
  constant in one contiguous device buffer plus every QuantizationParams (blob.py)
  — reaches the other ranks as ONE RCCL broadcast over xGMI (the blob header, a few
  hundred KB of JSON, goes over the control plane), so rank 0's model is the single
  source of truth and no other rank calibrates;
* per step, each rank's logits are gathered into rank 0's HBM over RCCL.

The control plane is control.py's TCP star (no PyTorch): rendezvous, the RCCL
unique id, the blob header, barriers and the max-over-ranks of the step time.  The
device collectives are libnqk's `nqk_comm_*` (RCCL).  With `force_device_comm`
(NQK_FORCE_COMM=1) a single process also builds a 1-rank RCCL communicator and runs the
broadcast / gather through it, so the device path runs on a 1-GPU box
(tests/test_gpu_rccl.py).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys

import numpy as np


@contextlib.contextmanager
def _stdout_to_stderr():
    """RCCL prints its version banner on stdout at communicator setup; the bench contract
    keeps stdout to one JSON line, so file descriptor 1 points at stderr meanwhile (C stdio
    flushed before it is restored)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def check_gather_sizes(rank: int, world: int, src_bytes: int, dst_bytes) -> None:
    """rank 0 gathers world * src bytes; raise before any collective is issued."""
    if rank == 0 and (dst_bytes is None or dst_bytes != world * src_bytes):
        raise ValueError(f"gather: rank 0 needs a destination of {world} x {src_bytes} bytes, got {dst_bytes}")


class ReplicaGroup:
    def __init__(self, rank: int | None = None, world: int | None = None, force_device_comm: bool | None = None):
        from .control import ControlPlane
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        if force_device_comm is None:
            force_device_comm = os.environ.get("NQK_FORCE_COMM", "0") == "1"
        self.force = bool(force_device_comm)
        self.device_comm = False
        self.ctrl = ControlPlane(self.rank, self.world)

    @property
    def use_device_comm(self) -> bool:
        return self.world > 1 or self.force

    # ------------------------------------------------------------------ control plane
    def broadcast_object(self, obj, src: int = 0):
        """A JSON-able object (or bytes) of rank `src` on every rank."""
        from .control import decode_bytes, encode_bytes
        if self.world == 1:
            return obj
        out = self.ctrl.broadcast(encode_bytes(obj) if isinstance(obj, bytes) else obj, src=src)
        return decode_bytes(out) if isinstance(out, dict) and "__bytes__" in out else out

    def barrier(self) -> None:
        self.ctrl.barrier()

    def max(self, x: float) -> float:
        """Max over ranks (the bench's step time)."""
        return self.ctrl.allreduce_max(x)

    def shared_calibration(self, calibrate):
        """Run `calibrate()` -> (vmin, vmax) on rank 0 only and hand every rank the
        same dicts (values kept as float32 bit patterns)."""
        payload = None
        if self.rank == 0:
            vmin, vmax = calibrate()
            payload = {k: (np.float32(vmin[k]).view(np.uint32).item(), np.float32(vmax[k]).view(np.uint32).item())
                       for k in vmin}
        payload = self.broadcast_object(payload)
        vmin = {k: np.uint32(a).view(np.float32) for k, (a, _) in payload.items()}
        vmax = {k: np.uint32(b).view(np.float32) for k, (_, b) in payload.items()}
        return vmin, vmax

    # ------------------------------------------------------------------ device (RCCL)
    def init_device_comm(self) -> None:
        if not self.use_device_comm or self.device_comm:
            return
        from . import _lib
        uid = (ctypes.c_char * 128)()
        if self.rank == 0:
            with _stdout_to_stderr():
                _lib.call("nqk_comm_unique_id", uid)
        raw = self.broadcast_object(bytes(uid))
        uid = (ctypes.c_char * 128).from_buffer_copy(raw)
        with _stdout_to_stderr():
            _lib.call("nqk_comm_init", uid, self.world, self.rank)
        self.device_comm = True

    def broadcast_qmodel(self, model, qmodel=None):
        """Rank 0 passes its QModel; every rank returns (qmodel, payload bytes): rank 0
        its own, the others one built on `model`'s graph from rank 0's blob, received
        with a single ncclBroadcast of the packed payload.  Forced device comm at world 1:
        the packed blob goes through a 1-rank ncclBroadcast and the returned QModel is the
        one attached to it (the device path of the other ranks, run on one GPU)."""
        if not self.use_device_comm:
            return qmodel, 0
        from . import _lib, blob
        from .device import DeviceArray
        if self.rank == 0 and qmodel is None:
            raise ValueError("broadcast_qmodel: rank 0 must supply its QModel")
        self.init_device_comm()
        header = payload = None
        if self.rank == 0:
            header, payload = blob.pack(qmodel)
        header = self.broadcast_object(header)
        n = int(header["payload_bytes"])
        if self.rank != 0:
            payload = DeviceArray((max(n, 1),), np.uint8)
        if n:
            _lib.call("nqk_comm_bcast", payload.vp, n, 0)
        _lib.call("nqk_sync")
        if self.rank == 0 and self.world > 1:
            return qmodel, n
        return blob.attach(model, header, payload), n

    def broadcast_constants(self, qmodel) -> int:
        """Broadcast every device-resident constant of `qmodel` from rank 0, one
        collective per constant (kept for models built on every rank; bench.py uses
        broadcast_qmodel's single blob broadcast)."""
        if not self.use_device_comm:
            return 0
        from . import _lib
        self.init_device_comm()
        nbytes = 0
        for v in qmodel.values:
            if v.__class__.__name__ != "Constant":
                continue
            dev = getattr(getattr(v, "data", None), "dev", None)
            if dev is not None and dev.nbytes:
                _lib.call("nqk_comm_bcast", dev.vp, dev.nbytes, 0)
                nbytes += dev.nbytes
        _lib.call("nqk_sync")
        return nbytes

    def gather(self, src, dst=None) -> None:
        """Gather each rank's `src` DeviceArray into rank 0's `dst` [world, *src.shape]."""
        if not self.use_device_comm or (self.world == 1 and dst is None):
            return
        from . import _lib
        check_gather_sizes(self.rank, self.world, src.nbytes, None if dst is None else dst.nbytes)
        self.init_device_comm()
        _lib.call("nqk_comm_gather", src.vp, dst.vp if self.rank == 0 else None, src.nbytes, 0)

    def close(self) -> None:
        if self.device_comm:
            from . import _lib
            _lib.call("nqk_comm_destroy")
            self.device_comm = False
        self.ctrl.close()
