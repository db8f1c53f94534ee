"""Independent replicas across GPUs: one process per GPU.

The quantized forward has no exchange step — images are independent — so N GPUs
run N replicas of the same QModel on their own batches (weak scaling).  What is
shared is set up once:

* calibration runs on rank 0 only; its per-value (min, max) are broadcast over the
  control plane, so every rank derives bit-identical QuantizationParams
  (numpy_quantization.quant_parameters is deterministic host arithmetic);
* the quantized constants (packed int8 weights, int64/f32 biases) are broadcast
  from rank 0's HBM over RCCL (xGMI) before the plan is compiled, so rank 0's
  weights are the single source of truth;
* per step, each rank's logits are gathered into rank 0's HBM over RCCL.

The control plane is torch.distributed with the gloo backend (CPU): rendezvous,
the RCCL unique id, barriers and the max-over-ranks of the step time.  The device
collectives are libnqk's `nqk_comm_*` (RCCL), never torch tensors.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np


class ReplicaGroup:
    def __init__(self, rank: int | None = None, world: int | None = None, init_process_group: bool = True):
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        self.device_comm = False
        if self.world > 1:
            import torch.distributed as dist
            if init_process_group and not dist.is_initialized():
                dist.init_process_group("gloo", init_method="env://")
            self.dist = dist

    # ------------------------------------------------------------------ control plane
    def broadcast_object(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        box = [obj if self.rank == src else None]
        self.dist.broadcast_object_list(box, src=src)
        return box[0]

    def barrier(self) -> None:
        if self.world > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        """Max over ranks (the bench's step time)."""
        if self.world == 1:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

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
        if self.world == 1 or self.device_comm:
            return
        from . import _lib
        uid = (ctypes.c_char * 128)()
        if self.rank == 0:
            _lib.call("nqk_comm_unique_id", uid)
        raw = self.broadcast_object(bytes(uid))
        uid = (ctypes.c_char * 128).from_buffer_copy(raw)
        _lib.call("nqk_comm_init", uid, self.world, self.rank)
        self.device_comm = True

    def broadcast_constants(self, qmodel) -> int:
        """Broadcast every device-resident constant of `qmodel` from rank 0 (call
        before QModel.compile(), which packs weights from these buffers)."""
        if self.world == 1:
            return 0
        from . import _lib
        self.init_device_comm()
        nbytes = 0
        for v in qmodel.values:
            dev = getattr(getattr(v, "data", None), "dev", None)
            if v.__class__.__name__ == "Constant" and dev is not None and dev.nbytes:
                _lib.call("nqk_comm_bcast", dev.vp, dev.nbytes, 0)
                nbytes += dev.nbytes
        _lib.call("nqk_sync")
        return nbytes

    def gather(self, src, dst=None) -> None:
        """Gather each rank's `src` DeviceArray into rank 0's `dst` [world, *src.shape]."""
        if self.world == 1:
            return
        from . import _lib
        if self.rank == 0 and (dst is None or dst.nbytes != self.world * src.nbytes):
            raise ValueError("gather: rank 0 needs a destination of world * src bytes")
        _lib.call("nqk_comm_gather", src.vp, dst.vp if self.rank == 0 else None, src.nbytes, 0)

    def close(self) -> None:
        if self.device_comm:
            from . import _lib
            _lib.call("nqk_comm_destroy")
            self.device_comm = False
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()
