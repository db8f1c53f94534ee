"""Multi-process replicas on the CPU: world_size 2 over the TCP control plane.

Covers the control plane of bench.py's N > 1 path — rank-0 calibration shared with
every replica (bit-identical quantization parameters on all ranks), the RCCL
unique-id exchange (a 128-byte object broadcast), barriers and the max-over-ranks
of the step time.  The RCCL device collectives themselves need GPUs.
"""
import os
import socket

import numpy as np
import pytest
import multiprocessing as mp

from numpy_quant.numpy_quantization import quant_parameters
from numpy_quant.replicas import ReplicaGroup


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _free_ports(n):
    """n distinct free ports (all sockets held open while probing)."""
    socks = [socket.socket() for _ in range(n)]
    try:
        for s in socks:
            s.bind(("127.0.0.1", 0))
        return [s.getsockname()[1] for s in socks]
    finally:
        for s in socks:
            s.close()


def _worker(rank, world, port, q, ctrl_port=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if ctrl_port is not None:  # a separately probed free port (MASTER_PORT + 1 may be taken)
        os.environ["NQK_CTRL_PORT"] = str(ctrl_port)
    try:
        g = ReplicaGroup()
        calls = []

        def calibrate():  # rank-dependent: only rank 0's result may survive
            calls.append(rank)
            rng = np.random.default_rng(100 + rank)
            names = [f"v{i}" for i in range(50)]
            lo = rng.standard_normal(50).astype(np.float32) - 1
            hi = rng.standard_normal(50).astype(np.float32) + 1
            lo[3] = np.float32(-0.0)
            hi[7] = np.float32(1e-38)  # keeps subnormal-adjacent bit patterns
            return dict(zip(names, lo)), dict(zip(names, hi))

        vmin, vmax = g.shared_calibration(calibrate)
        params = {}
        for k in sorted(vmin):
            for bw in (4, 8):
                for asym in (False, True):
                    s, z = quant_parameters(vmin[k], vmax[k], bit_width=bw, asymmetric=asym)
                    params[(k, bw, asym)] = (np.asarray(s).view(np.uint32).item(),
                                             None if z is None else int(z))
        bits = {k: (np.float32(vmin[k]).view(np.uint32).item(), np.float32(vmax[k]).view(np.uint32).item())
                for k in vmin}
        uid = g.broadcast_object(bytes(range(128)) if rank == 0 else None)
        g.barrier()
        mx = g.max(1.5 + rank)
        q.put((rank, calls, bits, params, uid, mx, all(isinstance(v, np.float32) for v in vmin.values())))
        g.close()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, "error", repr(e)))


def test_replica_control_plane_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, ctrl = _free_ports(2)
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, ctrl)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            item = q.get(timeout=120)
            res[item[0]] = item
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r][1] != "error", res[r]
    r0, r1 = res[0], res[1]
    assert r0[1] == [0] and r1[1] == []              # calibration ran on rank 0 only
    assert r0[2] == r1[2]                            # identical (min, max) bit patterns
    assert r0[3] == r1[3]                            # identical quantization parameters
    assert r0[4] == r1[4] == bytes(range(128))       # RCCL unique-id exchange
    assert r0[5] == r1[5] == 2.5                     # max over ranks
    assert r0[6] and r1[6]


def test_replica_group_single_process():
    g = ReplicaGroup(rank=0, world=1)
    assert g.broadcast_object(5) == 5
    assert g.max(3.0) == 3.0
    vmin, vmax = g.shared_calibration(lambda: ({"a": np.float32(-1)}, {"a": np.float32(2)}))
    assert vmin["a"] == np.float32(-1) and vmax["a"] == np.float32(2)
    g.barrier()
    g.close()
