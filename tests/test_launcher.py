"""bench.py's multi-GPU launcher and the replica control plane on the CPU (gloo,
world size 2): `--gpus N` without torchrun spawns N rank processes with their own
RANK / LOCAL_RANK / WORLD_SIZE and the 127.0.0.1 rendezvous; a WORLD_SIZE that
differs from --gpus is refused instead of reporting another n_gpus; rank 0 needs a
gather destination of world x src bytes; the blob header encodes quantization
parameters with their exact values and Python types."""
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_rank_environments():
    envs = bench.rank_environments(3, 29999, base={"FOO": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
               and e["FOO"] == "1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)


def test_launcher_spawns_world2_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    by = {d["rank"]: d for d in lines}
    assert set(by) == {0, 1}
    for rk, d in by.items():
        assert d["world"] == 2 and d["local_rank"] == rk and d["seed"] == 256 + rk
        assert d["master"] == "127.0.0.1" and d["header_from"] == 0 and d["max_rank"] == 1.0


def test_dead_rank_fails_the_launch_fast():
    """A rank that exits non-zero before the rendezvous leaves rank 0 waiting on the control
    plane (600 s) — or, past the rendezvous, inside an RCCL collective; the parent must notice
    the dead rank, stop the others and exit with its status within seconds."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["NQK_DRY_RUN_EXIT_RANK"] = "1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    dt = time.monotonic() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert dt < 30, dt
    assert "rank 1 exited with status 3" in r.stderr


def test_spawn_ranks_deadline(tmp_path):
    """Every rank still running past the launcher's deadline is stopped: status 124."""
    script = tmp_path / "sleeper.py"
    script.write_text("import time\ntime.sleep(60)\n")
    rc = bench.spawn_ranks(2, [], timeout=1.0, script=str(script))
    assert rc == 124


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_gather_size_check():
    from numpy_quant.replicas import check_gather_sizes
    check_gather_sizes(0, 4, 100, 400)
    check_gather_sizes(1, 4, 100, None)
    with pytest.raises(ValueError):
        check_gather_sizes(0, 4, 100, 300)
    with pytest.raises(ValueError):
        check_gather_sizes(0, 2, 100, None)


def test_blob_qparams_and_framing(tmp_path):
    from numpy_quant import blob
    from numpy_quant.model import QuantizationParams
    cases = [QuantizationParams(np.float32(0.5), None),
             QuantizationParams(np.array(np.float32(-3e-7), dtype=np.float32), np.int64(0)),
             QuantizationParams(np.float32(1e-38), np.array(-140, dtype=np.int64)),
             QuantizationParams(np.array(np.float32(np.nan), dtype=np.float32), np.array(2**40, dtype=np.int64))]
    for p in cases:
        q = blob._dec_qp(json.loads(json.dumps(blob._enc_qp(p))))
        assert type(q.scale) is type(p.scale)
        assert np.asarray(q.scale).tobytes() == np.asarray(p.scale).tobytes()
        assert type(q.zero_point) is type(p.zero_point)
        if p.zero_point is not None:
            assert int(q.zero_point) == int(p.zero_point)
    # the header keeps the reference's exact scale types: a float64 or Python float scale is
    # refused instead of being narrowed to float32 on the way
    for bad in (np.float64(0.5), 0.5, np.array(0.5)):
        with pytest.raises(ValueError):
            blob._enc_qp(QuantizationParams(bad, None))
    header = {"version": 1, "bit_width": 8, "qparams": {}, "constants": [], "payload_bytes": 512}
    hb = blob.encode_header(header)
    head = blob.MAGIC + struct.pack("<Q", len(hb)) + hb
    head += b"\0" * ((-len(head)) % blob.ALIGN)
    path = tmp_path / "x.nqk"
    path.write_bytes(head + bytes(range(256)) * 2)
    h2, body = blob.read(path)
    assert h2 == header and body.size == 512 and body[255] == 255
    path.write_bytes(head + bytes(10))
    with pytest.raises(ValueError):
        blob.read(path)
    path.write_bytes(b"NOTABLOB" + head[8:])
    with pytest.raises(ValueError):
        blob.read(path)


def test_openblas_thread_resolution(monkeypatch):
    """kernels.openblas_threads (the thread count whose GEMV-T column split the one-row
    float products reproduce) reads what OpenBLAS reads: NQK_BLAS_THREADS, then
    OPENBLAS_NUM_THREADS, GOTO_NUM_THREADS, OMP_NUM_THREADS, else the CPU affinity; at most
    64 (the conftest fixture that pins 8 for the other tests is bypassed here)."""
    import os
    from numpy_quant import kernels
    monkeypatch.setattr(kernels, "BLAS_THREADS", None)
    for v in ("NQK_BLAS_THREADS", "OPENBLAS_NUM_THREADS", "GOTO_NUM_THREADS", "OMP_NUM_THREADS"):
        monkeypatch.delenv(v, raising=False)
    assert kernels.openblas_threads() == max(1, min(len(os.sched_getaffinity(0)), 64))
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert kernels.openblas_threads() == 3
    monkeypatch.setenv("GOTO_NUM_THREADS", "5")
    assert kernels.openblas_threads() == 5
    monkeypatch.setenv("OPENBLAS_NUM_THREADS", "200")
    assert kernels.openblas_threads() == 64
    monkeypatch.setenv("NQK_BLAS_THREADS", "2")
    assert kernels.openblas_threads() == 2
    monkeypatch.setenv("NQK_BLAS_THREADS", "x")
    assert kernels.openblas_threads() == 64
