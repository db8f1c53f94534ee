"""The packed quantized-model blob: every quantized constant of a QModel and every
value's QuantizationParams in one contiguous buffer.

The reference's QModel lives only in memory (numpy_quant/model.py:454-565); its state
is `quant_params` (model.py:441-442) plus the quantized Constants that Model.quantize
creates (model.py:357-365 weights, :383-389 Gemm biases, :395-415 Add biases).  This
module serialises exactly that state, so

  * `QModel.save(path)` / `Model.load_quantized(path)` skip calibration and weight
    quantization on reload (the graph still comes from the ONNX file), and
  * N replicas receive rank 0's model as ONE RCCL broadcast of one device buffer
    (replicas.py), instead of one collective per constant.

Layout (little endian):
    b"NQKBLOB1" | u64 header bytes | header (UTF-8 JSON) | zero pad to 256 | payload
The payload holds each constant's device bytes (its narrow storage: int8 for bit
widths <= 8, int4 weights as int8 values in [-8, 7]) at a 256-byte aligned offset.
Header: {"version", "bit_width", "qparams": {name: [scale f32 bits, scale kind, zp kind,
zp]}, "constants": [{"name", "dtype", "shape", "bit_width", "offset", "nbytes"}],
"payload_bytes"}.  Scale kind 0 = np.float32 scalar, 1 = 0-d ndarray; zp kind 0 = None,
1 = np.int64 scalar, 2 = 0-d int64 ndarray (the reference's quant_parameters returns
each of these in some case, numpy_quantization.py:7-21; kept so reloaded parameters
are the same Python objects as the calibrated ones).
"""
from __future__ import annotations

import ctypes
import json
import struct
from typing import Dict, Tuple

import numpy as np

from . import _lib
from .device import DeviceArray

MAGIC = b"NQKBLOB1"
ALIGN = 256


def _enc_qp(p) -> list:
    s = p.scale
    # the header keeps the reference's exact types (np.float32 scalar or 0-d f32 array):
    # anything else would come back narrowed to float32, a different Python object
    if not ((isinstance(s, np.floating) and s.dtype == np.float32) or
            (isinstance(s, np.ndarray) and s.dtype == np.float32 and s.ndim == 0)):
        raise ValueError(f"blob: scale {s!r} ({type(s).__name__}) is not a float32 scalar")
    skind = 0 if isinstance(s, np.floating) else 1
    bits = int(np.asarray(s, dtype=np.float32).view(np.uint32))
    z = p.zero_point
    if z is None:
        return [bits, skind, 0, 0]
    zkind = 1 if isinstance(z, np.integer) else 2
    return [bits, skind, zkind, int(np.asarray(z))]


def _dec_qp(e):
    from .model import QuantizationParams
    bits, skind, zkind, zp = e
    f = np.uint32(bits).view(np.float32)
    scale = np.float32(f) if skind == 0 else np.array(f, dtype=np.float32)
    if zkind == 0:
        z = None
    elif zkind == 1:
        z = np.int64(zp)
    else:
        z = np.array(zp, dtype=np.int64)
    return QuantizationParams(scale, z)


def pack(qmodel) -> Tuple[dict, DeviceArray]:
    """(header, payload): the payload is one device buffer holding every quantized
    constant of `qmodel` (device-to-device copies, no host round trip)."""
    from .model import Constant
    from .tensor import QTensor
    consts = []
    off = 0
    for v in qmodel.values:
        if not isinstance(v, Constant):
            continue
        t = v.data
        if not isinstance(t, QTensor) or t._bias is not None:
            raise ValueError(f"blob: constant {v.name} is not a plain quantized tensor")
        consts.append((v.name, t, off))
        off += (t.dev.nbytes + ALIGN - 1) // ALIGN * ALIGN
    payload = DeviceArray((max(off, 1),), np.uint8)
    entries = []
    for name, t, o in consts:
        if t.dev.nbytes:
            _lib.call("nqk_memcpy_d2d", ctypes.c_void_p(payload.ptr + o), t.dev.vp, t.dev.nbytes)
        entries.append({"name": name, "dtype": t.dev.dtype.str, "shape": list(t.dev.shape),
                        "bit_width": int(t.bit_width), "offset": o, "nbytes": t.dev.nbytes})
    header = {"version": 1, "bit_width": int(qmodel.bit_width),
              "qparams": {k: _enc_qp(p) for k, p in qmodel.quant_params.items()},
              "constants": entries, "payload_bytes": off}
    return header, payload


def constants_from(header: dict, payload: DeviceArray) -> Dict[str, "QTensor"]:
    """QTensor views into `payload` for every constant of the header (no copies)."""
    from .tensor import QTensor
    qps = header["qparams"]
    out = {}
    need = header["payload_bytes"]
    if payload.nbytes < need:
        raise ValueError(f"blob payload holds {payload.nbytes} bytes, the header needs {need}")
    for e in header["constants"]:
        dt = np.dtype(e["dtype"])
        shape = tuple(e["shape"])
        if e["offset"] % ALIGN or e["offset"] + e["nbytes"] > need or \
                int(np.prod(shape, dtype=np.int64)) * dt.itemsize != e["nbytes"]:
            raise ValueError(f"blob: bad extent for constant {e['name']}")
        view = DeviceArray(shape, dt, payload.block, payload.ptr + e["offset"])
        p = _dec_qp(qps[e["name"]])
        t = QTensor(view, e["bit_width"], p.scale, p.zero_point)
        t._is_weight = True
        out[e["name"]] = t
    return out


def qparams_from(header: dict) -> dict:
    return {k: _dec_qp(e) for k, e in header["qparams"].items()}


def attach(model, header: dict, payload: DeviceArray):
    """The QModel of `model`'s graph with the blob's parameters and constants (the
    graph rewrite of Model.quantize, model.py:428-442, without calibration and without
    re-quantizing any constant)."""
    if header.get("version") != 1:
        raise ValueError(f"unsupported blob version {header.get('version')}")
    qp = qparams_from(header)
    consts = constants_from(header, payload)
    return model._rewrite(header["bit_width"], lambda value, asym: qp[value.name], constants=consts)


def encode_header(header: dict) -> bytes:
    return json.dumps(header, separators=(",", ":")).encode()


def save(qmodel, path) -> int:
    """Write the blob file; returns its size in bytes."""
    header, payload = pack(qmodel)
    hb = encode_header(header)
    head = MAGIC + struct.pack("<Q", len(hb)) + hb
    head += b"\0" * ((-len(head)) % ALIGN)
    host = payload.to_host()[:header["payload_bytes"]]
    with open(path, "wb") as f:
        f.write(head)
        f.write(host.tobytes())
    return len(head) + host.nbytes


def read(path) -> Tuple[dict, np.ndarray]:
    """(header, host payload bytes) of a blob file; validates the framing."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != MAGIC:
        raise ValueError(f"{path}: not an NQK blob")
    (hl,) = struct.unpack("<Q", data[8:16])
    header = json.loads(data[16:16 + hl].decode())
    start = (16 + hl + ALIGN - 1) // ALIGN * ALIGN
    body = np.frombuffer(data, dtype=np.uint8, offset=start)
    if body.size != header["payload_bytes"]:
        raise ValueError(f"{path}: payload is {body.size} bytes, header says {header['payload_bytes']}")
    return header, body


def load(model, path):
    """QModel of `model`'s graph from a blob file (one H2D copy of the payload)."""
    header, body = read(path)
    payload = DeviceArray.from_host(body if body.size else np.zeros(1, np.uint8))
    return attach(model, header, payload)
