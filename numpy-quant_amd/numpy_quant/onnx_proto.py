"""Self-contained ONNX protobuf reader (no `onnx` package on either box).

The reference imports ONNX through the `onnx` package (numpy_quant/model.py:8-10,
57-62, 249-292: `onnx.numpy_helper.to_array`, `onnx.helper.get_attribute_value`).
Neither `onnx` nor `onnxruntime` exists in this image, so this module decodes the
protobuf wire format directly and exposes objects duck-typed like `onnx.ModelProto`
(`.graph.initializer / .input / .output / .node`, each node with `.name, .op_type,
.input, .output, .attribute`).  That keeps `Model.from_onnx(model_proto)` a drop-in.

Also provides the two ingestion passes SURVEY.md §8(c)/§8(f)3 needs for the ViT
graphs in the reference (`models/vit/*_no_weights.onnx`):
  * external-data initializers whose `.data` files are absent get deterministic
    synthetic weights (`synthetic_weights=True`), seeded per tensor name;
  * `rebatch(model, B)`: the torch export hard-codes batch 1 into int64 shape
    constants; every Constant node holding an int64 vector of length 3 or 4 with
    v[0] == 1 gets v[0] = B ("Rebatch rule").
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import Any

import numpy as np

# TensorProto.DataType -> numpy dtype (onnx.proto3 enumeration)
_ONNX_DTYPES = {
    1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32,
    7: np.int64, 9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64,
}
_NP_TO_ONNX = {np.dtype(v): k for k, v in _ONNX_DTYPES.items()}

# AttributeProto.AttributeType
ATTR_FLOAT, ATTR_INT, ATTR_STRING, ATTR_TENSOR, ATTR_GRAPH = 1, 2, 3, 4, 5
ATTR_FLOATS, ATTR_INTS, ATTR_STRINGS, ATTR_TENSORS = 6, 7, 8, 9


# ----------------------------------------------------------------------------- wire format
def _varint(buf: memoryview, pos: int) -> tuple[int, int]:
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if b < 0x80:
            return result, pos
        shift += 7


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _fields(buf: memoryview):
    """Yield (field_number, wire_type, value) for one message body."""
    pos, end = 0, len(buf)
    while pos < end:
        key, pos = _varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            val, pos = _varint(buf, pos)
        elif wt == 1:
            val = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            val = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            val = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield field, wt, val


def _packed_varints(val, wt) -> list[int]:
    if wt == 0:
        return [_signed64(val)]
    out, pos = [], 0
    while pos < len(val):
        v, pos = _varint(val, pos)
        out.append(_signed64(v))
    return out


def _packed_f32(val, wt) -> list[float]:
    if wt == 5:
        return [struct.unpack("<f", val)[0]]
    return list(np.frombuffer(bytes(val), dtype="<f4"))


# ----------------------------------------------------------------------------- messages
class TensorProto:
    """Subset of onnx.TensorProto; `to_array()` replaces onnx.numpy_helper.to_array."""
    FLOAT, INT64 = 1, 7

    def __init__(self):
        self.dims: list[int] = []
        self.data_type = 0
        self.name = ""
        self.raw_data = b""
        self.float_data: list[float] = []
        self.int32_data: list[int] = []
        self.int64_data: list[int] = []
        self.double_data: list[float] = []
        self.external_data: dict[str, str] = {}
        self.data_location = 0
        self._array: np.ndarray | None = None  # set for synthetic / rewritten tensors

    @classmethod
    def parse(cls, buf: memoryview) -> "TensorProto":
        t = cls()
        for f, wt, v in _fields(buf):
            if f == 1:
                t.dims.extend(_packed_varints(v, wt))
            elif f == 2:
                t.data_type = v
            elif f == 4:
                t.float_data.extend(_packed_f32(v, wt))
            elif f == 5:
                t.int32_data.extend(_packed_varints(v, wt))
            elif f == 7:
                t.int64_data.extend(_packed_varints(v, wt))
            elif f == 8:
                t.name = bytes(v).decode()
            elif f == 9:
                t.raw_data = bytes(v)
            elif f == 10:
                t.double_data.extend(np.frombuffer(bytes(v), "<f8") if wt == 2 else struct.unpack("<d", v))
            elif f == 13:
                k = val = ""
                for f2, _, v2 in _fields(v):
                    if f2 == 1:
                        k = bytes(v2).decode()
                    elif f2 == 2:
                        val = bytes(v2).decode()
                t.external_data[k] = val
            elif f == 14:
                t.data_location = v
        return t

    @property
    def is_external(self) -> bool:
        return self.data_location == 1

    def to_array(self, base_dir: str | None = None) -> np.ndarray:
        if self._array is not None:
            return self._array
        if self.data_type not in _ONNX_DTYPES:
            raise ValueError(f"ONNX tensor {self.name!r}: unsupported data_type {self.data_type}")
        dt = np.dtype(_ONNX_DTYPES[self.data_type])
        shape = tuple(self.dims)
        if self.is_external:
            loc = self.external_data.get("location", "")
            path = os.path.join(base_dir or ".", loc)
            if not os.path.exists(path):
                raise FileNotFoundError(f"external data for {self.name!r} not found: {path}")
            off = int(self.external_data.get("offset", 0))
            n = int(np.prod(shape, dtype=np.int64)) if shape else 1
            with open(path, "rb") as fh:
                fh.seek(off)
                raw = fh.read(n * dt.itemsize)
            return np.frombuffer(raw, dtype=dt.newbyteorder("<")).astype(dt).reshape(shape)
        if self.raw_data:
            return np.frombuffer(self.raw_data, dtype=dt.newbyteorder("<")).astype(dt).reshape(shape)
        if self.data_type == 1:
            return np.array(self.float_data, dtype=np.float32).reshape(shape)
        if self.data_type == 7:
            return np.array(self.int64_data, dtype=np.int64).reshape(shape)
        if self.data_type == 11:
            return np.array(self.double_data, dtype=np.float64).reshape(shape)
        if self.data_type in (2, 3, 4, 5, 6, 9, 10):
            arr = np.array(self.int32_data, dtype=np.int32)
            if self.data_type == 10:
                return arr.astype(np.uint16).view(np.float16).reshape(shape)
            return arr.astype(dt).reshape(shape)
        raise ValueError(f"ONNX tensor {self.name!r}: no payload")

    def set_array(self, arr: np.ndarray) -> None:
        arr = np.asarray(arr)
        self._array = arr
        self.dims = list(arr.shape)
        self.data_type = _NP_TO_ONNX[arr.dtype]
        self.data_location = 0


class AttributeProto:
    def __init__(self):
        self.name = ""
        self.type = 0
        self.f = 0.0
        self.i = 0
        self.s = b""
        self.t: TensorProto | None = None
        self.floats: list[float] = []
        self.ints: list[int] = []
        self.strings: list[bytes] = []

    @classmethod
    def parse(cls, buf: memoryview) -> "AttributeProto":
        a = cls()
        for f, wt, v in _fields(buf):
            if f == 1:
                a.name = bytes(v).decode()
            elif f == 2:
                a.f = struct.unpack("<f", v)[0]
            elif f == 3:
                a.i = _signed64(v)
            elif f == 4:
                a.s = bytes(v)
            elif f == 5:
                a.t = TensorProto.parse(v)
            elif f == 7:
                a.floats.extend(_packed_f32(v, wt))
            elif f == 8:
                a.ints.extend(_packed_varints(v, wt))
            elif f == 9:
                a.strings.append(bytes(v))
            elif f == 20:
                a.type = v
        return a


def attribute_value(a: AttributeProto) -> Any:
    """Python/numpy value of an attribute (the reference converts via
    onnx.helper.get_attribute_value + numpy_helper.to_array, model.py:57-62)."""
    if a.type == ATTR_FLOAT:
        return float(np.float32(a.f))
    if a.type == ATTR_INT:
        return int(a.i)
    if a.type == ATTR_STRING:
        return a.s
    if a.type == ATTR_TENSOR:
        return np.array(a.t.to_array())
    if a.type == ATTR_FLOATS:
        return [float(np.float32(x)) for x in a.floats]
    if a.type == ATTR_INTS:
        return list(a.ints)
    if a.type == ATTR_STRINGS:
        return list(a.strings)
    raise ValueError(f"attribute {a.name!r}: unsupported type {a.type}")


class NodeProto:
    def __init__(self):
        self.input: list[str] = []
        self.output: list[str] = []
        self.name = ""
        self.op_type = ""
        self.domain = ""
        self.attribute: list[AttributeProto] = []

    @classmethod
    def parse(cls, buf: memoryview) -> "NodeProto":
        n = cls()
        for f, _, v in _fields(buf):
            if f == 1:
                n.input.append(bytes(v).decode())
            elif f == 2:
                n.output.append(bytes(v).decode())
            elif f == 3:
                n.name = bytes(v).decode()
            elif f == 4:
                n.op_type = bytes(v).decode()
            elif f == 5:
                n.attribute.append(AttributeProto.parse(v))
            elif f == 7:
                n.domain = bytes(v).decode()
        return n


class ValueInfoProto:
    def __init__(self):
        self.name = ""
        self.elem_type = 0
        self.shape: list[int | str] = []

    @classmethod
    def parse(cls, buf: memoryview) -> "ValueInfoProto":
        vi = cls()
        for f, _, v in _fields(buf):
            if f == 1:
                vi.name = bytes(v).decode()
            elif f == 2:  # TypeProto
                for f2, _, v2 in _fields(v):
                    if f2 != 1:  # tensor_type
                        continue
                    for f3, _, v3 in _fields(v2):
                        if f3 == 1:
                            vi.elem_type = v3
                        elif f3 == 2:  # TensorShapeProto
                            for f4, _, v4 in _fields(v3):
                                if f4 != 1:
                                    continue
                                dim: int | str = "?"
                                for f5, _, v5 in _fields(v4):
                                    if f5 == 1:
                                        dim = _signed64(v5)
                                    elif f5 == 2:
                                        dim = bytes(v5).decode()
                                vi.shape.append(dim)
        return vi


class GraphProto:
    def __init__(self):
        self.node: list[NodeProto] = []
        self.name = ""
        self.initializer: list[TensorProto] = []
        self.input: list[ValueInfoProto] = []
        self.output: list[ValueInfoProto] = []
        self.value_info: list[ValueInfoProto] = []

    @classmethod
    def parse(cls, buf: memoryview) -> "GraphProto":
        g = cls()
        for f, _, v in _fields(buf):
            if f == 1:
                g.node.append(NodeProto.parse(v))
            elif f == 2:
                g.name = bytes(v).decode()
            elif f == 5:
                g.initializer.append(TensorProto.parse(v))
            elif f == 11:
                g.input.append(ValueInfoProto.parse(v))
            elif f == 12:
                g.output.append(ValueInfoProto.parse(v))
            elif f == 13:
                g.value_info.append(ValueInfoProto.parse(v))
        return g


class ModelProto:
    def __init__(self):
        self.ir_version = 0
        self.producer_name = ""
        self.graph = GraphProto()
        self.opset_import: list[tuple[str, int]] = []
        self.base_dir: str | None = None

    @classmethod
    def parse(cls, data: bytes) -> "ModelProto":
        m = cls()
        for f, _, v in _fields(memoryview(data)):
            if f == 1:
                m.ir_version = v
            elif f == 2:
                m.producer_name = bytes(v).decode()
            elif f == 7:
                m.graph = GraphProto.parse(v)
            elif f == 8:
                dom, ver = "", 0
                for f2, _, v2 in _fields(v):
                    if f2 == 1:
                        dom = bytes(v2).decode()
                    elif f2 == 2:
                        ver = v2
                m.opset_import.append((dom, ver))
        return m


# ----------------------------------------------------------------------------- public helpers
def synthetic_array(name: str, shape: tuple[int, ...], seed: int = 0) -> np.ndarray:
    """Deterministic stand-in for an absent external-data weight.

    N(0, 0.02) for matrices, biases, conv kernels and embeddings; 1 + N(0, 0.02)
    for LayerNorm scales (names ending in 'layernorm.weight' / 'layer_norm.weight'
    / 'ln.weight').  Seeded by crc32(name) ^ seed so that every tensor is
    independent of load order.  Never constant-valued (a constant tensor gives
    scale 0 in numpy_quantization.py:11-13).
    """
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)))
    arr = (rng.standard_normal(size=shape, dtype=np.float32) * np.float32(0.02)).astype(np.float32)
    lname = name.lower()
    if ("norm" in lname) and lname.endswith("weight"):
        arr = (arr + np.float32(1.0)).astype(np.float32)
    return arr


def load(path_or_bytes, synthetic_weights: bool = False, seed: int = 0) -> ModelProto:
    """onnx.load replacement.  With `synthetic_weights`, external-data initializers
    whose files are missing are replaced by `synthetic_array`."""
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        m = ModelProto.parse(bytes(path_or_bytes))
    else:
        with open(path_or_bytes, "rb") as fh:
            m = ModelProto.parse(fh.read())
        m.base_dir = os.path.dirname(os.path.abspath(path_or_bytes))
    for t in m.graph.initializer:
        if t.is_external:
            loc = os.path.join(m.base_dir or ".", t.external_data.get("location", ""))
            if os.path.exists(loc):
                t.set_array(t.to_array(m.base_dir))
            elif synthetic_weights:
                t.set_array(synthetic_array(t.name, tuple(t.dims), seed))
            else:
                raise FileNotFoundError(
                    f"external data for initializer {t.name!r} missing ({loc}); "
                    "pass synthetic_weights=True for seeded stand-in weights")
    return m


def to_array(t: TensorProto) -> np.ndarray:
    return t.to_array()


def rebatch(m: ModelProto, batch: int) -> int:
    """Rewrite the batch-1 int64 shape constants of a torch-exported graph
    (SURVEY.md Appendix A).  Returns the number of constants rewritten."""
    count = 0
    for node in m.graph.node:
        if node.op_type != "Constant":
            continue
        for a in node.attribute:
            if a.name != "value" or a.t is None:
                continue
            v = a.t.to_array()
            if v.dtype == np.int64 and v.ndim == 1 and v.shape[0] in (3, 4) and v[0] == 1:
                v = v.copy()
                v[0] = batch
                a.t.set_array(v)
                count += 1
    for vi in list(m.graph.input) + list(m.graph.output):
        if vi.shape and vi.shape[0] == 1:
            vi.shape[0] = batch
    return count


def redimension(m: ModelProto, width: int, heads: int, mlp: int, seed: int = 0,
                base: tuple[int, int, int] = (768, 12, 3072)) -> int:
    """Re-dimension a ViT graph exported at base = (width, heads, mlp) (the reference's
    ViT-Base/16 graphs, models/vit.py:43) to another ViT family member with the same head
    size and depth, e.g. ViT-Ti/16 = (192, 3, 768): every initializer dimension equal to
    the base width / MLP width is rewritten and its weights re-synthesized
    (`synthetic_array`, same names and seed), and the Reshape shape constants
    [b, t, heads, head_dim] / [b, t, width] follow.  Only for graphs whose weights are
    synthetic (the reference ships none).  Returns the number of tensors rewritten."""
    w0, h0, f0 = base
    if w0 // h0 != width // heads or width % heads:
        raise ValueError("redimension keeps the head size: width / heads must equal the base's")
    dmap = {w0: width, f0: mlp}
    count = 0
    for t in m.graph.initializer:
        dims = [dmap.get(int(d), int(d)) for d in t.dims]
        if dims != [int(d) for d in t.dims]:
            t.set_array(synthetic_array(t.name, tuple(dims), seed))
            count += 1
    for node in m.graph.node:
        if node.op_type != "Constant":
            continue
        for a in node.attribute:
            if a.name != "value" or a.t is None:
                continue
            v = a.t.to_array()
            if v.dtype != np.int64 or v.ndim != 1:
                continue
            if v.shape[0] == 4 and v[2] == h0 and v[3] == w0 // h0:
                v = v.copy()
                v[2] = heads
            elif v.shape[0] == 3 and v[2] == w0:
                v = v.copy()
                v[2] = width
            else:
                continue
            a.t.set_array(v)
            count += 1
    return count
