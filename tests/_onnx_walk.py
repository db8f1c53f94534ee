"""A second, independent reader of the ONNX protobuf wire format, for cross-checking
numpy_quant.onnx_proto (which the product and the fixture generator share, VERDICT r01
weak #8).  Written separately from it on purpose: a table of the few ONNX field numbers
(onnx.proto3: ModelProto.graph = 7; GraphProto node 1, initializer 5, input 11,
output 12; NodeProto input 1, output 2, name 3, op_type 4, attribute 5; AttributeProto
name 1, f 2, i 3, s 4, t 5, floats 7, ints 8, type 20; TensorProto dims 1, data_type 2,
name 8; ValueInfoProto name 1) and a generic tag walker.  It returns plain tuples."""
import struct

WIRE_VARINT, WIRE_I64, WIRE_LEN, WIRE_I32 = 0, 1, 2, 5


def _read_varint(b, i):
    shift = value = 0
    while True:
        byte = b[i]
        i += 1
        value |= (byte & 0x7F) << shift
        if byte < 0x80:
            return value, i
        shift += 7


def _walk(b):
    """[(field number, wire type, value)] of one message; LEN values as bytes."""
    out, i, n = [], 0, len(b)
    while i < n:
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == WIRE_VARINT:
            v, i = _read_varint(b, i)
        elif wt == WIRE_I64:
            v, i = b[i:i + 8], i + 8
        elif wt == WIRE_I32:
            v, i = b[i:i + 4], i + 4
        elif wt == WIRE_LEN:
            ln, i = _read_varint(b, i)
            v, i = b[i:i + ln], i + ln
        else:
            raise ValueError(f"wire type {wt}")
        out.append((num, wt, v))
    return out


def _ints(entries, num):
    vals = []
    for f, wt, v in entries:
        if f != num:
            continue
        if wt == WIRE_LEN:  # packed
            j = 0
            while j < len(v):
                x, j = _read_varint(v, j)
                vals.append(x)
        else:
            vals.append(v)
    return [x - (1 << 64) if x >= 1 << 63 else x for x in vals]


def _floats(entries, num):
    vals = []
    for f, wt, v in entries:
        if f != num:
            continue
        if wt == WIRE_LEN:
            vals.extend(struct.unpack(f"<{len(v) // 4}f", v))
        else:
            vals.append(struct.unpack("<f", v)[0])
    return vals


def _strs(entries, num):
    return [bytes(v).decode() for f, _, v in entries if f == num]


def _attr(b):
    e = _walk(b)
    name = _strs(e, 1)[0]
    kind = _ints(e, 20)[0] if _ints(e, 20) else 0
    if kind == 1:  # FLOAT
        val = _floats(e, 2)[0]
    elif kind == 2:  # INT
        val = _ints(e, 3)[0]
    elif kind == 3:  # STRING
        val = _strs(e, 4)[0]
    elif kind == 6:  # FLOATS
        val = tuple(_floats(e, 7))
    elif kind == 7:  # INTS
        val = tuple(_ints(e, 8))
    elif kind == 4:  # TENSOR: its shape and element type
        t = _walk([v for f, _, v in e if f == 5][0])
        val = ("tensor", tuple(_ints(t, 1)), _ints(t, 2)[0])
    else:
        val = ("type", kind)
    return name, val


def read(path):
    """(nodes, initializers, inputs, outputs): nodes as (name, op_type, inputs, outputs,
    {attribute: value}), initializers as (name, dims, data_type)."""
    model = _walk(open(path, "rb").read())
    graph = _walk([v for f, _, v in model if f == 7][0])
    nodes = []
    for f, _, v in graph:
        if f != 1:
            continue
        e = _walk(v)
        nodes.append((_strs(e, 3)[0] if _strs(e, 3) else "", _strs(e, 4)[0], tuple(_strs(e, 1)), tuple(_strs(e, 2)),
                      dict(_attr(a) for fa, _, a in e if fa == 5)))
    inits = []
    for f, _, v in graph:
        if f == 5:
            e = _walk(v)
            inits.append((_strs(e, 8)[0], tuple(_ints(e, 1)), _ints(e, 2)[0]))
    ins = [_strs(_walk(v), 1)[0] for f, _, v in graph if f == 11]
    outs = [_strs(_walk(v), 1)[0] for f, _, v in graph if f == 12]
    return nodes, inits, ins, outs
