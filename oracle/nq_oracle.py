"""ORACLE — test infrastructure only, never part of the product path.

CPU restatement of numpy-quant's quantized-inference hot path (reference commit
mounted at /root/reference, "v1").  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and only as the checker
or as the timed CPU baseline.  The product (`numpy-quant_amd/numpy_quant`) never
imports it and fails loudly when its HIP library is missing.

Pinned by: `tests/golden/*.npz`, generated in the build container by
`tests/golden/make_golden.py` from the reference itself (its numpy-only modules
numpy_quant/numpy_quantization.py, tensor.py, numpy_helper.py imported directly,
and numpy_quant/model.py with an empty placeholder for the absent `onnx` package,
see DESIGN.md §Oracle).  `tests/test_oracle.py` checks every function here
against those vectors bit-exactly.

Arithmetic contract (NumPy 2.2 / NEP 50, the NumPy in this image and on the GPU
box): every dtype promotion below is written out explicitly instead of being
left to NumPy's promotion rules, so the restatement documents the semantics the
HIP kernels must reproduce.
"""
from __future__ import annotations

import time
from collections import OrderedDict

import numpy as np

# ----------------------------------------------------------------------------- L1 arithmetic


def qrange(bit_width: int) -> tuple[float, float]:
    """Integer range as Python floats (numpy_quantization.py:8, :30, :66)."""
    return -(2.0 ** (bit_width - 1)), 2.0 ** (bit_width - 1) - 1.0


def quant_parameters(min_val, max_val, bit_width: int, asymmetric: bool):
    """numpy_quantization.py:7-21.

    Asymmetric: s = f32((max-min)/(hi-lo)) (f32 scalar arithmetic when min/max are
    np.float32), zp = int64(rint(lo - min/s)) computed in f32 and NOT clamped.
    Symmetric: s = f32(2*max(max, min)/(hi-lo)) — max of the two, not abs-max.
    A zero point that rounds to 0 is returned as the np.int64 scalar 0 (the
    reference's `zero_point and np.array(...)`, :19), otherwise as a 0-d int64 array.
    """
    lo, hi = qrange(bit_width)
    span = hi - lo
    if asymmetric:
        s = (max_val - min_val) / span
        zp_f = lo - min_val / s
        zp_i = np.rint(zp_f).astype(np.int64)
    else:
        s = (2 * max(max_val, min_val)) / span
        zp_i = None
    scale = np.array(s, dtype=np.float32)
    if zp_i is None:
        return scale, None
    if not zp_i:
        return scale, zp_i  # falsy np.int64(0) survives `zp and ...`
    return scale, np.array(zp_i, dtype=np.int64)


def quantize(x: np.ndarray, bit_width: int, scale, zero_point) -> np.ndarray:
    """numpy_quantization.py:24-34 (via tensor.py:299-301 quantize_tensor).

    t = f32(x / s) (correctly rounded f32 division)
    with zp: u = f64(zp) + f64(t); clip to [lo, hi] in f64; rint half-even
    without: clip t to [f32(lo), f32(hi)] in f32; rint
    -> int64.
    """
    lo, hi = qrange(bit_width)
    x = np.asarray(x)
    t = np.true_divide(x, scale)
    if t.dtype != np.float32 and x.dtype == np.float32:
        raise AssertionError("quantize expects float32 activations")
    if zero_point is not None:
        u = np.asarray(zero_point).astype(np.float64) + t.astype(np.float64)
        u = np.minimum(np.maximum(u, np.float64(lo)), np.float64(hi))
    else:
        u = np.minimum(np.maximum(t, t.dtype.type(lo)), t.dtype.type(hi))
    return np.rint(u).astype(np.int64)


def dequantize(q: np.ndarray, scale, zero_point) -> np.ndarray:
    """numpy_quantization.py:37-41, tensor.py:261-265.  f32( f64(q - zp) * f64(s) )."""
    centred = q if zero_point is None else (q - zero_point)
    prod = np.asarray(centred, dtype=np.int64).astype(np.float64) * np.float64(np.float32(scale))
    return prod.astype(np.float32)


def q_matmul(a: np.ndarray, scale_a, zp_a, b: np.ndarray, scale_b, zp_b):
    """numpy_quantization.py:44-61.  Raw int64 product plus the zero-point term.

    Returns (acc int64, s_out f32, zp_term | None) with
      zp_a None, zp_b None : None
      zp_a None            : rowsum(A) * zp_b                         shape (..., M, 1)
      zp_b None            : colsum(B) * zp_a                         shape (..., 1, N)
      both                 : rowsum(A)*zp_b + colsum(B)*zp_a - zp_a*zp_b*K  (broadcast)
    """
    acc = np.matmul(a.astype(np.int64), b)
    s_out = np.float32(scale_a) * np.float32(scale_b)
    k = a.shape[-1]
    if zp_a is None and zp_b is None:
        return acc, s_out, None
    row = a.sum(axis=-1, keepdims=True)
    col = b.sum(axis=-2, keepdims=True)
    if zp_a is None:
        return acc, s_out, row * zp_b
    if zp_b is None:
        return acc, s_out, col * zp_a
    return acc, s_out, row * zp_b + col * zp_a - zp_a * zp_b * k


def requantize(acc: np.ndarray, acc_scale, acc_zp, res_scale, res_zp, bit_width: int) -> np.ndarray:
    """numpy_quantization.py:64-72.

    d = dequantize(acc); r = f32(1 / rs); v = f32(r * d);
    with rz: u = f64(rz) + f64(v), else u = v; q = int64(clip(rint(u), lo, hi)).
    """
    lo, hi = qrange(bit_width)
    d = dequantize(acc, acc_scale, acc_zp)
    r = np.float32(1) / np.float32(res_scale)
    v = (r * d).astype(np.float32)
    if res_zp is None:
        u = np.rint(v)
        return np.minimum(np.maximum(u, np.float32(lo)), np.float32(hi)).astype(np.int64)
    u = np.rint(np.asarray(res_zp).astype(np.float64) + v.astype(np.float64))
    return np.minimum(np.maximum(u, np.float64(lo)), np.float64(hi)).astype(np.int64)


# ----------------------------------------------------------------------------- float kernels


def erf(x: np.ndarray) -> np.ndarray:
    """numpy_helper.py:95-112 — Abramowitz & Stegun 7.1.26 in float32, np.exp."""
    f = np.float32
    sgn = np.sign(x)
    ax = np.abs(x)
    t = f(1.0) / (f(1.0) + f(0.3275911) * ax)
    poly = f(1.061405429) * t + f(-1.453152027)
    poly = poly * t
    poly = poly + f(1.421413741)
    poly = poly * t + f(-0.284496736)
    poly = poly * t + f(0.254829592)
    y = f(1.0) - poly * t * np.exp(-ax * ax)
    return sgn * y


def conv2d_nchw(x: np.ndarray, w: np.ndarray, b: np.ndarray, pads, strides) -> np.ndarray:
    """tensor.py:328-336 (fconv2d) + numpy_helper.py:18-92 (im2col + dot).

    The im2col matrix [N*H'*W', KH*KW*C] (column order kh, kw, c) and the weight
    matrix [KH*KW*C, K] are both C-contiguous, so `dot` issues the same sgemm the
    reference does (bit-identical result on the same BLAS).
    """
    n, c, h, wd = x.shape
    k, _, kh, kw = w.shape
    ph0, pw0, ph1, pw1 = pads
    sh, sw = strides
    xt = np.pad(x.transpose(0, 2, 3, 1), ((0, 0), (ph0, ph1), (pw0, pw1), (0, 0)))
    ho = int(np.ceil((h - kh + ph0 + ph1 + 1) / sh))
    wo = int(np.ceil((wd - kw + pw0 + pw1 + 1) / sw))
    cols = np.empty((n, ho, wo, kh, kw, c), dtype=x.dtype)
    for i in range(kh):
        for j in range(kw):
            cols[:, :, :, i, j, :] = xt[:, i:i + sh * ho:sh, j:j + sw * wo:sw, :][:, :ho, :wo, :]
    wm = np.ascontiguousarray(w.transpose(2, 3, 1, 0)).reshape(kh * kw * c, k)
    y = cols.reshape(n * ho * wo, kh * kw * c).dot(wm).reshape(n, ho, wo, k)
    return y.transpose(0, 3, 1, 2) + b.reshape(1, k, 1, 1)


# ----------------------------------------------------------------------------- tensors
# Tagged tensors: ('I', arr) int64 shape data, ('F', arr) float32, ('Q', arr, bw, s, zp)


def F(a):
    a = np.asarray(a)
    if a.dtype != np.float32:
        raise ValueError("float tensors must be float32 (tensor.py:49-50)")
    return ("F", a)


def I(a):
    return ("I", np.asarray(a))


def Q(a, bw, s, zp):
    return ("Q", np.asarray(a, dtype=np.int64), bw, s, zp)


def q_dequant(t):
    return F(dequantize(t[1], t[3], t[4]))


def _float_op(op: str, ins: list, attrs: dict):
    """onnx_operator_implementation, model.py:65-213, restated per op."""
    a = ins[0] if ins else None
    d = [t[1] if t is not None else None for t in ins]
    if op == "Add":
        if a[0] == "Q":
            x, y = ins
            return [Q(x[1] + y[1], x[2], x[3], x[4])]
        return [(a[0], d[0] + d[1])]
    if op == "Concat":
        kinds = {t[0] for t in ins}
        if len(kinds) != 1:
            raise AssertionError("Concat of mixed tensor kinds (tensor.py:317-320)")
        return [(a[0], np.concatenate(d, axis=attrs["axis"]))]
    if op == "Constant":
        v = attrs["value"]
        if v.dtype == np.float32:
            return [F(v)]
        if v.dtype == np.int64:
            return [I(v)]
        raise ValueError(f"Constant dtype {v.dtype} not supported")
    if op == "ConstantOfShape":
        v = attrs["value"]
        arr = np.full(tuple(d[0]), fill_value=v, dtype=v.dtype)
        return [F(arr) if v.dtype == np.float32 else I(arr)]
    if op == "Conv":
        return [F(conv2d_nchw(d[0], d[1], d[2], tuple(attrs["pads"]), tuple(attrs["strides"])))]
    if op == "Div":
        return [F(d[0] / d[1])]
    if op == "Equal":
        return [I(np.array(d[0] == d[1], np.int64))]
    if op == "Erf":
        return [F(erf(d[0]))]
    if op == "Expand":
        cur = np.array(d[0].shape, dtype=np.int64)
        tgt = np.array(d[1], dtype=np.int64).copy()
        keep = (tgt < cur) & (tgt == 1)
        tgt[keep] = cur[keep]
        return [F(np.broadcast_to(d[0], tuple(tgt)))]
    if op == "Gather":
        idx = ins[1][1]
        if a[0] == "I":
            return [I(d[0].take(np.atleast_1d(idx), attrs["axis"]))]
        return [F(d[0].take(idx, attrs["axis"]))]
    if op == "Gemm":
        x, w, bias = ins
        if attrs.get("transA"):
            x = _T(x)
        if attrs.get("transB"):
            w = _T(w)
        if x[0] == "Q":
            if x[2] != w[2]:
                raise AssertionError(f"{x[2]} != {w[2]}")
            acc, s, z = q_matmul(x[1], x[3], x[4], w[1], w[3], w[4])
            return [Q(acc + bias[1], 4 * x[2], s, z)]
        return [F(np.matmul(x[1], w[1]) + bias[1])]
    if op == "Identity":
        return [(a[0], d[0].copy())]
    if op == "LayerNormalization":
        x, g, bt = d
        ax = attrs["axis"]
        mean = x.mean(axis=ax, keepdims=True)
        dev = x + (-mean)
        var = (dev * dev).mean(axis=ax, keepdims=True)
        std = np.sqrt(var + np.float32(attrs["epsilon"]))
        return [F((dev * (np.float32(1) / std)) * g + bt)]
    if op == "MatMul":
        x, w = ins
        if x[0] == "Q":
            if x[2] != w[2]:
                raise AssertionError(f"{x[2]} != {w[2]}")
            acc, s, z = q_matmul(x[1], x[3], x[4], w[1], w[3], w[4])
            return [Q(acc, 4 * x[2], s, z)]
        return [F(np.matmul(d[0], d[1]))]
    if op == "Mul":
        return [(a[0], d[0] * d[1])]
    if op == "ReduceMean":
        return [F(d[0].mean(attrs["axis"], keepdims=attrs["keepdims"]))]
    if op == "Relu":
        return [F((d[0] > 0) * d[0])]
    if op == "Reshape":
        if a[0] == "Q":
            return [Q(d[0].reshape(d[1]), a[2], a[3], a[4])]
        return [(a[0], d[0].reshape(d[1]))]
    if op == "Sigmoid":
        return [F(np.float32(1) / (np.exp(-d[0]) + np.float32(1.0)))]
    if op == "Shape":
        return [I(np.array(d[0].shape, dtype=np.int64))]
    if op == "Slice":
        sl = [slice(None)] * d[0].ndim
        for s0, e0, ax in zip(d[1], d[2], d[3]):
            sl[ax] = slice(s0, e0)
        return [(a[0], d[0][tuple(sl)])]
    if op == "Softmax":
        ax = attrs["axis"]
        m = d[0] + (-d[0].max(axis=ax, keepdims=True))
        e = np.exp(m)
        return [F(e / e.sum(axis=ax, keepdims=True))]
    if op == "Tanh":
        return [F(np.tanh(d[0]))]
    if op == "Transpose":
        if a[0] == "Q":
            return [Q(d[0].transpose(attrs["perm"]), a[2], a[3], a[4])]
        return [(a[0], d[0].transpose(attrs["perm"]))]
    if op == "Unsqueeze":
        # model.py:203-206 returns the tensor itself rather than a 1-list; the
        # executor then unpacks it element-wise, so the output is its first row.
        return [I(np.expand_dims(d[0], axis=tuple(d[1]))[0])]
    if op == "Where":
        if ins[1][0] != ins[2][0]:
            raise AssertionError("Where of mixed tensor kinds (tensor.py:323-325)")
        return [(ins[1][0], np.where(d[0], d[1], d[2]))]
    raise ValueError(f"ONNX operand {op} not supported.")


def _T(t):
    if t[0] == "Q":
        zp = t[4]
        return Q(t[1].T, t[2], t[3], None if zp is None else np.asarray(zp).T)
    return (t[0], t[1].T)


# ----------------------------------------------------------------------------- graph + executors


class Graph:
    """Plain graph restated from Model.from_onnx (model.py:249-292): initializers
    are float32 constants, graph inputs are variables, node order = file order."""

    def __init__(self, model_proto):
        g = model_proto.graph
        self.constants = OrderedDict()
        for t in g.initializer:
            arr = np.array(t.to_array())
            if arr.dtype != np.float32:
                raise ValueError("User np.float32 for FTensor")
            self.constants[t.name] = arr
        self.inputs = [vi.name for vi in g.input]
        self.outputs = [vi.name for vi in g.output]
        from importlib import import_module
        attr_value = import_module("numpy_quant.onnx_proto").attribute_value
        self.nodes = [(n.name, n.op_type, {a.name: attr_value(a) for a in n.attribute},
                       list(n.input), list(n.output)) for n in g.node]
        # value order as the reference's value_dict (initializers, inputs, then first
        # appearance as node input/output)
        order = list(self.constants) + [i for i in self.inputs if i not in self.constants]
        seen = set(order)
        for _, _, _, ins, outs in self.nodes:
            for v in ins + outs:
                if v not in seen:
                    seen.add(v)
                    order.append(v)
        self.value_order = order


def float_forward(graph: Graph, inputs: list[np.ndarray], profile: bool = False):
    """Model.__call__, model.py:294-326.  Returns {value: tagged tensor}."""
    vals: dict = {n: F(a) for n, a in graph.constants.items()}
    for arr, name in zip(inputs, graph.inputs):
        if arr.dtype == np.float32:
            vals[name] = F(arr.copy())
        elif arr.dtype == np.int64:
            vals[name] = I(arr.copy())
        else:
            raise ValueError(f"Array dtype {arr.dtype} not supported")
    times = {}
    for name, op, attrs, ins, outs in graph.nodes:
        t0 = time.time()
        res = _float_op(op, [vals[i] for i in ins], attrs)
        times[op] = times.get(op, 0.0) + time.time() - t0
        for o, r in zip(outs, res):
            vals[o] = r
    if profile:
        return vals, times
    return vals


class QParams:
    __slots__ = ("scale", "zero_point")

    def __init__(self, scale, zero_point):
        self.scale = scale
        self.zero_point = zero_point


def calibrate(graph: Graph, calibration_inputs: list[np.ndarray], bit_width: int = 8):
    """Model.quantize, model.py:328-442.  Returns (qparams, qconstants)."""
    vals = float_forward(graph, calibration_inputs)
    vmin, vmax = {}, {}
    for name in graph.value_order:
        arr = vals[name][1]
        flat = arr.reshape((arr.shape[0], -1) if arr.shape else (-1,))
        vmin[name] = np.mean(flat.min())
        vmax[name] = np.mean(flat.max())

    def params(name, asym):
        s, z = quant_parameters(vmin[name], vmax[name], bit_width, asym)
        return QParams(s, z)

    qp: dict[str, QParams] = {}
    qconst: dict[str, tuple] = {}
    for name in graph.inputs:
        qp[name] = params(name, True)
    for name, arr in graph.constants.items():
        p = params(name, False)
        qconst[name] = Q(quantize(arr, bit_width, p.scale, p.zero_point), bit_width, p.scale, p.zero_point)
        qp[name] = p
    is_const = set(graph.constants)
    for _, op, _, ins, outs in graph.nodes:
        if op == "MatMul":
            qp[outs[0]] = params(outs[0], True)
        if op == "Gemm":
            for v in ins[:2]:
                if v not in is_const:
                    qp[v] = params(v, True)
            bias = ins[2]
            bscale = qp[ins[0]].scale * qp[ins[1]].scale
            qp[bias] = QParams(bscale, None)
            qconst[bias] = Q(quantize(graph.constants[bias], 4 * bit_width, bscale, None),
                             4 * bit_width, bscale, None)
            qp[outs[0]] = params(outs[0], True)
        if op == "Add" and (ins[0] in is_const or ins[1] in is_const):
            bi, xi = (0, 1) if ins[0] in is_const else (1, 0)
            bscale = qp[ins[xi]].scale
            qconst[ins[bi]] = Q(quantize(graph.constants[ins[bi]], 4 * bit_width, bscale, None),
                                4 * bit_width, bscale, None)
            qp[ins[bi]] = QParams(bscale, None)
            qp[outs[0]] = params(outs[0], True)
        elif op in ("Identity", "Relu"):
            qp[outs[0]] = qp[ins[0]]
        else:
            qp[outs[0]] = params(outs[0], True)
    return qp, qconst


def quantize_with(graph: Graph, qparams: dict, bit_width: int = 8):
    """Model.quantize's constant handling (model.py:328-442, as calibrate above) for GIVEN
    per-value parameters (e.g. another implementation's calibration): every constant quantized
    with its own parameters, Gemm biases and constants added to a value at 4 * bit_width with
    the product / input scale.  Returns (qparams, qconstants)."""
    qp = dict(qparams)
    qconst: dict[str, tuple] = {}
    for name, arr in graph.constants.items():
        p = qp[name]
        qconst[name] = Q(quantize(arr, bit_width, p.scale, p.zero_point), bit_width, p.scale, p.zero_point)
    is_const = set(graph.constants)
    for _, op, _, ins, outs in graph.nodes:
        if op == "Gemm":
            bias = ins[2]
            bscale = qp[ins[0]].scale * qp[ins[1]].scale
            qp[bias] = QParams(bscale, None)
            qconst[bias] = Q(quantize(graph.constants[bias], 4 * bit_width, bscale, None),
                             4 * bit_width, bscale, None)
        if op == "Add" and (ins[0] in is_const or ins[1] in is_const):
            bi, xi = (0, 1) if ins[0] in is_const else (1, 0)
            bscale = qp[ins[xi]].scale
            qconst[ins[bi]] = Q(quantize(graph.constants[ins[bi]], 4 * bit_width, bscale, None),
                                4 * bit_width, bscale, None)
            qp[ins[bi]] = QParams(bscale, None)
    return qp, qconst


def quantized_forward(graph: Graph, qp: dict, qconst: dict, inputs: list[np.ndarray],
                      bit_width: int, profile: bool = False):
    """QModel.__call__, model.py:486-565.  Returns {value: tagged tensor} (and the
    per-op-type profile dict with the TinyqQuant/TinyqDequant buckets)."""
    vals: dict = dict(qconst)
    for arr, name in zip(inputs, graph.inputs):
        p = qp[name]
        if arr.dtype == np.float32:
            vals[name] = Q(quantize(arr, bit_width, p.scale, p.zero_point), bit_width, p.scale, p.zero_point)
        elif arr.dtype == np.int64:
            vals[name] = I(arr)
        else:
            raise ValueError(f"Array dtype {arr.dtype} not supported")
    times = {op: 0.0 for op in {n[1] for n in graph.nodes}}
    times["TinyqQuant"] = 0.0
    times["TinyqDequant"] = 0.0
    for _, op, attrs, ins, outs in graph.nodes:
        args = []
        for i in ins:
            t = vals[i]
            if op in ("MatMul", "Gemm") and t[0] == "F":
                t0 = time.time()
                p = qp[i]
                t = Q(quantize(t[1], bit_width, p.scale, p.zero_point), bit_width, p.scale, p.zero_point)
                times["TinyqQuant"] += time.time() - t0
            elif op not in ("MatMul", "Gemm") and t[0] == "Q":
                t0 = time.time()
                t = q_dequant(t)
                times["TinyqDequant"] += time.time() - t0
            args.append(t)
        t0 = time.time()
        res = _float_op(op, args, attrs)
        times[op] += time.time() - t0
        for o, r in zip(outs, res):
            if op == "Gemm":
                p = qp[outs[0]]
                r = Q(requantize(r[1], r[3], r[4], p.scale, p.zero_point, bit_width), bit_width,
                      p.scale, p.zero_point)
            vals[o] = r
    if profile:
        return vals, times
    return vals


def outputs_of(graph: Graph, vals: dict) -> list[np.ndarray]:
    """model.py:552-559: float outputs as-is, quantized outputs dequantized."""
    out = []
    for name in graph.outputs:
        t = vals[name]
        if t[0] == "F":
            out.append(t[1])
        elif t[0] == "Q":
            out.append(q_dequant(t)[1])
        else:
            raise ValueError
    return out
