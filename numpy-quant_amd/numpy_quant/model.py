"""ONNX graph IR, float and quantized executors — the drop-in for
numpy_quant/model.py (Model.from_onnx / Model.quantize / Model.__call__ /
QModel.__call__), running every tensor op in libnqk.so on the MI355X.

The node loop is the reference's (model.py:294-326, 486-565): per node, QTensor
inputs of float ops are dequantized, float inputs of MatMul / Gemm are quantized
with the calibrated parameters, Gemm outputs are requantized.  All intermediate
values stay in HBM; `value.data.data` copies one to the host on request.
`QModel.__call__` runs through a fused device plan (plan.py, compiled on first
use) with bit-identical results for the hot MatMul chains; `qmodel.keep_values = True`
(or `profile=True`) keeps the reference's node-by-node loop, which materialises every
intermediate `value.data`.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from time import time
from typing import Any, List, Union

import numpy as np

from . import _lib
from . import onnx_proto
from .device import sync
from .numpy_quantization import quant_parameters
from .tensor import (FTensor, ITensor, QTensor, Tensor, concat, fconv2d, quantize_tensor, where)
from . import kernels as K


class Constant:
    def __init__(self, name: str, outputs: List["Node"], data: Tensor = None):
        self.name = name
        self.outputs = outputs
        self.data = data

    def __repr__(self):
        return f"Constant({self.name})"


class Variable:
    def __init__(self, name: str, inputs: List["Node"], outputs: List["Node"], data: Tensor = None):
        self.name = name
        self.inputs = inputs
        self.outputs = outputs
        self.data = data

    def __repr__(self):
        return f"Variable({self.name})"


Value = Union[Constant, Variable]


class Node:
    def __init__(self, name: str, op: str, attrs: dict[str, Any], inputs: List[Value], outputs: List[Value]):
        self.name = name
        self.op = op
        self.attrs = attrs
        self.inputs = inputs
        self.outputs = outputs

    def __repr__(self):
        return f"Node({self.name})"


class QuantizationParams:
    def __init__(self, scale: np.float32, zero_point: Union[np.int64, None]):
        self.scale = scale
        self.zero_point = zero_point

    def __repr__(self):
        return f"QuantizationParams(scale={self.scale}, zero_point={self.zero_point})"


def _listing(kind: str, fields) -> str:
    """Readable multi-line dump of an IR object: one line per element of each list or
    dict field (the reference prints its models this way, model.py:223-234, 464-484)."""
    out = [f"{kind}("]
    for name, val in fields:
        if isinstance(val, dict):
            out.append(f"  {name}={{")
            out.extend(f"    {k}: {v}," for k, v in val.items())
            out.append("  },")
        elif isinstance(val, list):
            out.append(f"  {name}=[")
            out.extend(f"    {e}" for e in val)
            out.append("  ],")
        else:
            out.append(f"  {name}={val},")
    out.append(")")
    return "\n".join(out) + "\n"


# ----------------------------------------------------------------------------- operators
def _gemm(inputs, attrs):
    x, w, b = inputs
    if attrs.get("transA"):
        x = x.T
    if attrs.get("transB"):
        if (isinstance(x, FTensor) and isinstance(w, FTensor) and x.dev.ndim == 2 and w.dev.ndim == 2
                and x.dev.shape[0] == 1):
            # x[1, K] @ w.T: NumPy's matmul takes OpenBLAS GEMV-T for this layout (the
            # w.T view has its columns contiguous), or sdot for one column, whose summation
            # orders differ from GEMM's
            n, k = w.dev.shape
            if K.small_one_row(n, k):
                return [FTensor(K.sgemv_small(x.dev, w.dev)) + b]
            if K.gemv_t_applies(1, n, k):
                return [FTensor(K.sgemv_t(x.dev, w.dev)) + b]
        w = w.T
    return [x.matmul(w) + b]


def _layernorm(inputs, attrs):
    x, g, b = inputs
    return [FTensor(K.layernorm(x.dev, g.dev, b.dev, attrs.get("axis", -1), attrs.get("epsilon", 1e-5)))]


def _slice(inputs, attrs):
    x = inputs[0]
    starts, ends, axes = inputs[1].data, inputs[2].data, inputs[3].data
    slices = [slice(None, None, None)] * x.shape.size
    for s, e, a in zip(starts, ends, axes):
        slices[a] = slice(s, e)
    return [x.__getitem__(tuple(slices))]


def _constant(inputs, attrs):
    v = attrs["value"]
    if v.dtype == np.float32:
        return [FTensor(v)]
    if v.dtype == np.int64:
        return [ITensor(v)]
    cls = v.dtype.__class__
    raise ValueError(f"Constant value type {cls.__module__}.{cls.__qualname__} not supported.")


def _constant_of_shape(inputs, attrs):
    v = attrs["value"]
    arr = np.full(tuple(inputs[0].data), fill_value=v, dtype=v.dtype)
    if v.dtype == np.float32:
        return [FTensor(arr)]
    if v.dtype == np.int64:
        return [ITensor(arr)]
    cls = v.dtype.__class__
    raise ValueError(f"Constant value type {cls.__module__}.{cls.__qualname__} not supported.")


_OPS = {
    "Add": lambda i, a: [i[0] + i[1]],
    "Concat": lambda i, a: [concat(list(i), axis=a["axis"])],
    "Constant": _constant,
    "ConstantOfShape": _constant_of_shape,
    "Conv": lambda i, a: [fconv2d(i[0], i[1], i[2], tuple(a["pads"]), tuple(a["strides"]))],
    "Div": lambda i, a: [i[0].div(i[1])],
    "Equal": lambda i, a: [i[0] == i[1]],
    "Erf": lambda i, a: [i[0].erf()],
    "Expand": lambda i, a: [i[0].expand(i[1])],
    "Gather": lambda i, a: [i[0].take(i[1], axis=a["axis"])],
    "Gemm": _gemm,
    "Identity": lambda i, a: [i[0].copy()],
    "LayerNormalization": _layernorm,
    "MatMul": lambda i, a: [i[0].matmul(i[1])],
    "Mul": lambda i, a: [i[0] * i[1]],
    "ReduceMean": lambda i, a: [i[0].mean(a["axis"], keepdims=a["keepdims"])],
    "Relu": lambda i, a: [i[0].relu()],
    "Reshape": lambda i, a: [i[0].reshape(i[1])],
    "Sigmoid": lambda i, a: [i[0].sigmoid()],
    "Shape": lambda i, a: [i[0].shape],
    "Slice": _slice,
    "Softmax": lambda i, a: [i[0].softmax(axis=a["axis"])],
    "Tanh": lambda i, a: [i[0].tanh()],
    "Transpose": lambda i, a: [i[0].transpose(a["perm"])],
    # model.py:203-206 returns the tensor itself instead of a 1-list; the executor
    # then unpacks it element-wise: the output is row 0 (kept bug-compatible)
    "Unsqueeze": lambda i, a: i[0].expand_dims(axis=i[1]),
    "Where": lambda i, a: [where(i[0], i[1], i[2])],
}


def onnx_operator_implementation(op: str, inputs: list[Tensor], attrs: dict[str, object]) -> list[Tensor]:
    """Device implementation of model.py:65-213 (same op set, same results)."""
    fn = _OPS.get(op)
    if fn is None:
        raise ValueError(f"ONNX operand {op} not supported.")
    return fn(inputs, attrs)


# ----------------------------------------------------------------------------- models
class Model:
    def __init__(self, nodes: list[Node], values: list[Value], inputs: List[Variable], outputs: List[Variable]):
        self.nodes = nodes
        self.values = values
        self.inputs = inputs
        self.outputs = outputs

    def __repr__(self):
        return f"Model({len(self.nodes)} nodes, {len(self.values)} values, inputs={self.inputs}, outputs={self.outputs})"

    def __str__(self):
        return _listing("Model", [("nodes", self.nodes), ("values", self.values), ("inputs", self.inputs),
                                  ("outputs", self.outputs)])

    def __del__(self):
        # break node <-> value cycles so device buffers are released promptly (model.py:236-247)
        for node in getattr(self, "nodes", []):
            node.inputs = []
            node.outputs = []
        for value in getattr(self, "values", []):
            if isinstance(value, Variable):
                value.inputs = []
            value.outputs = []

    @classmethod
    def from_onnx(cls, onnx_model):
        """model.py:249-292.  Accepts a decoded onnx_proto.ModelProto (or anything
        duck-typed like onnx.ModelProto), a file path or raw bytes."""
        if isinstance(onnx_model, (str, os.PathLike, bytes, bytearray)):
            onnx_model = onnx_proto.load(onnx_model)
        graph = onnx_model.graph
        value_dict: dict[str, Value] = {}
        for t in graph.initializer:
            arr = np.array(t.to_array() if hasattr(t, "to_array") else onnx_proto.to_array(t))
            value_dict[t.name] = Constant(t.name, outputs=[], data=FTensor(arr))
        inputs: List[Value] = []
        for vi in graph.input:
            var = Variable(vi.name, inputs=[], outputs=[])
            value_dict[vi.name] = var
            inputs.append(var)
        nodes: dict[str, Node] = {}
        for n in graph.node:
            node = Node(name=n.name, op=n.op_type,
                        attrs={a.name: onnx_proto.attribute_value(a) for a in n.attribute},
                        inputs=[value_dict[i] for i in n.input], outputs=[])
            for i in n.input:
                value_dict[i].outputs.append(node)
            for o in n.output:
                if o in value_dict:
                    value_dict[o].inputs.append(node)
                else:
                    value_dict[o] = Variable(name=o, inputs=[node], outputs=[])
            node.outputs = [value_dict[o] for o in n.output]
            nodes[n.name] = node
        outputs = [value_dict[vi.name] for vi in graph.output]
        return cls(list(nodes.values()), list(value_dict.values()), inputs, outputs)

    def rebatch(self, batch: int) -> int:
        """Rewrite the batch-1 int64 shape constants of a torch export in place
        (onnx_proto.rebatch).  The batch-1 original is kept in
        the node's attribute dict, which a QModel built from this model shares, so
        either one may be rebatched any number of times."""
        count = 0
        for node in self.nodes:
            if node.op != "Constant":
                continue
            v = node.attrs.setdefault("__batch1_value__", node.attrs.get("value"))
            if isinstance(v, np.ndarray) and v.dtype == np.int64 and v.ndim == 1 and v.shape[0] in (3, 4) and v[0] == 1:
                v = v.copy()
                v[0] = batch
                node.attrs["value"] = v
                count += 1
        return count

    def _set_inputs(self, inputs):
        for array, variable in zip(inputs, self.inputs):
            if array.dtype == np.float32:
                variable.data = FTensor(np.ascontiguousarray(array))
            elif array.dtype == np.int64:
                variable.data = ITensor(array.copy())
            else:
                raise ValueError(f"Array dtype {array.dtype} not supported")

    def __call__(self, inputs: List[np.ndarray], profile=False):
        """Float executor (model.py:294-326), on device."""
        times = {op: 0.0 for op in {n.op for n in self.nodes}}
        self._set_inputs(inputs)
        for node in self.nodes:
            args = [i.data for i in node.inputs]
            t0 = time()
            outs = onnx_operator_implementation(node.op, args, node.attrs)
            if profile:
                sync()
            times[node.op] += time() - t0
            for o, tensor in zip(node.outputs, outs):
                o.data = tensor
        result = [out.data.data for out in self.outputs]
        return (result, times) if profile else result

    def calibrate(self, calibration_inputs: list[np.ndarray]) -> tuple[dict, dict]:
        """Float forward + per-value global min / max (model.py:329-336), min/max on device."""
        self(calibration_inputs)
        vmin, vmax = {}, {}
        for val in self.values:
            t = val.data
            if isinstance(t, FTensor):
                mn, mx = K.minmax(t.dev)
                vmin[val.name], vmax[val.name] = np.mean(mn), np.mean(mx)
            else:
                d = t.data
                flat = d.reshape((d.shape[0], -1) if d.shape else (-1,))
                vmin[val.name], vmax[val.name] = np.mean(flat.min()), np.mean(flat.max())
        return vmin, vmax

    def quantize(self, calibration_inputs: list[np.ndarray], bit_width=8):
        """Calibration + graph rewrite (model.py:328-442)."""
        vmin, vmax = self.calibrate(calibration_inputs)

        def params(value: Value, asym: bool):
            s, z = quant_parameters(vmin[value.name], vmax[value.name], bit_width=bit_width, asymmetric=asym)
            return QuantizationParams(s, z)

        return self._rewrite(bit_width, params)

    def quantize_with(self, quant_params: dict, bit_width=8):
        """The graph rewrite of Model.quantize with given per-value quantization
        parameters (e.g. calibrated on a smaller batch, or the reference's own),
        skipping the calibration forward."""
        return self._rewrite(bit_width, lambda value, asym: quant_params[value.name])

    def load_quantized(self, path):
        """The QModel saved by `QModel.save(path)` (blob.py) on this model's graph:
        no calibration forward and no constant re-quantization."""
        from . import blob
        return blob.load(self, path)

    def _rewrite(self, bit_width, params, constants=None):
        """model.py:338-442.  `constants`: name -> ready quantized QTensor (blob.py);
        those constants are taken as they are instead of being quantized here."""
        constants = constants or {}
        wanted = {}
        if constants:
            # a blob must carry exactly this graph's constants, each with this graph's shape:
            # never quietly re-quantize a missing one from local weights, never attach a
            # blob of another model whose initializer names happen to match
            graph_consts = {v.name: v for v in self.values if isinstance(v, Constant)}
            missing = sorted(set(graph_consts) - set(constants))
            extra = sorted(set(constants) - set(graph_consts))
            if missing or extra:
                raise ValueError(f"blob constants differ from the graph's: missing {missing[:5]}, "
                                 f"unknown {extra[:5]}")
            for name, t in constants.items():
                d = graph_consts[name].data
                want = None if d is None else tuple(d.dev.shape if hasattr(d, "dev") else np.shape(d.data))
                if want is not None and tuple(t.dev.shape) != want:
                    raise ValueError(f"blob constant {name}: shape {tuple(t.dev.shape)}, graph {want}")

        def qconst(value, bw, scale, zp):
            t = constants.get(value.name)
            if t is None:
                return quantize_tensor(value.data, bw, scale, zp)
            wanted[value.name] = bw  # a bias is quantized at bw, then again at 4*bw: last wins
            return t

        node_dict = {node.name: node for node in self.nodes}
        value_dict = {value.name: value for value in self.values}

        qnodes: OrderedDict[str, Node] = OrderedDict()
        qvalues: dict[str, Value] = {}
        qp: dict[str, QuantizationParams] = {}
        for value in self.inputs:
            qvalues[value.name] = value
            qp[value.name] = params(value, isinstance(value, Variable))
        for value in self.values:
            if isinstance(value, Constant):
                p = params(value, False)
                qt = qconst(value, bit_width, p.scale, p.zero_point)
                qt._is_weight = True
                qvalues[value.name] = Constant(value.name, [], qt)
                qp[value.name] = p
        for node in self.nodes:
            out_val = node.outputs[0]
            if node.op == "MatMul":
                qnodes[node.name] = Node(node.name, "MatMul", node.attrs, [], [])
                qp[out_val.name] = params(out_val, True)
                qvalues[out_val.name] = Variable(out_val.name, [], [], None)
            if node.op == "Gemm":
                for iv in node.inputs[:2]:
                    if isinstance(iv, Variable):
                        qvalues[iv.name] = Variable(iv.name, [], [], None)
                        qp[iv.name] = params(iv, True)
                bias = node.inputs[2]
                bscale = qp[node.inputs[0].name].scale * qp[node.inputs[1].name].scale
                qp[bias.name] = QuantizationParams(bscale, None)
                qvalues[bias.name] = Constant(bias.name, [], qconst(bias, 4 * bit_width, bscale, None))
                qnodes[node.name] = Node(node.name, "Gemm", node.attrs, [], [])
                qp[out_val.name] = params(out_val, True)
                qvalues[out_val.name] = Variable(out_val.name, [], [], None)
            if node.op == "Add" and (isinstance(node.inputs[0], Constant) or isinstance(node.inputs[1], Constant)):
                bi, xi = (0, 1) if isinstance(node.inputs[0], Constant) else (1, 0)
                bname = node.inputs[bi].name
                bscale = qp[node.inputs[xi].name].scale
                qvalues[bname] = Constant(bname, [], qconst(node.inputs[bi], 4 * bit_width, bscale, None))
                qp[bname] = QuantizationParams(bscale, None)
                qnodes[node.name] = Node(node.name, "Add", node.attrs, [], [])
                qp[out_val.name] = params(out_val, True)
                qvalues[out_val.name] = Variable(out_val.name, [], [], None)
            elif node.op in ("Identity", "Relu"):
                qvalues[out_val.name] = Variable(out_val.name, [], [], None)
                qp[out_val.name] = qp[node.inputs[0].name]
                qnodes[node.name] = Node(node.name, node.op, node.attrs, [], [])
            else:
                qvalues[out_val.name] = Variable(out_val.name, [], [], None)
                qp[out_val.name] = params(out_val, True)
                qnodes[node.name] = Node(node.name, node.op, node.attrs, [], [])
        for name, qnode in qnodes.items():
            qnode.inputs = [qvalues[i.name] for i in node_dict[name].inputs]
            qnode.outputs = [qvalues[o.name] for o in node_dict[name].outputs]
        for name, qvalue in qvalues.items():
            if isinstance(qvalue, Variable):
                qvalue.inputs = [qnodes[i.name] for i in value_dict[name].inputs]
            qvalue.outputs = [qnodes[o.name] for o in value_dict[name].outputs]
        for name, bw in wanted.items():
            if qvalues[name].data.bit_width != bw:
                raise ValueError(f"blob constant {name}: bit width {qvalues[name].data.bit_width}, the graph needs {bw}")
        qoutputs = [qvalues[o.name] for o in self.outputs]
        qinputs = [qvalues[i.name] for i in self.inputs]
        return QModel(list(qnodes.values()), list(qvalues.values()), qinputs, qoutputs, bit_width, qp)


class QModel(Model):
    def __init__(self, nodes, values, inputs, outputs, bit_width: int, quant_params: dict[str, QuantizationParams]):
        super().__init__(nodes, values, inputs, outputs)
        self.bit_width = bit_width
        self.quant_params = quant_params
        self._deq_cache: dict[str, FTensor] = {}
        self._plan = None
        # QModel.__call__ compiles the fused plan on first use (NQK_FUSE=0: never);
        # keep_values = True runs the reference's node loop instead, so every
        # intermediate value.data is populated (reference test/test_mlp.py:159-168)
        self.fuse = os.environ.get("NQK_FUSE", "1") != "0"
        self.keep_values = False

    def __repr__(self):
        return (f"QModel({len(self.nodes)} nodes, {len(self.values)} values, bit_width={self.bit_width}, "
                f"inputs={self.inputs}, outputs={self.outputs})")

    def __str__(self):
        return _listing("QModel", [("nodes", self.nodes), ("values", self.values), ("inputs", self.inputs),
                                   ("outputs", self.outputs), ("bit_width", self.bit_width),
                                   ("quant_params", self.quant_params)])

    def _dequant_input(self, value: Value) -> FTensor:
        if isinstance(value, Constant):
            hit = self._deq_cache.get(value.name)
            if hit is None:
                hit = value.data.dequantize()
                self._deq_cache[value.name] = hit
            return hit
        return value.data.dequantize()

    def set_inputs(self, inputs: List[np.ndarray]):
        for array, variable in zip(inputs, self.inputs):
            qp = self.quant_params[variable.name]
            if isinstance(array, FTensor):
                variable.data = quantize_tensor(array, self.bit_width, qp.scale, qp.zero_point)
            elif array.dtype == np.float32:
                variable.data = quantize_tensor(FTensor(np.ascontiguousarray(array)), self.bit_width, qp.scale,
                                                qp.zero_point)
            elif array.dtype == np.int64:
                variable.data = ITensor(array)
            else:
                raise ValueError(f"Array dtype {array.dtype} not supported")

    def compile(self):
        """Build the fused device plan (plan.py): matched transformer layers run as
        fused launches with bit-identical results; everything else stays eager.
        Values inside fused layers are not materialised (their `.data` is None)."""
        from .plan import compile_plan
        self._plan = compile_plan(self)
        return self._plan

    def save(self, path) -> int:
        """Write the packed quantized constants + every QuantizationParams (blob.py);
        `Model.load_quantized(path)` rebuilds this QModel on the same graph."""
        from . import blob
        return blob.save(self, path)

    def graph(self, example_inputs):
        """Capture one forward on inputs of this shape as a hipGraph (graph.py); the
        returned DeviceGraph replays it with one launch and the same results."""
        from .graph import DeviceGraph
        return DeviceGraph(self, example_inputs)

    def _run_node(self, node, times, profile=False):
        """One iteration of the node loop of QModel.__call__ (model.py:502-550)."""
        args = []
        if node.op in ("MatMul", "Gemm"):
            for i in node.inputs:
                if isinstance(i.data, FTensor):
                    qp = self.quant_params[i.name]
                    t0 = time()
                    args.append(quantize_tensor(i.data, self.bit_width, qp.scale, qp.zero_point))
                    if profile:
                        sync()
                    if times is not None:
                        times["TinyqQuant"] += time() - t0
                else:
                    args.append(i.data)
        else:
            for i in node.inputs:
                if isinstance(i.data, QTensor):
                    t0 = time()
                    args.append(self._dequant_input(i))
                    if profile:
                        sync()
                    if times is not None:
                        times["TinyqDequant"] += time() - t0
                else:
                    args.append(i.data)
        t0 = time()
        outs = onnx_operator_implementation(node.op, args, node.attrs)
        if node.op == "Gemm":
            qp = self.quant_params[node.outputs[0].name]
            outs = [t.requantize(self.bit_width, qp.scale, qp.zero_point) for t in outs]
        if profile:
            sync()
        if times is not None:
            times[node.op] += time() - t0
        for o, tensor in zip(node.outputs, outs):
            o.data = tensor

    def run(self, profile=False, eager=False):
        """The node loop of QModel.__call__ (model.py:497-550) on device tensors,
        through the fused plan when one was compiled (and not `eager`)."""
        times = {op: 0.0 for op in {n.op for n in self.nodes}}
        times["TinyqQuant"] = 0.0
        times["TinyqDequant"] = 0.0
        if self._plan is not None and not eager:
            self._plan.run(self, times, profile)
        else:
            for node in self.nodes:
                self._run_node(node, times, profile)
        return times

    def outputs_device(self) -> list[FTensor]:
        res = []
        for out_var in self.outputs:
            d = out_var.data
            if isinstance(d, FTensor):
                res.append(d)
            elif isinstance(d, QTensor):
                res.append(d.dequantize())
            else:
                raise ValueError
        return res

    def __call__(self, inputs: List[np.ndarray], profile=False):
        """QModel.__call__ (model.py:486-565).  The fused plan (bit-identical) unless
        keep_values is set or a per-op profile is asked for (profile=True returns the
        reference's {op_type: seconds} dict, which needs the node loop)."""
        eager = self.keep_values or profile
        if not eager and self._plan is None and self.fuse:
            self.compile()
        self.set_inputs(inputs)
        times = self.run(profile=profile, eager=eager)
        outs = [t.data for t in self.outputs_device()]
        return (outs, times) if profile else outs
