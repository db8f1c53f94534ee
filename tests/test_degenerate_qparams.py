"""The calibration's degenerate quantization parameters.

`Model.quantize` (reference model.py:328-442) calls `quant_parameters` (numpy_quantization.py:7-21)
asymmetrically for EVERY node output, including the outputs of the graph's ONNX `Constant` nodes
(the reference IR makes them Variables: model.py:270-292).  Those values are the same number on
every calibration image, so min == max, the scale is (max - min) / 255 = 0 and the zero point
is rint(-128 - min / 0) = rint(-inf), cast to int64: INT64_MIN.  That is where the calibration's
"divide by zero" / "invalid value" warnings come from (numpy_quantization.py:10-13), in the
reference and in this build alike.  On the ViT-Base graph they are, per layer,
  * attention/Constant_3_output_0             the Div constant sqrt(64) = 8 of QK^T / 8,
  * intermediate_act_fn/Constant{,_1,_2}       GELU's sqrt(2), 1 and 0.5,
and in the embeddings the shape arithmetic of the CLS-token Expand (Constant_*, ConstantOfShape,
Mul, Where) and of the patch Reshape: 60 values of 717.

`QModel.__call__` (model.py:486-565) reads quantization parameters only for (1) the graph
inputs, (2) the FLOAT inputs of MatMul / Gemm (quantize) and (3) Gemm outputs (requantize).
None of the 60 values is any of those (every consumer is Div / Mul / Add / Erf / Reshape /
Expand / Where / Equal / Concat), so the NaN-free but meaningless (0, INT64_MIN) pairs never
reach a kernel.  These tests pin both halves of that claim:
  * CPU: on the reference's own recorded parameters (tests/golden/vit_b1.json, api.json), the
    degenerate set is exactly the Constant-node outputs (+ the shape values computed only from
    them), and no MatMul / Gemm / graph input reads one of them;
  * GPU: the device calibration produces the same degenerate set, and neither the fused B = 256
    plan (plan build + forward) nor the node loop looks one of them up.
"""
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")
VIT = "vit_image_classifier_no_weights.onnx"
INT64_MIN = -(1 << 63)


def _degenerate_names(qparams_json: dict) -> set:
    out = set()
    for name, p in qparams_json.items():
        s = struct.unpack("<f", struct.pack("<I", p["scale_bits"]))[0]
        if s == 0.0 or not np.isfinite(s) or p["zp"] == INT64_MIN:
            out.add(name)
    return out


def _graph():
    from numpy_quant import onnx_proto
    return onnx_proto.load(os.path.join(MODELS, VIT), synthetic_weights=True, seed=0).graph


def test_degenerate_qparams_are_constant_node_outputs_never_read():
    g = _graph()
    for fixture, key in (("vit_b1.json", ("bw8", "qparams")), ("api.json", ("vit_b8_calibration", "qparams"))):
        meta = json.load(open(os.path.join(GOLDEN, fixture)))
        qp = meta[key[0]][key[1]]
        bad = _degenerate_names(qp)
        assert bad, fixture
        # every degenerate value is a Constant node's output, or a node output computed only from them
        const_outs = {o for n in g.node if n.op_type == "Constant" for o in n.output}
        derived = set(const_outs)
        for n in g.node:  # topological order
            if n.input and all(i in derived for i in n.input if i):
                derived.update(n.output)
        assert bad <= derived, sorted(bad - derived)[:5]
        assert {n for n in bad if "intermediate_act_fn/Constant" in n} and \
            {n for n in bad if "attention/attention/Constant_3" in n}
        # and no reader of quantization parameters in QModel.__call__ touches one
        assert not bad & {vi.name for vi in g.input}
        for n in g.node:
            if n.op_type in ("MatMul", "Gemm"):
                assert not bad & set(n.input), (n.name, bad & set(n.input))
            if n.op_type == "Gemm":
                assert not bad & set(n.output)
            if any(i in bad for i in n.input):
                assert n.op_type not in ("MatMul", "Gemm", "Conv")


class _Recording(dict):
    """quant_params that remembers every name looked up"""

    def __init__(self, *a):
        super().__init__(*a)
        self.seen = set()

    def __getitem__(self, k):
        self.seen.add(k)
        return super().__getitem__(k)

    def get(self, k, default=None):
        self.seen.add(k)
        return super().get(k, default)


@pytest.mark.gpu
def test_degenerate_qparams_never_read_by_b256_plan_or_node_loop():
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    arrs = np.load(os.path.join(GOLDEN, "vit_b1.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "vit_b1.json")))
    proto = onnx_proto.load(os.path.join(MODELS, VIT), synthetic_weights=True, seed=meta["seed"])
    model = Model.from_onnx(proto)
    with np.errstate(divide="ignore", invalid="ignore"):
        qmodel = model.quantize([arrs["x_cal"]], bit_width=8)  # device calibration
    dev_bad = {k for k, p in qmodel.quant_params.items()
               if not np.isfinite(np.float32(p.scale)) or np.float32(p.scale) == 0.0
               or (p.zero_point is not None and int(p.zero_point) == INT64_MIN)}
    assert dev_bad == _degenerate_names(meta["bw8"]["qparams"])
    rec = _Recording(qmodel.quant_params)
    qmodel.quant_params = rec
    # the node loop at batch 1 (the reference's executor)
    qmodel.keep_values = True
    out1 = qmodel([arrs["x_run"]])[0]
    qmodel.keep_values = False
    np.testing.assert_array_equal(out1, arrs["bw8_out"])
    assert rec.seen and not rec.seen & dev_bad, sorted(rec.seen & dev_bad)[:5]
    # the fused plan at the benchmarked batch: plan build (every epilogue's parameters) + forward
    rec.seen.clear()
    model.rebatch(256)
    x = np.random.default_rng(2560).standard_normal((256, 3, 224, 224)).astype(np.float32)
    x[0] = arrs["x_run"][0]
    out = qmodel([x])[0]
    assert qmodel._plan is not None and qmodel._plan.fused == 12
    np.testing.assert_array_equal(out[0], arrs["bw8_out"][0])
    assert rec.seen and not rec.seen & dev_bad, sorted(rec.seen & dev_bad)[:5]
