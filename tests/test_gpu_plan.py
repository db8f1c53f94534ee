"""GPU parity of the fused device plan (plan.py): the fused encoder layers must
reproduce the eager node loop — and therefore the reference — bit for bit."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")


def _vit(batch, seed=0):
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    proto = onnx_proto.load(os.path.join(MODELS, "vit_image_classifier_no_weights.onnx"), synthetic_weights=True,
                            seed=seed)
    if batch != 1:
        onnx_proto.rebatch(proto, batch)
    return Model.from_onnx(proto)


def test_plan_matches_reference_vit_b1():
    from test_gpu_models import ref_qparams
    meta = json.load(open(os.path.join(GOLDEN, "vit_b1.json")))
    arrs = np.load(os.path.join(GOLDEN, "vit_b1.npz"))
    model = _vit(1, meta["seed"])
    qmodel = model.quantize_with(ref_qparams(meta["bw8"]["qparams"]), bit_width=8)
    plan = qmodel.compile()
    assert plan.fused == 12 and plan.embeds == 1 and plan.pushdowns == 1
    out = qmodel([arrs["x_run"]])[0]
    np.testing.assert_array_equal(out, arrs["bw8_out"])
    # every layer output (residual stream) equals the reference's value
    hashes = meta["bw8"]["hashes"]
    for step, layer in [s for s in plan.steps if s[0] == "layer"]:
        v = layer.m.x_out
        arr = np.ascontiguousarray(v.data.data)
        assert hashlib.sha256(arr.tobytes()).hexdigest() == hashes[v.name][2], v.name


@pytest.mark.parametrize("batch,bw", [(3, 8), (2, 4)])
def test_plan_equals_eager(batch, bw):
    rng = np.random.default_rng(batch)
    x = rng.standard_normal((batch, 3, 224, 224)).astype(np.float32)
    model = _vit(batch)
    qmodel = model.quantize([x], bit_width=bw)
    qmodel.keep_values = True
    eager = qmodel([x])[0]
    qmodel.keep_values = False
    layer_outs = {}
    plan = qmodel.compile()
    assert plan.fused == 12 and plan.embeds == 1 and plan.pushdowns == 1
    for _, layer in [s for s in plan.steps if s[0] == "layer"]:
        layer_outs[layer.m.x_out.name] = None
    fused = qmodel([x])[0]
    np.testing.assert_array_equal(fused, eager)


def test_plan_encoder_layer_graph_matches_oracle():
    """The encoder-layer graph: a quantized graph input feeds the fused layer, and the
    second LayerNorm's parameters come through Identity nodes (shared by the exporter)."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model, QuantizationParams
    from oracle import nq_oracle as O
    path = os.path.join(MODELS, "vit_image_classifier_encoder_layer_no_weights.onnx")
    x = np.random.default_rng(5).standard_normal((1, 197, 768)).astype(np.float32)
    graph = O.Graph(onnx_proto.load(path, synthetic_weights=True))
    with np.errstate(all="ignore"):
        qp, qc = O.calibrate(graph, [x], 8)
        ref = O.outputs_of(graph, O.quantized_forward(graph, qp, qc, [x], 8))[0]
    model = Model.from_onnx(onnx_proto.load(path, synthetic_weights=True))
    qmodel = model.quantize_with({k: QuantizationParams(v.scale, v.zero_point) for k, v in qp.items()}, bit_width=8)
    qmodel.keep_values = True
    np.testing.assert_array_equal(qmodel([x])[0], ref)
    qmodel.keep_values = False
    plan = qmodel.compile()
    assert plan.fused == 1
    np.testing.assert_array_equal(qmodel([x])[0], ref)


def _split_vs_one_stream(qmodel, x):
    plan = qmodel.compile()
    assert plan.split
    two = qmodel([x])[0]
    plan.split = False
    one = qmodel([x])[0]
    plan.split = True
    return plan, two, one


def test_plan_split_with_unsplit_layers(monkeypatch):
    """Split embedding followed by layers that run whole-batch (three-launch attention):
    the layers must wait for both embedding halves (plan.Streams.join)."""
    from numpy_quant import plan as P
    monkeypatch.setattr(P, "FUSED_ATTENTION", False)
    x = np.random.default_rng(11).standard_normal((3, 3, 224, 224)).astype(np.float32)
    model = _vit(3)
    qmodel = model.quantize([x], bit_width=8)
    qmodel.keep_values = True
    eager = qmodel([x])[0]
    qmodel.keep_values = False
    plan, two, one = _split_vs_one_stream(qmodel, x)
    assert plan.fused == 12 and not any(l.attn_fused for k, l in plan.steps if k == "layer")
    np.testing.assert_array_equal(two, eager)
    np.testing.assert_array_equal(one, eager)


def test_plan_encoder_layer_graph_batch2_split():
    """A quantized graph input feeding a split layer: its whole-batch dequantize on
    stream 0 must precede the stream-1 half (fork after the dequantize)."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    path = os.path.join(MODELS, "vit_image_classifier_encoder_layer_no_weights.onnx")
    x = np.random.default_rng(6).standard_normal((2, 197, 768)).astype(np.float32)
    proto = onnx_proto.load(path, synthetic_weights=True)
    onnx_proto.rebatch(proto, 2)
    qmodel = Model.from_onnx(proto).quantize([x], bit_width=8)
    qmodel.keep_values = True
    eager = qmodel([x])[0]
    qmodel.keep_values = False
    plan, two, one = _split_vs_one_stream(qmodel, x)
    assert plan.fused == 1
    for _ in range(3):
        np.testing.assert_array_equal(qmodel([x])[0], eager)
    np.testing.assert_array_equal(two, eager)
    np.testing.assert_array_equal(one, eager)


def test_plan_restores_stream_after_error():
    """An exception inside a split half leaves the library on stream 0 and joined."""
    from numpy_quant import _lib
    from numpy_quant.plan import Streams
    s = Streams(True)

    def boom(s_idx, i0, nb):
        if s_idx == 1:
            raise RuntimeError("boom")

    with pytest.raises(RuntimeError):
        s.halves(4, boom)
    s.join()
    import ctypes
    cur, base = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.call("nqk_stream", ctypes.byref(cur))
    _lib.call("nqk_set_stream", 0)
    _lib.call("nqk_stream", ctypes.byref(base))
    assert cur.value == base.value


def test_vit_tiny_fused_plan_matches_node_loop_and_oracle():
    """The metric's ViT-tiny (the reference's ViT graph re-dimensioned to ViT-Ti/16 by
    onnx_proto.redimension: width 192, 3 heads of 64, MLP 768): the fused plan at batch 3
    equals the node-by-node loop image by image, and batch 1 equals the oracle's
    restatement of the reference (quantized forward with the oracle's calibration) bit
    for bit."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model, QuantizationParams
    from oracle import nq_oracle as O
    path = os.path.join(MODELS, "vit_image_classifier_no_weights.onnx")
    rng = np.random.default_rng(21)
    x = rng.standard_normal((3, 3, 224, 224)).astype(np.float32)
    proto = onnx_proto.load(path, synthetic_weights=True)
    assert onnx_proto.redimension(proto, 192, 3, 768) > 0
    graph = O.Graph(proto)
    with np.errstate(all="ignore"):
        qp, qc = O.calibrate(graph, [x[:1]], 8)
        ref = O.outputs_of(graph, O.quantized_forward(graph, qp, qc, [x[:1]], 8))[0]
    model = Model.from_onnx(proto)
    # the oracle's parameters (its calibration runs the box's own OpenBLAS, whose kernel
    # family may differ from the fixtures' host; device calibration is pinned there)
    qmodel = model.quantize_with({k: QuantizationParams(v.scale, v.zero_point) for k, v in qp.items()}, bit_width=8)
    qmodel.keep_values = True
    np.testing.assert_array_equal(qmodel([x[:1]])[0], ref)
    model.rebatch(3)
    eager = qmodel([x])[0]
    qmodel.keep_values = False
    plan = qmodel.compile()
    assert plan.fused == 12
    out = qmodel([x])[0]
    np.testing.assert_array_equal(out, eager)
    np.testing.assert_array_equal(out[:1], ref)


def test_fused_run_leaves_no_stale_intermediates():
    """after an eager keep_values run, a fused run with other inputs must not
    leave the eager run's tensors in the values its steps compute internally: every value
    either holds this run's tensor or raises on access (plan.FusedAway)."""
    from numpy_quant.plan import FusedAway
    rng = np.random.default_rng(7)
    x1 = rng.standard_normal((2, 3, 224, 224)).astype(np.float32)
    x2 = rng.standard_normal((2, 3, 224, 224)).astype(np.float32)
    model = _vit(2)
    qmodel = model.quantize([x1], bit_width=8)
    qmodel.keep_values = True
    qmodel([x1])
    before = {id(v): v.data for v in qmodel.values}
    qmodel.keep_values = False
    qmodel.compile()
    out2 = qmodel([x2])[0]
    stale = []
    for v in qmodel.values:
        ins = getattr(v, "inputs", None)
        if not ins or ins[0].op == "Constant":  # Constant values / Constant-node outputs persist
            continue
        if v in qmodel.inputs:
            continue
        if v.data is before[id(v)] and v.data is not None:
            stale.append(v.name)
    assert not stale, stale[:10]
    n_away = sum(isinstance(v.data, FusedAway) for v in qmodel.values)
    assert n_away > 100
    with pytest.raises(RuntimeError):
        next(v for v in qmodel.values if isinstance(v.data, FusedAway)).data.data
    # and an eager run of x2 gives the same output
    qmodel.keep_values = True
    np.testing.assert_array_equal(qmodel([x2])[0], out2)
