"""GPU parity, end to end: Model.from_onnx -> Model.quantize -> QModel.__call__ on
the reference's own graphs, against golden outputs / quantization parameters /
per-value SHA-256 recorded from the reference (tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")


def _check_qparams(qp, ref, strict=True):
    bad = []
    for name, r in ref.items():
        p = qp[name]
        sb = int(np.asarray(p.scale, np.float32).view(np.uint32))
        zp_ok = (p.zero_point is None) if r["zp"] is None else (p.zero_point is not None and int(p.zero_point) == r["zp"])
        if sb != r["scale_bits"] or not zp_ok:
            bad.append(name)
    if strict:
        assert not bad, bad[:10]
    return bad


def _canon(t):
    from numpy_quant.tensor import FTensor, QTensor
    if isinstance(t, QTensor):
        return "Q", np.ascontiguousarray(t.data.astype(np.int64))
    if isinstance(t, FTensor):
        return "F", np.ascontiguousarray(t.data.astype(np.float32))
    return "I", np.ascontiguousarray(np.asarray(t.data))


def test_mlp_all_bit_widths():
    from numpy_quant.model import Model
    g = np.load(os.path.join(GOLDEN, "mlp.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "mlp_qparams.json")))
    X = g["X"]
    model = Model.from_onnx(os.path.join(MODELS, "mlp.onnx"))
    for bw in range(1, 17):
        qmodel = model.quantize([X], bit_width=bw)
        _check_qparams(qmodel.quant_params, meta[f"bw{bw}"]["qparams"])
        out = qmodel([X])[0]
        np.testing.assert_array_equal(out, g[f"bw{bw}_out"], err_msg=f"bw={bw}")
        if bw in (8, 4):
            vals = {v.name: v for v in qmodel.values}
            for key in g.files:
                if key.startswith(f"bw{bw}|"):
                    _, kind, name = key.split("|", 2)
                    k2, arr = _canon(vals[name].data)
                    assert k2 == kind, name
                    np.testing.assert_array_equal(arr, g[key], err_msg=name)


@pytest.mark.parametrize("bw", [8, 4])
def test_mlp_batch_4096_matches_oracle(bw):
    """BASELINE configs[1]: mlp.onnx at batch 4096, inputs U[-1.2, 1.2]
    (seed 4096), calibrated on the committed make_circles X; the device QModel equals the
    oracle's quantized forward bit for bit (the oracle is pinned to the reference's
    vectors by test_oracle.py)."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    from oracle import nq_oracle as O
    X = np.load(os.path.join(GOLDEN, "mlp.npz"))["X"]
    x = np.random.default_rng(4096).uniform(-1.2, 1.2, size=(4096, 2)).astype(np.float32)
    path = os.path.join(MODELS, "mlp.onnx")
    graph = O.Graph(onnx_proto.load(path))
    qp, qc = O.calibrate(graph, [X], bw)
    ref = O.outputs_of(graph, O.quantized_forward(graph, qp, qc, [x], bw))[0]
    qmodel = Model.from_onnx(path).quantize([X], bit_width=bw)
    np.testing.assert_array_equal(qmodel([x])[0], ref)


def ref_qparams(meta_qp):
    """QuantizationParams objects equal (values and types) to the reference's."""
    from numpy_quant.model import QuantizationParams
    out = {}
    for name, r in meta_qp.items():
        scale = np.array(np.uint32(r["scale_bits"]).view(np.float32), dtype=np.float32)
        if r["zp"] is None:
            zp = None
        elif r["zp_is_scalar_zero"]:
            zp = np.int64(r["zp"])
        else:
            zp = np.array(r["zp"], dtype=np.int64)
        out[name] = QuantizationParams(scale, zp)
    return out


def tainted_values(model):
    """Values downstream of a float one-row product (M = 1) whose OpenBLAS order is not
    reproduced.  Since round 6 every one is (kernels.one_row_restated): a one-row Gemm against a
    transposed weight goes to OpenBLAS GEMV-T (its regular or small-m kernels) or sdot for one
    column (nqk_sgemv_t / nqk_sgemv_small), a one-row MatMul against a row-major weight to GEMV-N
    (nqk_sgemv_n), all restated in oracle/openblas_order.py; every GEMM with M > 1, any K, is
    reproduced (OpenBLAS's GEMM_Q = 448 K blocks).  So the set is empty unless
    one_row_restated says otherwise."""
    from numpy_quant.kernels import one_row_restated
    bad = set()
    for node in model.nodes:
        ins = [i.name for i in node.inputs]
        if node.op in ("MatMul", "Gemm"):
            a = node.inputs[0].data
            w = node.inputs[1].data
            if a.dev.ndim >= 2 and a.dev.shape[-2] == 1:
                gemm_t = (node.op == "Gemm" and node.attrs.get("transB") and not node.attrs.get("transA")
                          and a.dev.ndim == 2 and w.dev.ndim == 2)
                n = w.dev.shape[0] if gemm_t else w.dev.shape[-1]
                covered = one_row_restated(n, a.dev.shape[-1])
                if not covered:
                    bad.update(o.name for o in node.outputs)
        if any(i in bad for i in ins):
            bad.update(o.name for o in node.outputs)
            # constants quantized with a tainted value's scale (Gemm / Add biases at 4*bw)
            if node.op in ("Gemm", "Add"):
                bad.update(i.name for i in node.inputs if i.__class__.__name__ == "Constant")
    return bad


@pytest.mark.parametrize("tag,fname,batch", [
    ("attn_b1", "vit_image_classifier_self_attention_no_weights.onnx", 1),
    ("attn_b2", "vit_image_classifier_self_attention_no_weights.onnx", 2),
    ("layer_b1", "vit_image_classifier_encoder_layer_no_weights.onnx", 1),
    ("vit_b1", "vit_image_classifier_no_weights.onnx", 1),
    # configs[4] at the full-classifier level: the reference's Model.quantize(bit_width=4) +
    # QModel.__call__ (round 6, tests/golden/make_golden.py --only vit4)
    ("vit_b1_bw4", "vit_image_classifier_no_weights.onnx", 1),
])
def test_vit_graphs_bit_exact(tag, fname, batch):
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    meta = json.load(open(os.path.join(GOLDEN, f"{tag}.json")))
    arrs = np.load(os.path.join(GOLDEN, f"{tag}.npz"))
    proto = onnx_proto.load(os.path.join(MODELS, fname), synthetic_weights=True, seed=meta["seed"])
    if batch != 1:
        onnx_proto.rebatch(proto, batch)
    model = Model.from_onnx(proto)
    bw_keys = [k for k in meta if k.startswith("bw")]
    for bw_key in bw_keys:
        bw = int(bw_key[2:])
        # 1) device calibration: float forward + min/max + quant_parameters
        qmodel = model.quantize([arrs["x_cal"]], bit_width=bw)
        taint = tainted_values(model)
        if bw_key == bw_keys[0]:
            fbad = []
            for v in model.values:
                if v in model.inputs:
                    continue  # the reference's input Variable is shared with its QModel
                kind, arr = _canon(v.data)
                if hashlib.sha256(arr.tobytes()).hexdigest() != meta["float_hashes"][v.name][2]:
                    fbad.append(v.name)
            assert set(fbad) <= taint, f"float values differing outside the one-row cone: {sorted(set(fbad) - taint)[:8]}"
        qbad = _check_qparams(qmodel.quant_params, meta[bw_key]["qparams"], strict=False)
        assert set(qbad) <= taint, sorted(set(qbad) - taint)[:8]
        if not taint:
            out = qmodel([arrs["x_run"]])[0]
            np.testing.assert_array_equal(out, arrs[f"{bw_key}_out"])
        # 2) QModel.__call__ with the reference's quantization parameters: bit-exact
        qmodel = model.quantize_with(ref_qparams(meta[bw_key]["qparams"]), bit_width=bw)
        qmodel.keep_values = True  # the node loop: every intermediate value is checked
        out = qmodel([arrs["x_run"]])[0]
        np.testing.assert_array_equal(out, arrs[f"{bw_key}_out"])
        hashes = meta[bw_key]["hashes"]
        bad = []
        for v in qmodel.values:
            if v.data is None or v.name not in hashes:
                continue
            kind, arr = _canon(v.data)
            if kind != hashes[v.name][0] or hashlib.sha256(arr.tobytes()).hexdigest() != hashes[v.name][2]:
                bad.append(v.name)
        assert not bad, f"quantized values differing from the reference: {bad[:8]} ({len(bad)})"
