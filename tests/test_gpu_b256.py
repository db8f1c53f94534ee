"""GPU parity at the benchmarked size (BASELINE configs[2] / configs[4]): ViT-Base at
batch 256 through QModel.__call__ (fused plan, two half-batch streams, the GEMMs'
ragged last tiles and XCD tile order at M = 50 432 rows).

With fixed quantization parameters every op of the quantized forward is per image, so
  * image 0, the reference fixture's image, must give the reference's logits
    (tests/golden/vit_b1.npz, recorded from the reference's own QModel.__call__,
    model.py:486-565) bit for bit,
  * the WHOLE [256, 1000] output of the fused two-stream plan must equal one batch-256 run
    of the node-by-node loop (keep_values=True: the reference's executor, pinned to the
    reference by tests/test_gpu_models.py), and
  * the images at both ends of the two stream halves must equal a batch-1 run of the
    same image through the node-by-node loop."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
B = 256
CHECK = (0, 1, B // 2 - 1, B // 2, B - 1)


def _batch(seed_image):
    rng = np.random.default_rng(2560)
    x = rng.standard_normal((B, 3, 224, 224)).astype(np.float32)
    x[0] = seed_image[0]
    return x


def _eager_rows(model, qmodel, x, rows):
    model.rebatch(1)
    qmodel.keep_values = True
    try:
        return {i: qmodel([x[i:i + 1]])[0][0] for i in rows}
    finally:
        qmodel.keep_values = False
        model.rebatch(B)


def _eager_batch(qmodel, x):
    qmodel.keep_values = True
    try:
        return qmodel([x])[0]
    finally:
        qmodel.keep_values = False


def test_vit_b256_int8_matches_reference_fixture():
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    from test_gpu_models import ref_qparams
    meta = json.load(open(os.path.join(GOLDEN, "vit_b1.json")))
    arrs = np.load(os.path.join(GOLDEN, "vit_b1.npz"))
    proto = onnx_proto.load(os.path.join(ROOT, "numpy-quant_amd", "models", "vit_image_classifier_no_weights.onnx"),
                            synthetic_weights=True, seed=meta["seed"])
    model = Model.from_onnx(proto)
    model.rebatch(B)
    qmodel = model.quantize_with(ref_qparams(meta["bw8"]["qparams"]), bit_width=8)
    x = _batch(arrs["x_run"])
    out = qmodel([x])[0]
    plan = qmodel._plan
    assert plan is not None and plan.split and plan.fused == 12 and plan.embeds == 1
    np.testing.assert_array_equal(out[0], arrs["bw8_out"][0])
    np.testing.assert_array_equal(out, _eager_batch(qmodel, x), err_msg="fused B=256 vs node loop B=256")
    for i, ref in _eager_rows(model, qmodel, x, CHECK[1:]).items():
        np.testing.assert_array_equal(out[i], ref, err_msg=f"image {i}")


def test_vit_b256_int4_matches_reference_fixture():
    """configs[4]: the device calibration at bit width 4 gives the reference's quantization
    parameters (tests/golden/vit_b1_bw4.json, the reference's own Model.quantize(bit_width=4)),
    image 0 of the fused B = 256 int4 forward gives the reference's logits bit for bit, and all
    256 rows equal the node loop."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    from test_gpu_models import _check_qparams
    meta = json.load(open(os.path.join(GOLDEN, "vit_b1_bw4.json")))
    arrs = np.load(os.path.join(GOLDEN, "vit_b1_bw4.npz"))
    proto = onnx_proto.load(os.path.join(ROOT, "numpy-quant_amd", "models", "vit_image_classifier_no_weights.onnx"),
                            synthetic_weights=True, seed=meta["seed"])
    model = Model.from_onnx(proto)
    qmodel = model.quantize([arrs["x_cal"]], bit_width=4)  # batch-1 device calibration
    assert not _check_qparams(qmodel.quant_params, meta["bw4"]["qparams"], strict=True)
    model.rebatch(B)
    x = _batch(arrs["x_run"])
    out = qmodel([x])[0]
    plan = qmodel._plan
    assert plan.fused == 12
    np.testing.assert_array_equal(out[0], arrs["bw4_out"][0], err_msg="image 0 vs the reference's int4 logits")
    # the nibble-packed int4 weight images are in use, by the persistent 16x16x64 GEMM (k_pg)
    from numpy_quant import _lib
    layers = [layer for kind, layer in plan.steps if kind == "layer"]
    assert all(layer.bp["1"][1] == 2 for layer in layers)
    assert all(layer.bpg[k] is not None and layer.bpg[k].dtype == np.uint8 for layer in layers for k in layer.bpg)
    assert _lib.load().nqk_qgemm_last_kernel() in (4, 5)  # the last FFN-down GEMM of the forward: k_pg
    np.testing.assert_array_equal(out, _eager_batch(qmodel, x), err_msg="fused B=256 vs node loop B=256")
    for i, ref in _eager_rows(model, qmodel, x, CHECK).items():
        np.testing.assert_array_equal(out[i], ref, err_msg=f"image {i}")
