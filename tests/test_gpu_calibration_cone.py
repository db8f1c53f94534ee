"""The calibration cone, now closed on the reference's fixtures.

Model.quantize (reference model.py:328-442) calibrates on a float forward whose MatMuls
are OpenBLAS np.matmul (reference tensor.py:100-101).  The device float forward equals
it bit for bit: every GEMM with more than one row through nqk_sgemm (OpenBLAS's
GEMM_Q = 448 K blocks, k-ordered fma chains), and the one-row classifier Gemm on the CLS
token through nqk_sgemv_t (OpenBLAS's GEMV-T order, oracle/openblas_order.py, with the
fixtures' 8-thread column split, tests/conftest.py).  Values downstream of one-row
products whose order is not restated (tests/test_gpu_models.py:tainted_values) form the
"cone"; for the fixtures below it is empty, so this test asserts:

  * every scale and zero point bit-identical to the reference's (the SCALE_ULPS / |dzp|
    bounds remain the contract for a non-empty cone);
  * the device-calibrated QModel's output on the reference's run input equal to the
    reference's output, bit for bit (north_star's 1e-5 bound for a non-empty cone).

History: round 1 (GEMM_Q = 384, no GEMV order) had 318 of 438 vit_b1 scales off by up to
8 ulps; GEMM_Q = 448 left one (the logits' scale, 4 ulps, from the classifier's GEMV)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from test_gpu_models import tainted_values

pytestmark = pytest.mark.gpu
MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")
SCALE_ULPS = 16
OUT_ATOL = 1e-5           # north_star's tolerance on dequantized float outputs


def _bits(scale):
    return int(np.asarray(scale, np.float32).view(np.uint32))


@pytest.mark.parametrize("tag,fname", [
    ("layer_b1", "vit_image_classifier_encoder_layer_no_weights.onnx"),
    ("vit_b1", "vit_image_classifier_no_weights.onnx"),
])
def test_calibration_cone_is_bounded(tag, fname):
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    meta = json.load(open(os.path.join(GOLDEN, f"{tag}.json")))
    arrs = np.load(os.path.join(GOLDEN, f"{tag}.npz"))
    proto = onnx_proto.load(os.path.join(MODELS, fname), synthetic_weights=True, seed=meta["seed"])
    model = Model.from_onnx(proto)
    bw_key = [k for k in meta if k.startswith("bw")][0]
    bw = int(bw_key[2:])
    qmodel = model.quantize([arrs["x_cal"]], bit_width=bw)
    taint = tainted_values(model)
    ref = meta[bw_key]["qparams"]
    ulps, dzp, outside = [], [], []
    for name, r in ref.items():
        p = qmodel.quant_params[name]
        du = abs(_bits(p.scale) - r["scale_bits"])
        z = None if p.zero_point is None else int(p.zero_point)
        dz = 0 if (z is None and r["zp"] is None) else abs((z or 0) - (r["zp"] or 0))
        if name not in taint:
            if du or dz:
                outside.append(name)
            continue
        ulps.append(du)
        dzp.append(dz)
    assert not outside, f"parameters differing outside the cone: {outside[:8]}"
    n_scale = sum(u > 0 for u in ulps)
    n_zp = sum(d > 0 for d in dzp)
    msg = (f"{tag}: cone of {len(ulps)} parameters: {n_scale} scales differ (max {max(ulps, default=0)} ulps), "
           f"{n_zp} zero points differ (max {max(dzp, default=0)})")
    print(msg)
    assert max(ulps, default=0) <= SCALE_ULPS, msg
    assert max(dzp, default=0) <= 1, msg
    assert not taint, f"{tag}: one-row products outside the restated GEMV order: {sorted(taint)[:8]}"
    assert n_scale == 0 and n_zp == 0, msg
    out = np.asarray(qmodel([arrs["x_run"]])[0], dtype=np.float32)
    want = np.asarray(arrs[f"{bw_key}_out"], dtype=np.float32)
    assert out.shape == want.shape
    diff = np.abs(out - want)
    msg2 = f"{tag}: output |diff| max {diff.max():.3g}, {float(np.mean(diff > 0)):.2%} of {diff.size} elements differ"
    print(msg2)
    assert diff.max() <= OUT_ATOL, msg2
    np.testing.assert_array_equal(out, want)
