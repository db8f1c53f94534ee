"""GPU parity of reference API surfaces outside the node loops, against fixtures recorded
from the reference itself (tests/golden/make_golden.py gen_api -> api.npz / api.json):

  * QTensor.sigmoid (reference tensor.py:217-221) and QTensor.relu (tensor.py:212-215);
  * tensor_min_max / quantize_tensor_min_max (tensor.py:232-242): min / max bits and
    dtypes, scales, zero points and quantized data;
  * Model.quantize of the MLP on ONE calibration sample (model.py:328-442): the float
    forward's one-row Gemms (K = 2, N = 5 and K = 5, N = 2) take OpenBLAS's small-m GEMV-T
    kernels in NumPy (nqk_sgemv_small restates them), so every quantization parameter and
    the QModel's output on the whole set are bit-identical;
  * Model.quantize of the full ViT-Base graph on the bench's 8 calibration images
    (bench.py build_vit, seed 12345): every scale and zero point bit-identical;
  * the profile=True dicts of QModel.__call__ / Model.__call__ have the reference's keys
    (model.py:497-499 / 296)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")


@pytest.fixture(scope="module")
def api():
    return np.load(os.path.join(GOLDEN, "api.npz")), json.load(open(os.path.join(GOLDEN, "api.json")))


def _bits(v):
    return int(np.asarray(v, np.float32).view(np.uint32))


def _zp(z):
    return None if z is None else (np.int64(0) if z == 0 else np.array(z, np.int64))


def test_qtensor_sigmoid(api):
    from numpy_quant.tensor import QTensor
    arrs, meta = api
    for i, c in enumerate(meta["sigmoid"]):
        t = QTensor(arrs[f"sig{i}_q"], c["bw"], np.array(c["scale"], np.float32), _zp(c["zp"]))
        y = t.sigmoid()
        np.testing.assert_array_equal(np.asarray(y.data, np.int64), arrs[f"sig{i}_y"], err_msg=str(c))
        assert _bits(y.scale) == _bits(c["scale"])


def test_qtensor_relu(api):
    from numpy_quant.tensor import QTensor
    arrs, meta = api
    for i, c in enumerate(meta["relu"]):
        q = arrs[f"relu{i}_q"]
        t = QTensor(q, 8, np.array(0.02, np.float32), np.array(c["zp"], np.int64))
        np.testing.assert_array_equal(np.asarray(t.relu().data, np.int64), arrs[f"relu{i}_y"], err_msg=f"zp={c['zp']}")
        # int8 device storage (as the quantize kernels produce it) must give the same values
        from numpy_quant.device import DeviceArray
        t8 = QTensor(DeviceArray.from_host(q.astype(np.int8)), 8, np.array(0.02, np.float32), np.array(c["zp"], np.int64))
        np.testing.assert_array_equal(np.asarray(t8.relu().data, np.int64), arrs[f"relu{i}_y"], err_msg=f"zp={c['zp']} int8")


def test_tensor_min_max_and_quantize_tensor_min_max(api):
    from numpy_quant.tensor import FTensor, quantize_tensor_min_max, tensor_min_max
    arrs, meta = api
    for i, rec in enumerate(meta["minmax"]):
        x = arrs[f"mm{i}_x"]
        mn, mx = tensor_min_max(FTensor(x))
        assert (_bits(mn), _bits(mx)) == (rec["min_bits"], rec["max_bits"]), i
        assert (str(np.asarray(mn).dtype), str(np.asarray(mx).dtype)) == (rec["min_dtype"], rec["max_dtype"])
        for key, want in rec["q"].items():
            bw, asym = (int(v) for v in key.split("_"))
            qt = quantize_tensor_min_max(FTensor(x), bw, bool(asym))
            assert _bits(qt.scale) == want["scale_bits"], (i, key)
            assert (None if qt.zero_point is None else int(qt.zero_point)) == want["zp"], (i, key)
            np.testing.assert_array_equal(np.asarray(qt.data, np.int64), arrs[f"mm{i}_q{key}"], err_msg=f"{i} {key}")


def _check_qparams(qp, ref):
    bad = []
    for name, r in ref.items():
        p = qp[name]
        zp_ok = (p.zero_point is None) if r["zp"] is None else (p.zero_point is not None and int(p.zero_point) == r["zp"])
        if _bits(p.scale) != r["scale_bits"] or not zp_ok:
            bad.append(name)
    assert not bad, bad[:10]


def test_mlp_calibrated_on_one_sample(api):
    from numpy_quant.model import Model
    arrs, meta = api
    X = np.load(os.path.join(GOLDEN, "mlp.npz"))["X"]
    model = Model.from_onnx(os.path.join(MODELS, "mlp.onnx"))
    for i in (0, 7):
        for bw in (8, 4):
            qmodel = model.quantize([X[i:i + 1]], bit_width=bw)
            _check_qparams(qmodel.quant_params, meta["mlp_one_sample"][f"{i}_bw{bw}"])
            np.testing.assert_array_equal(qmodel([X])[0], arrs[f"mlp1_{i}_bw{bw}_out"], err_msg=f"{i} bw{bw}")


def test_vit_calibration_batch_8():
    """The bench's own calibration (8 images) reproduces the reference's parameters."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    meta = json.load(open(os.path.join(GOLDEN, "api.json")))["vit_b8_calibration"]
    proto = onnx_proto.load(os.path.join(MODELS, "vit_image_classifier_no_weights.onnx"), synthetic_weights=True)
    model = Model.from_onnx(proto)
    model.rebatch(8)
    x_cal = np.random.default_rng(meta["seed"]).standard_normal((8, 3, 224, 224)).astype(np.float32)
    qmodel = model.quantize([x_cal], bit_width=8)
    _check_qparams(qmodel.quant_params, meta["qparams"])


def test_profile_dicts_have_the_reference_keys():
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    meta = json.load(open(os.path.join(GOLDEN, "attn_b1.json")))
    arrs = np.load(os.path.join(GOLDEN, "attn_b1.npz"))
    proto = onnx_proto.load(os.path.join(MODELS, "vit_image_classifier_self_attention_no_weights.onnx"),
                            synthetic_weights=True, seed=meta["seed"])
    model = Model.from_onnx(proto)
    qmodel = model.quantize([arrs["x_cal"]], bit_width=8)
    out, prof = qmodel([arrs["x_run"]], profile=True)
    assert sorted(prof) == sorted(meta["bw8"]["profile"])
    assert all(isinstance(v, float) and v >= 0.0 for v in prof.values())
    np.testing.assert_array_equal(out[0], arrs["bw8_out"])
    fout, fprof = model([arrs["x_run"]], profile=True)
    assert sorted(fprof) == sorted({n.op for n in model.nodes})


def test_one_row_kernels_match_numpy_matmul():
    """nqk_sgemv_small (cblas_sdot, every length: the vector kernel from 32 elements) and
    nqk_sgemv_t (GEMV-T: the small-m kernels for K <= 8 per thread chunk of at most 16 384
    columns, the regular kernels otherwise) equal the oracle's restatement of NumPy's orders on
    every column (oracle/openblas_order.py, pinned against np.matmul in the build container by
    tests/test_host.py; the GPU box's own NumPy may run other OpenBLAS kernels), at OpenBLAS
    thread counts 1 and 8 (chunks straddling 16 384 columns included)."""
    from numpy_quant import kernels as K
    from numpy_quant.device import DeviceArray
    from oracle.openblas_order import sdot, sgemv_t
    rng = np.random.default_rng(31)
    cases = [(k, n) for k in (1, 2, 3, 4, 5, 6, 7, 8, 9, 20, 31) for n in (1, 2, 3, 5, 7, 12, 16, 19, 37, 70)]
    cases += [(k, 1) for k in (32, 33, 63, 64, 65, 97, 768, 3072, 10001)]
    cases += [(k, n) for k in (2, 3, 4, 7, 8) for n in (16385, 60001, 131075)]
    old = K.BLAS_THREADS
    try:
        for threads in (1, 8):
            K.BLAS_THREADS = threads
            for k, n in cases:
                x = rng.standard_normal((1, k)).astype(np.float32)
                w = rng.standard_normal((n, k)).astype(np.float32)
                xd, wd = DeviceArray.from_host(x), DeviceArray.from_host(w)
                if n == 1:
                    ref = np.array([sdot(x[0], w[0])], np.float32)
                    got = K.sgemv_small(xd, wd).to_host()[0]
                else:
                    ref = sgemv_t(w, x[0], threads)
                    got = K.sgemv_t(xd, wd).to_host()[0]
                np.testing.assert_array_equal(got.view(np.int32), ref.view(np.int32),
                                              err_msg=f"K={k} N={n} threads={threads}")
    finally:
        K.BLAS_THREADS = old
