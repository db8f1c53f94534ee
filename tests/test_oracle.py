"""The oracle (oracle/nq_oracle.py) against golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only; bit-exact."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from oracle import nq_oracle as O
from numpy_quant import onnx_proto

L1 = np.load(os.path.join(GOLDEN, "l1.npz"))


def test_quant_parameters():
    for mn, mx, bw, asym, s, zp, zp_none, zp_scalar0 in L1["qp_cases"]:
        so, zo = O.quant_parameters(np.float32(mn), np.float32(mx), int(bw), bool(asym))
        assert np.float32(so).view(np.uint32) == np.float32(s).view(np.uint32) or (np.isnan(so) and np.isnan(s))
        assert (zo is None) == bool(zp_none)
        if zo is not None:
            assert int(zo) == int(zp)
            assert (not isinstance(zo, np.ndarray)) == bool(zp_scalar0)


def test_quantize():
    x = L1["q_x"]
    for (bw, s, has, zp), ref in zip(L1["q_cases"], L1["q_out"]):
        z = None if has < 0 else (np.int64(0) if zp == 0 else np.array(int(zp), np.int64))
        out = O.quantize(x, int(bw), np.array(s, np.float32), z)
        np.testing.assert_array_equal(out, ref)


def test_dequantize():
    q, s = L1["dq_in"], L1["dq_s"]
    np.testing.assert_array_equal(O.dequantize(q, s, None), L1["dq_none"])
    np.testing.assert_array_equal(O.dequantize(q, s, np.array(-37, np.int64)), L1["dq_scalar"])
    np.testing.assert_array_equal(O.dequantize(q, s, L1["dq_zrow"]), L1["dq_row"])
    np.testing.assert_array_equal(O.dequantize(q, s, L1["dq_zfull"]), L1["dq_full"])
    np.testing.assert_array_equal(O.dequantize(L1["dq_big"], np.array(0.1, np.float32), None), L1["dq_big_out"])


@pytest.mark.parametrize("sfx", ["", "2"])
@pytest.mark.parametrize("tag", ["nn", "an", "na", "aa"])
def test_q_matmul_requantize(tag, sfx):
    a, b = L1["mm_a" + sfx], L1["mm_b" + sfx]
    za = None if tag[0] == "n" else np.array(-9 if tag == "an" else -138, np.int64)
    zb = None if tag[1] == "n" else np.array(5 if tag == "na" else 11, np.int64)
    acc, s, z = O.q_matmul(a, np.array(0.031, np.float32), za, b, np.array(0.0047, np.float32), zb)
    np.testing.assert_array_equal(acc, L1[f"mm{sfx}_{tag}_acc"])
    assert np.float32(s) == L1[f"mm{sfx}_{tag}_s"]
    ref_z = L1[f"mm{sfx}_{tag}_zp"]
    if z is None:
        assert ref_z.size == 0
    else:
        np.testing.assert_array_equal(np.broadcast_to(z, ref_z.shape), ref_z)
    for rz in (None, np.array(-3, np.int64)):
        for bw in (8, 4):
            out = O.requantize(acc, s, z, np.array(0.37, np.float32), rz, bw)
            np.testing.assert_array_equal(out, L1[f"rq{sfx}_{tag}_{'n' if rz is None else 'a'}_{bw}"])


def test_erf_conv_float_ops():
    np.testing.assert_array_equal(O.erf(L1["erf_x"]), L1["erf_y"])
    np.testing.assert_array_equal(O.conv2d_nchw(L1["cv_x"], L1["cv_w"], L1["cv_b"], (0, 2, 2, 1), (2, 1)), L1["cv_y"])
    np.testing.assert_array_equal(O.conv2d_nchw(L1["cv2_x"], L1["cv2_w"], L1["cv2_b"], (0, 0, 0, 0), (16, 16)),
                                  L1["cv2_y"])
    ln = O._float_op("LayerNormalization", [O.F(L1["ln_x"]), O.F(L1["ln_g"]), O.F(L1["ln_b"])],
                     {"axis": -1, "epsilon": 9.999999960041972e-13})[0][1]
    np.testing.assert_array_equal(ln, L1["ln_y"])
    np.testing.assert_array_equal(O._float_op("Softmax", [O.F(L1["sm_x"])], {"axis": -1})[0][1], L1["sm_y"])
    np.testing.assert_array_equal(O._float_op("Sigmoid", [O.F(L1["sg_x"])], {})[0][1], L1["sg_y"])
    np.testing.assert_array_equal(O._float_op("Relu", [O.F(L1["sg_x"])], {})[0][1], L1["relu_y"])


def _check_qparams(qp, ref):
    for name, r in ref.items():
        p = qp[name]
        assert int(np.asarray(p.scale, np.float32).view(np.uint32)) == r["scale_bits"], name
        if r["zp"] is None:
            assert p.zero_point is None, name
        else:
            assert int(p.zero_point) == r["zp"], name


def test_mlp_all_bit_widths():
    g = np.load(os.path.join(GOLDEN, "mlp.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "mlp_qparams.json")))
    graph = O.Graph(onnx_proto.load(os.path.join(GOLDEN, "..", "..", "numpy-quant_amd", "models", "mlp.onnx")))
    X = g["X"]
    for bw in range(1, 17):
        qp, qc = O.calibrate(graph, [X], bw)
        _check_qparams(qp, meta[f"bw{bw}"]["qparams"])
        vals = O.quantized_forward(graph, qp, qc, [X], bw)
        np.testing.assert_array_equal(O.outputs_of(graph, vals)[0], g[f"bw{bw}_out"])
        if bw in (8, 4):
            for key in g.files:
                if key.startswith(f"bw{bw}|"):
                    _, kind, name = key.split("|", 2)
                    assert vals[name][0] == kind
                    np.testing.assert_array_equal(vals[name][1], g[key], err_msg=name)
