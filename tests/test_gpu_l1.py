"""GPU parity, L1: the reference's numpy_quantization / numpy_helper / float-op
functions through the device API, bit-exact against golden vectors generated
from the reference itself (tests/golden/l1.npz)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

L1 = np.load(os.path.join(GOLDEN, "l1.npz"))


@pytest.fixture(scope="module")
def nq():
    from numpy_quant import numpy_quantization as nqz
    from numpy_quant import _lib
    _lib.ensure_init()
    return nqz


def test_quantize(nq):
    x = L1["q_x"]
    for (bw, s, has, zp), ref in zip(L1["q_cases"], L1["q_out"]):
        z = None if has < 0 else (np.int64(0) if zp == 0 else np.array(int(zp), np.int64))
        out = nq.quantize(x, int(bw), np.array(s, np.float32), z)
        np.testing.assert_array_equal(out, ref, err_msg=f"bw={bw} s={s} zp={zp}")


def test_dequantize(nq):
    q, s = L1["dq_in"], L1["dq_s"]
    np.testing.assert_array_equal(nq.dequantize(q, s, None), L1["dq_none"])
    np.testing.assert_array_equal(nq.dequantize(q, s, np.array(-37, np.int64)), L1["dq_scalar"])
    np.testing.assert_array_equal(nq.dequantize(q, s, L1["dq_zrow"]), L1["dq_row"])
    np.testing.assert_array_equal(nq.dequantize(q, s, L1["dq_zfull"]), L1["dq_full"])
    np.testing.assert_array_equal(nq.dequantize(L1["dq_big"], np.array(0.1, np.float32), None), L1["dq_big_out"])


@pytest.mark.parametrize("sfx", ["", "2"])
@pytest.mark.parametrize("tag", ["nn", "an", "na", "aa"])
def test_q_matmul_requantize(nq, tag, sfx):
    a, b = L1["mm_a" + sfx], L1["mm_b" + sfx]
    za = None if tag[0] == "n" else np.array(-9 if tag == "an" else -138, np.int64)
    zb = None if tag[1] == "n" else np.array(5 if tag == "na" else 11, np.int64)
    acc, s, z = nq.q_matmul(a, np.array(0.031, np.float32), za, b, np.array(0.0047, np.float32), zb)
    np.testing.assert_array_equal(acc, L1[f"mm{sfx}_{tag}_acc"])
    assert np.float32(s) == L1[f"mm{sfx}_{tag}_s"]
    ref_z = L1[f"mm{sfx}_{tag}_zp"]
    if z is None:
        assert ref_z.size == 0
    else:
        np.testing.assert_array_equal(np.broadcast_to(z, ref_z.shape), ref_z)
    for rz in (None, np.array(-3, np.int64)):
        for bw in (8, 4):
            out = nq.requantize(acc, s, z, np.array(0.37, np.float32), rz, bw)
            np.testing.assert_array_equal(out, L1[f"rq{sfx}_{tag}_{'n' if rz is None else 'a'}_{bw}"])


def test_float_ops_bit_exact():
    from numpy_quant.tensor import FTensor, fconv2d
    from numpy_quant.model import onnx_operator_implementation as op
    np.testing.assert_array_equal(FTensor(L1["erf_x"]).erf().data, L1["erf_y"])
    y = fconv2d(FTensor(L1["cv_x"]), FTensor(L1["cv_w"]), FTensor(L1["cv_b"]), (0, 2, 2, 1), (2, 1)).data
    np.testing.assert_array_equal(y, L1["cv_y"])
    y = fconv2d(FTensor(L1["cv2_x"]), FTensor(L1["cv2_w"]), FTensor(L1["cv2_b"]), (0, 0, 0, 0), (16, 16)).data
    np.testing.assert_array_equal(y, L1["cv2_y"])
    ln = op("LayerNormalization", [FTensor(L1["ln_x"]), FTensor(L1["ln_g"]), FTensor(L1["ln_b"])],
            {"axis": -1, "epsilon": 9.999999960041972e-13})[0].data
    np.testing.assert_array_equal(ln, L1["ln_y"])
    np.testing.assert_array_equal(op("Softmax", [FTensor(L1["sm_x"])], {"axis": -1})[0].data, L1["sm_y"])
    np.testing.assert_array_equal(op("Sigmoid", [FTensor(L1["sg_x"])], {})[0].data, L1["sg_y"])
    np.testing.assert_array_equal(op("Relu", [FTensor(L1["sg_x"])], {})[0].data, L1["relu_y"])
