"""GPU parity of the fused-plan element kernels against NumPy / the oracle on the same
seeded inputs: nqk_ln_quant (LayerNormalization model.py:134-152 -> quantize
numpy_quantization.py:24-34), both the register-tree path (rows of 2, 4 or 8 leaves
of 96 columns) and the LDS path.  Integer outputs: bit-exact."""
import ctypes

import numpy as np
import pytest

from oracle import nq_oracle as O

pytestmark = pytest.mark.gpu


def _ln_ref(x, g, b, eps):
    mean = x.mean(axis=-1, keepdims=True)
    d = x + (-mean)
    var = (d * d).mean(axis=-1, keepdims=True)
    return d * (np.float32(1) / np.sqrt(var + np.float32(eps))) * g + b


@pytest.mark.parametrize("rows,cols", [(1, 768), (257, 768), (1000, 192), (33, 384), (64, 197), (5, 1000),
                                       (3, 96), (7, 3072)])
@pytest.mark.parametrize("bw,zp", [(8, -3), (8, 140), (4, 2)])
def test_ln_quant(rows, cols, bw, zp):
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(rows * cols + bw)
    x = (rng.standard_normal((rows, cols)) * 2 + 0.3).astype(np.float32)
    g = (1 + 0.02 * rng.standard_normal(cols)).astype(np.float32)
    b = (0.02 * rng.standard_normal(cols)).astype(np.float32)
    eps = np.float32(1e-12)
    s = np.float32(0.031) if bw == 8 else np.float32(0.6)
    ref = O.quantize(_ln_ref(x, g, b, eps), bw, s, np.int64(zp))
    dx, dg, db = DeviceArray.from_host(x), DeviceArray.from_host(g), DeviceArray.from_host(b)
    out = DeviceArray((rows, cols), np.int8)
    _lib.call("nqk_ln_quant", dx.vp, dg.vp, db.vp, out.vp, rows, cols, float(eps), float(s), zp, bw)
    np.testing.assert_array_equal(out.to_host().astype(np.int64), ref)


@pytest.mark.parametrize("s_out,zp,bw", [(0.041, -7, 8), (0.0023, 0, 8), (0.31, -3, 4), (1e-5, 100, 8)])
def test_gelu_epilogue_filter_matches_exact_chain(s_out, zp, bw, monkeypatch):
    """FFN-up GEMM with the GELU epilogue (model.py MatMul -> Add -> Div -> Erf -> Add ->
    Mul -> Mul -> quantize): the filtered epilogue (cheap GELU where its proven error
    bound cannot change the rounding, exact chain elsewhere) equals the exact chain
    everywhere.  Small output scales put many values next to rounding boundaries."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, _gemm
    rng = np.random.default_rng(int(s_out * 1e6) + bw)
    M, N, K = 1024 + 77, 3072, 768
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-20, 21, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col = DeviceArray.from_host(bt_h.astype(np.int64).sum(axis=1))
    bias = DeviceArray.from_host((0.02 * rng.standard_normal(N)).astype(np.float32))
    outs = []
    for flag in (None, "1"):
        if flag:
            monkeypatch.setenv("NQK_NO_GELU_FILTER", flag)
        out = DeviceArray((M, N), np.int8)
        e = _lib.Epilogue()
        e.zp_flags, e.bit_width, e.group_cols = _lib.ZP_COL, bw, 1 << 30
        e.zpa, e.col = 5, col.ptr
        e.s_acc[0] = float(np.float32(1.3e-4))
        e.s_out[0], e.zp_out[0], e.out[0] = s_out, zp, out.ptr
        e.bias = bias.ptr
        e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
        _gemm(EPI_GELU, a, bt, 1, M, N, K, K, K, None, 0, 0, e)
        outs.append(out.to_host())
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("n,c,h,w,kh,kw,zp", [(2, 3, 224, 224, 16, 16, -5), (1, 3, 32, 48, 16, 16, 0),
                                             (3, 2, 12, 15, 4, 5, 7), (1, 1, 8, 8, 2, 2, -128)])
def test_patchify_dequant_equals_dequantize_then_im2col(n, c, h, w, kh, kw, zp):
    """Conv input path of the fused patch embedding: dequantize (numpy_quantization.py:37-41)
    then numpy_helper.py:18-70 sliding windows, in one pass over the int8 input."""
    from numpy_quant import _lib
    from numpy_quant import kernels as KM
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(h * w + c)
    q = rng.integers(-128, 128, size=(n, c, h, w), dtype=np.int8)
    s = np.float32(0.0173)
    x = O.dequantize(q.astype(np.int64), s, np.int64(zp) if zp else None)
    ref_cols, _, _ = KM.im2col(DeviceArray.from_host(x), kh, kw, (0, 0, 0, 0), (kh, kw))
    cols = DeviceArray(ref_cols.shape, np.float32)
    _lib.call("nqk_patchify_dequant", DeviceArray.from_host(q).vp, cols.vp, n, c, h, w, kh, kw, float(s), zp)
    np.testing.assert_array_equal(cols.to_host(), ref_cols.to_host())
