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
