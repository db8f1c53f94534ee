"""GPU parity of the strided / broadcast element kernels (Transpose, Reshape-copies,
Expand, Concat, Add/Sub/Mul/Div with NumPy broadcasting — model.py:65-213) against
NumPy on the same inputs: bit-exact, on shapes whose extents are not powers of two
(the 32-bit magic-number divmod of the index decomposition)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PERMS = [((2, 768, 196), (0, 2, 1)), ((3, 5, 7, 11), (0, 2, 1, 3)), ((4, 197, 12, 64), (0, 2, 1, 3)),
         ((2, 12, 197, 64), (0, 2, 3, 1)), ((1, 1, 5), (2, 0, 1)), ((6, 1, 9, 2), (3, 2, 1, 0))]


@pytest.mark.parametrize("shape,perm", PERMS)
@pytest.mark.parametrize("dtype", [np.float32, np.int8, np.int64])
def test_permute(shape, perm, dtype):
    from numpy_quant.device import DeviceArray, permute
    rng = np.random.default_rng(len(shape))
    x = (rng.standard_normal(shape) * 50).astype(dtype)
    out = permute(DeviceArray.from_host(x), perm).to_host()
    np.testing.assert_array_equal(out, np.ascontiguousarray(np.transpose(x, perm)))


BCAST = [((2, 768, 196), (768, 1)), ((5, 197, 768), (1, 197, 768)), ((3, 1, 7), (1, 4, 1)), ((13,), ()),
         ((2, 3, 4, 5, 6), (3, 1, 5, 1)), ((1000,), (1000,))]


@pytest.mark.parametrize("sa,sb", BCAST)
@pytest.mark.parametrize("op", ["Add", "Sub", "Mul", "Div"])
def test_broadcast_binary(sa, sb, op):
    from numpy_quant import kernels as K
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(7)
    a = rng.standard_normal(sa).astype(np.float32)
    b = (rng.standard_normal(sb) + 3).astype(np.float32)
    code = {"Add": _lib.ADD, "Sub": _lib.SUB, "Mul": _lib.MUL, "Div": _lib.DIV}[op]
    ref = {"Add": np.add, "Sub": np.subtract, "Mul": np.multiply, "Div": np.divide}[op](a, b)
    out = K.binary(code, DeviceArray.from_host(a), DeviceArray.from_host(b)).to_host()
    np.testing.assert_array_equal(out, ref)
