"""L1 quantization API of numpy_quant/numpy_quantization.py:7-72, on the GPU.

Same names, arguments and results as the reference (NumPy arrays in and out), so
code written against the reference module runs unchanged; the arithmetic runs in
libnqk.so kernels.  `quant_parameters` is scalar host logic (calibration), kept
in NumPy with the reference's exact float32 scalar semantics.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from . import kernels as K
from .device import DeviceArray, materialize_broadcast


def quant_parameters(min_val: np.float32, max_val: np.float32, bit_width: int, asymmetric: bool):
    """numpy_quantization.py:7-21 (scalar host math, NumPy float32 semantics)."""
    lo = -(2.0 ** (bit_width - 1))
    hi = 2.0 ** (bit_width - 1) - 1.0
    if asymmetric:
        scale = (max_val - min_val) / (hi - lo)
        zp = np.rint(lo - min_val / scale).astype(np.int64)
    else:
        scale = (2 * max(max_val, min_val)) / (hi - lo)
        zp = None
    scale = np.array(scale, dtype=np.float32)
    if zp is not None and zp:
        zp = np.array(zp, dtype=np.int64)
    return scale, zp


def _zp_dev(zero_point, shape):
    """A broadcast int64 zero-point array as a flat device array (NQK_ZP_FULL)."""
    z = DeviceArray.from_host(np.asarray(zero_point, dtype=np.int64))
    return materialize_broadcast(z, tuple(shape))


def quantize(data: np.ndarray, bit_width: int, scale, zero_point) -> np.ndarray:
    """numpy_quantization.py:24-34."""
    x = DeviceArray.from_host(np.asarray(data, dtype=np.float32))
    q, _ = K.quantize(x, bit_width, scale, None if zero_point is None else int(zero_point),
                      out_dtype=np.int64)
    return q.to_host()


def _dequant_dev(arr: np.ndarray, scale, zero_point) -> DeviceArray:
    a = np.asarray(arr, dtype=np.int64)
    zp = None if zero_point is None else np.asarray(zero_point, dtype=np.int64)
    shape = np.broadcast_shapes(a.shape, zp.shape) if zp is not None else a.shape
    q = DeviceArray.from_host(np.broadcast_to(a, shape))
    if zp is None or zp.ndim == 0:
        return q, (None if zp is None else int(zp))
    return q, ("full", _zp_dev(zp, shape))


def dequantize(arr: np.ndarray, scale, zero_point) -> np.ndarray:
    """numpy_quantization.py:37-41."""
    q, zp = _dequant_dev(arr, scale, zero_point)
    if isinstance(zp, tuple):
        out = DeviceArray(q.shape, np.float32)
        _lib.call("nqk_dequantize", q.vp, q.code, out.vp, 1, 1, q.size, float(np.float32(scale)), _lib.ZP_FULL,
                  0, 0, 0, 0, zp[1].vp, None, None)
        return out.to_host()
    return K.dequantize(q, scale, zp).to_host()


def q_matmul(arr_a: np.ndarray, scale_a, zero_point_a, arr_b: np.ndarray, scale_b, zero_point_b):
    """numpy_quantization.py:44-61: (int64 product, s_a*s_b, zero-point term)."""
    a = np.asarray(arr_a, dtype=np.int64)
    b = np.asarray(arr_b, dtype=np.int64)
    lim = np.iinfo(np.int8)
    narrow = (a.size == 0 or (a.min() >= lim.min and a.max() <= lim.max)) and \
             (b.size == 0 or (b.min() >= lim.min and b.max() <= lim.max))
    dt = np.int8 if narrow else np.int64
    da = DeviceArray.from_host(a.astype(dt))
    db = DeviceArray.from_host(b.astype(dt))
    za = None if zero_point_a is None else int(zero_point_a)
    zb = None if zero_point_b is None else int(zero_point_b)
    acc, zt = K.qmatmul(da, db, za, zb)
    scale = scale_a * scale_b
    return acc.to_host().astype(np.int64), scale, (None if zt is None else zt.to_host())


def requantize(arr: np.ndarray, arr_scale, arr_zero_points, res_scale, res_zero_point, bit_width: int):
    """numpy_quantization.py:64-72."""
    q, zp = _dequant_dev(arr, arr_scale, arr_zero_points)
    rz = None if res_zero_point is None else int(res_zero_point)
    out = DeviceArray(q.shape, np.int64)
    if isinstance(zp, tuple):
        flags, z, row = _lib.ZP_FULL, 0, zp[1].vp
    elif zp is None:
        flags, z, row = _lib.ZP_NONE, 0, None
    else:
        flags, z, row = _lib.ZP_SCALAR, zp, None
    _lib.call("nqk_requantize", q.vp, q.code, None, _lib.NQK_I64, out.vp, out.code, 1, 1, q.size,
              float(np.float32(arr_scale)), flags, z, 0, 0, 0, row, None, None, float(np.float32(res_scale)),
              0 if rz is None else rz, 0 if rz is None else 1, int(bit_width))
    return out.to_host()
