"""Tensor types of the MI355X backend, mirroring numpy_quant/tensor.py.

  ITensor — int64 shape/index data; stays on the host (shape plumbing).
  FTensor — float32, resident in HBM (DeviceArray).
  QTensor — quantized integers in HBM, narrow storage (int8 for bit widths <= 8),
            with bit_width / scale / zero_point as in the reference (tensor.py:227-293).
            A q_matmul output keeps its zero-point term as a ZpTerm (row/column sums).

`.data` returns a host numpy array exactly like the reference (`QTensor.data` is
int64, `FTensor.data` float32); the device buffer is `.dev`.  Host reads are
lazy D2H copies, so the node loop never leaves the GPU unless asked.
"""
from __future__ import annotations

from typing import Any, Optional, Union

import numpy as np

from . import _lib
from . import kernels as K
from .device import DeviceArray, contiguous_strides, copy_strided, permute


class ITensor:
    """Host int64 tensor (tensor.py:84-116)."""

    def __init__(self, data: np.ndarray):
        self._data = data

    @property
    def data(self):
        return self._data

    def expand_dims(self, axis: "ITensor"):
        return ITensor(np.expand_dims(self._data, axis=tuple(axis.data)))

    @property
    def shape(self):
        return ITensor(np.array(self._data.shape, dtype=np.int64))

    @property
    def size(self):
        return self._data.size

    def __eq__(self, other: "ITensor"):
        return ITensor(np.array(self._data == other.data, np.int64))

    def __getitem__(self, ind):
        return ITensor(self._data.__getitem__(ind))

    def __mul__(self, other: "ITensor"):
        return ITensor(self._data * other.data)

    def reshape(self, shape: "ITensor"):
        return ITensor(self._data.reshape(shape.data))

    def take(self, indices: "ITensor", axis: int):
        return ITensor(self._data.take(np.atleast_1d(indices.data), axis))


def _reshape_target(cur_shape, target) -> tuple[int, ...]:
    """numpy reshape target resolution (one -1 inferred, 0 is a literal 0)."""
    tgt = [int(t) for t in np.atleast_1d(np.asarray(target, dtype=np.int64))] if np.ndim(target) else [int(target)]
    size = int(np.prod(cur_shape, dtype=np.int64))
    if tgt.count(-1) > 1:
        raise ValueError("can only specify one unknown dimension")
    if -1 in tgt:
        known = int(np.prod([t for t in tgt if t != -1], dtype=np.int64))
        if known == 0 or size % known:
            raise ValueError(f"cannot reshape array of size {size} into shape {tuple(tgt)}")
        tgt[tgt.index(-1)] = size // known
    if int(np.prod(tgt, dtype=np.int64)) != size:
        raise ValueError(f"cannot reshape array of size {size} into shape {tuple(tgt)}")
    return tuple(tgt)


class FTensor:
    """float32 tensor in HBM (tensor.py:119-224)."""

    def __init__(self, data: Union[np.ndarray, DeviceArray]):
        if isinstance(data, DeviceArray):
            if data.dtype != np.float32:
                raise ValueError("User np.float32 for FTensor")
            self.dev = data
        else:
            if not data.dtype == np.float32:
                raise ValueError("User np.float32 for FTensor")
            self.dev = DeviceArray.from_host(data)
        self._host = None

    @property
    def data(self) -> np.ndarray:
        if self._host is None:
            self._host = self.dev.to_host()
        return self._host

    @property
    def shape(self):
        return ITensor(np.array(self.dev.shape, dtype=np.int64))

    @property
    def T(self):
        return FTensor(permute(self.dev, list(range(self.dev.ndim))[::-1]))

    def copy(self):
        return FTensor(self.dev.copy())

    def reshape(self, shape: ITensor):
        return FTensor(self.dev.reshape(_reshape_target(self.dev.shape, shape.data)))

    def take(self, indices: ITensor, axis: int):
        return FTensor(take(self.dev, np.asarray(indices.data), axis))

    def transpose(self, *axes):
        perm = axes[0] if len(axes) == 1 and not isinstance(axes[0], int) else axes
        if not perm:
            perm = list(range(self.dev.ndim))[::-1]
        return FTensor(permute(self.dev, list(perm)))

    def __neg__(self):
        return FTensor(K.unary(_lib.NEG, self.dev))

    def __mul__(self, other: "FTensor"):
        if isinstance(other, FTensor):
            return FTensor(K.binary(_lib.MUL, self.dev, other.dev))
        raise ValueError(f"Value of type {type(other)} cannot be multiplied")

    def __add__(self, other: "FTensor"):
        if isinstance(other, FTensor):
            return FTensor(K.binary(_lib.ADD, self.dev, other.dev))
        if isinstance(other, float):
            return FTensor(K.add_scalar(self.dev, other))
        raise ValueError(f"Value of type {type(other)} cannot be added")

    def __radd__(self, other):
        return self.__add__(other)

    def __getitem__(self, ind):
        return FTensor(slice_dev(self.dev, ind))

    def matmul(self, other: "FTensor"):
        return FTensor(K.matmul_f32(self.dev, other.dev))

    def div(self, other: "FTensor"):
        return FTensor(K.binary(_lib.DIV, self.dev, other.dev))

    def erf(self):
        return FTensor(K.unary(_lib.ERF, self.dev))

    def exp(self):
        return FTensor(K.unary(_lib.EXP, self.dev))

    def expand(self, shape: ITensor):
        curr = np.array(self.dev.shape, dtype=np.int64)
        new = np.array(shape.data, dtype=np.int64).copy()
        adjust = np.logical_and(new < curr, new == 1)
        new[adjust] = curr[adjust]
        from .device import materialize_broadcast
        return FTensor(materialize_broadcast(self.dev, tuple(int(v) for v in new)))

    def inv(self):
        return FTensor(K.unary(_lib.RECIP, self.dev))

    def mean(self, axis: int, keepdims: bool):
        axis = axis % self.dev.ndim
        x = self.dev
        if axis != x.ndim - 1:
            perm = [k for k in range(x.ndim) if k != axis] + [axis]
            x = permute(x, perm)
        m = K.mean_lastdim(x)
        shape = list(self.dev.shape)
        shape[axis] = 1
        if not keepdims:
            shape.pop(axis)
        return FTensor(m.reshape(shape))

    def relu(self):
        return FTensor(K.unary(_lib.RELU, self.dev))

    def sigmoid(self):
        return FTensor(K.unary(_lib.SIGMOID, self.dev))

    def softmax(self, axis: int):
        return FTensor(K.softmax(self.dev, axis))

    def sqrt(self):
        return FTensor(K.unary(_lib.SQRT, self.dev))

    def tanh(self):
        return FTensor(K.unary(_lib.TANH, self.dev))


class QTensor:
    """Quantized tensor (tensor.py:227-293).  `dev` holds the integers in narrow
    storage; `zero_point` is None, an int64 scalar, or a ZpTerm (q_matmul output).
    A pending Gemm bias (QTensor.__add__) is applied inside `requantize`."""

    def __init__(self, data: Union[np.ndarray, DeviceArray], bit_width: int, scale: np.float32,
                 zero_point: Optional[Any] = None, bias: Optional["QTensor"] = None):
        if isinstance(data, DeviceArray):
            if data.dtype.kind != "i":
                raise ValueError("Use np.int64 for quantized tensors")
            self.dev = data
        else:
            if data.dtype != np.int64:
                raise ValueError("Use np.int64 for quantized tensors")
            st = K.storage_dtype(bit_width)
            if data.size and (data.min() < np.iinfo(st).min or data.max() > np.iinfo(st).max):
                st = np.dtype(np.int64)
            self.dev = DeviceArray.from_host(data.astype(st))
        if zero_point is not None and not isinstance(zero_point, K.ZpTerm):
            zp = np.asarray(zero_point)
            if zp.dtype != np.int64:
                raise ValueError("Use np.int64 for zero_point of quantized tensors")
            if zp.ndim:
                raise ValueError("array zero points are only produced by q_matmul (ZpTerm)")
        self.bit_width = bit_width
        self.scale = scale
        self._zero_point = zero_point
        self._bias = bias
        self._bt = None  # cached (Bt, colsum) when this is a constant weight

    @property
    def shape(self):
        return self.dev.shape

    @property
    def zero_point(self):
        zp = self._zero_point
        if isinstance(zp, K.ZpTerm):
            return zp.to_host()
        return zp

    @property
    def zp_scalar(self) -> Optional[int]:
        zp = self._zero_point
        if zp is None:
            return None
        if isinstance(zp, K.ZpTerm):
            raise ValueError("q_matmul output cannot be a q_matmul operand (bit width 4*bw)")
        return int(zp)

    @property
    def data(self) -> np.ndarray:
        d = self.dev.to_host().astype(np.int64)
        if self._bias is not None:
            d = d + self._bias.data
        return d

    @property
    def T(self):
        if isinstance(self._zero_point, K.ZpTerm) or self._bias is not None:
            raise ValueError("transpose of a q_matmul output is not on the QModel path")
        return QTensor(permute(self.dev, list(range(self.dev.ndim))[::-1]), self.bit_width, self.scale,
                       self._zero_point)

    def reshape(self, shape: ITensor):
        return QTensor(self.dev.reshape(_reshape_target(self.dev.shape, shape.data)), self.bit_width,
                       self.scale, self._zero_point, self._bias)

    def transpose(self, *axes):
        perm = axes[0] if len(axes) == 1 and not isinstance(axes[0], int) else axes
        return QTensor(permute(self.dev, list(perm)), self.bit_width, self.scale, self._zero_point)

    def __add__(self, other: "QTensor"):
        if isinstance(other, QTensor):
            if self._bias is not None:
                raise ValueError("only one pending bias is supported")
            return QTensor(self.dev, self.bit_width, self.scale, self._zero_point, bias=other)
        raise ValueError(f"Cannot add QTensor with {other.__class__}")

    def dequantize(self):
        if self._bias is not None:
            raise ValueError("dequantize of a biased Gemm accumulator: requantize it first")
        return FTensor(K.dequantize(self.dev, self.scale, self._zero_point))

    def requantize(self, bit_width: int, scale: np.float32, zero_point):
        bias = None
        if self._bias is not None:
            bias = self._bias.dev
        q = K.requantize(self.dev, self.scale, self._zero_point, bias, scale,
                         None if zero_point is None else int(zero_point), bit_width)
        return QTensor(q, bit_width, scale, zero_point)

    def weight_operand(self):
        """(Bt, colsum) of a constant int8 weight, computed once."""
        if self._bt is None:
            self._bt = K.weight_bt(self.dev)
        return self._bt

    def matmul(self, other: "QTensor"):
        assert self.bit_width == other.bit_width, f"{self.bit_width} != {other.bit_width}"
        bt = col = None
        if other._bt is not None or getattr(other, "_is_weight", False):
            if other.dev.dtype == np.int8 and other.dev.ndim == 2:
                bt, col = other.weight_operand()
        acc, zt = K.qmatmul(self.dev, other.dev, self.zp_scalar, other.zp_scalar, bt, col)
        scale = np.float32(self.scale) * np.float32(other.scale)
        return QTensor(acc, 4 * self.bit_width, scale, zt)

    def relu(self):
        """tensor.py:212-215: values below the zero point become the zero point (the
        dequantized value is clamped at 0).  The reference compares with a scalar zero
        point; without one its comparison with None raises TypeError, and so does this."""
        zp = self._zero_point
        if zp is None:
            raise TypeError("'<' not supported between instances of 'numpy.ndarray' and 'NoneType'")
        if isinstance(zp, K.ZpTerm) or self._bias is not None:
            raise ValueError("relu of a q_matmul accumulator is not on the QModel path")
        zp = int(zp)
        st = self.dev.dtype
        info = np.iinfo(st)
        if not (info.min <= zp <= info.max):
            st = np.dtype(np.int64)  # the zero point itself must be storable
        out = DeviceArray(self.dev.shape, st)
        from .device import dtype_code
        _lib.call("nqk_relu_q", self.dev.vp, dtype_code(self.dev.dtype), out.vp, dtype_code(st), self.dev.size, zp)
        return QTensor(out, self.bit_width, self.scale, self._zero_point)

    def sigmoid(self):
        act = self.dequantize().sigmoid()
        return quantize_tensor(act, self.bit_width, self.scale, self.zero_point)


Tensor = Union[ITensor, FTensor, QTensor]


def quantize_tensor(tensor: FTensor, bit_width: int, scale: np.float32, zero_point):
    """tensor.py:299-301 on device."""
    q, _ = K.quantize(tensor.dev, bit_width, scale, None if zero_point is None else int(zero_point))
    return QTensor(q, bit_width, scale=scale, zero_point=zero_point)


def tensor_min_max(tensor: Tensor):
    """tensor.py:304-308: global min/max clamped to include 0."""
    zero_val = np.array(0.0).astype(np.float32)
    if isinstance(tensor, FTensor):
        mn, mx = K.minmax(tensor.dev)
    else:
        mn, mx = tensor.data.min(), tensor.data.max()
    return np.minimum(mn, zero_val), np.maximum(mx, zero_val)


def quantize_tensor_min_max(tensor: Tensor, bit_width: int, asymmetric: bool):
    from .numpy_quantization import quant_parameters
    min_val, max_val = tensor_min_max(tensor)
    scale, zero_point = quant_parameters(min_val, max_val, bit_width, asymmetric)
    return quantize_tensor(tensor, bit_width, scale, zero_point)


def concat(x_list: list[Tensor], axis: int):
    assert all(x.__class__ == x_list[0].__class__ for x in x_list), (
        f"types {[x.__class__ for x in x_list]} of x_list entries do no match")
    if isinstance(x_list[0], ITensor):
        return ITensor(np.concatenate([x.data for x in x_list], axis=axis))
    if isinstance(x_list[0], QTensor):
        raise ValueError("Concat of quantized tensors is not on the QModel path")
    devs = [x.dev for x in x_list]
    nd = devs[0].ndim
    axis %= nd
    for d in devs[1:]:
        if d.ndim != nd or any(d.shape[k] != devs[0].shape[k] for k in range(nd) if k != axis):
            raise ValueError("all the input array dimensions except for the concatenation axis must match "
                             f"exactly ({devs[0].shape} vs {d.shape}, axis {axis})")
    out_shape = list(devs[0].shape)
    out_shape[axis] = sum(d.shape[axis] for d in devs)
    out = DeviceArray(out_shape, np.float32)
    ost = contiguous_strides(out_shape)
    off = 0
    for d in devs:
        copy_strided(d, out, d.shape, contiguous_strides(d.shape), ost, 0, off * ost[axis])
        off += d.shape[axis]
    return FTensor(out)


def where(condition: ITensor, a: Tensor, b: Tensor):
    assert a.__class__ == b.__class__, f"types {a.__class__} and {b.__class__} do not match"
    if isinstance(a, ITensor):
        return ITensor(np.where(condition.data, a.data, b.data))
    if isinstance(a, QTensor):
        raise ValueError("Where of quantized tensors is not on the QModel path")
    return FTensor(K.where(condition.data, a.dev, b.dev))


def fconv2d(x: FTensor, w: FTensor, b: FTensor, pads, strides):
    """tensor.py:328-336 + numpy_helper.conv2d: im2col + BLAS-order f32 GEMM + bias."""
    n, c, h, wd = x.dev.shape
    kout, c2, kh, kw = w.dev.shape
    if c != c2:
        raise ValueError("Conv channel mismatch")
    cols, ho, wo = K.im2col(x.dev, kh, kw, tuple(int(p) for p in pads), tuple(int(s) for s in strides))
    # weight matrix [(kh, kw, c), kout] = w.transpose(2, 3, 1, 0)
    wm = permute(w.dev, [2, 3, 1, 0]).reshape((kh * kw * c, kout))
    kk = kh * kw * c
    y = K.sgemm(cols, kk, 1, wm, kout, 1, n * ho * wo, kout, kk)  # [n*ho*wo, kout]
    # NHWC -> NCHW fused with the bias add
    out_shape = (n, kout, ho, wo)
    y_st = [ho * wo * kout, 1, wo * kout, kout]
    out = DeviceArray(out_shape, np.float32)
    from .device import collapse
    bst = [0, 1, 0, 0]
    shp, (sa, sb) = collapse(out_shape, y_st, bst)
    _lib.call("nqk_binary_f32", _lib.ADD, y.vp, b.dev.vp, out.vp, len(shp), _lib.i64arr(shp), _lib.i64arr(sa),
              _lib.i64arr(sb))
    return FTensor(out)


# ----------------------------------------------------------------------------- device views
def take(x: DeviceArray, indices: np.ndarray, axis: int) -> DeviceArray:
    """ndarray.take along one axis (ITensor indices on the host)."""
    axis %= x.ndim
    idx = np.asarray(indices, dtype=np.int64)
    flat = idx.reshape(-1)
    n_ax = x.shape[axis]
    flat = np.where(flat < 0, flat + n_ax, flat)
    if flat.size and (flat.min() < 0 or flat.max() >= n_ax):
        raise IndexError("index out of bounds")
    out_shape = x.shape[:axis] + idx.shape + x.shape[axis + 1:]
    out = DeviceArray(out_shape, x.dtype)
    xs = contiguous_strides(x.shape)
    piece = x.shape[:axis] + x.shape[axis + 1:]
    ost_full = contiguous_strides(x.shape[:axis] + (flat.size,) + x.shape[axis + 1:])
    src_st = xs[:axis] + xs[axis + 1:]
    dst_st = ost_full[:axis] + ost_full[axis + 1:]
    for j, i in enumerate(flat):
        copy_strided(x, out, piece, src_st, dst_st, int(i) * xs[axis], j * ost_full[axis])
    return out


def slice_dev(x: DeviceArray, ind) -> DeviceArray:
    if not isinstance(ind, tuple):
        ind = (ind,)
    starts, shape, steps = [], [], []
    for k, n in enumerate(x.shape):
        s = ind[k] if k < len(ind) else slice(None)
        if not isinstance(s, slice):
            raise ValueError("only slice indexing is supported on device tensors")
        a, b, st = s.indices(n)
        starts.append(a)
        steps.append(st)
        shape.append(max(0, (b - a + (st - (1 if st > 0 else -1))) // st))
    xs = contiguous_strides(x.shape)
    out = DeviceArray(shape, x.dtype)
    off = sum(a * s for a, s in zip(starts, xs))
    copy_strided(x, out, shape, [s * st for s, st in zip(xs, steps)], contiguous_strides(shape), off, 0)
    return out
