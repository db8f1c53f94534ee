"""Device memory for the MI355X backend: a size-bucketed caching allocator on top of
nqk_malloc (hipMalloc synchronises the device, so buffers are recycled instead of
freed) and `DeviceArray`, a contiguous n-d buffer with a numpy dtype.

All arrays are C-contiguous.  Strided views of the reference (transposes, slices,
broadcasts — tensor.py:133-191) are materialised with `nqk_copy_strided`.
"""
from __future__ import annotations

import ctypes
import math
import weakref
from typing import Sequence

import numpy as np

from . import _lib

_DTYPE_CODE = {np.dtype(np.int8): _lib.NQK_I8, np.dtype(np.int16): _lib.NQK_I16,
               np.dtype(np.int32): _lib.NQK_I32, np.dtype(np.int64): _lib.NQK_I64,
               np.dtype(np.float32): _lib.NQK_F32}


def dtype_code(dt) -> int:
    return _DTYPE_CODE[np.dtype(dt)]


class _Pool:
    """Caching allocator: blocks are rounded up (256 B granule, then to 1/8 of the
    next power of two) and kept on per-size free lists after release."""

    def __init__(self):
        self.free: dict[int, list[int]] = {}
        self.live_bytes = 0
        self.cached_bytes = 0
        self.peak_bytes = 0
        # during a hipGraph capture (graph.py) every new block is appended here, so the
        # graph holds it and the pool never hands it out while the graph can replay
        self.capture: list | None = None

    @staticmethod
    def round(nbytes: int) -> int:
        n = max(256, (nbytes + 255) // 256 * 256)
        if n > (1 << 20):
            step = 1 << max(8, (n.bit_length() - 4))
            n = (n + step - 1) // step * step
        return n

    def alloc(self, nbytes: int) -> tuple[int, int]:
        size = self.round(nbytes)
        lst = self.free.get(size)
        if lst:
            ptr = lst.pop()
            self.cached_bytes -= size
        else:
            p = ctypes.c_void_p()
            try:
                _lib.call("nqk_malloc", ctypes.byref(p), size)
            except _lib.NQKError:
                self.trim()
                _lib.call("nqk_malloc", ctypes.byref(p), size)
            ptr = p.value
        self.live_bytes += size
        self.peak_bytes = max(self.peak_bytes, self.live_bytes)
        return ptr, size

    def release(self, ptr: int, size: int) -> None:
        self.live_bytes -= size
        self.cached_bytes += size
        self.free.setdefault(size, []).append(ptr)

    def trim(self) -> None:
        _lib.call("nqk_sync")
        for lst in self.free.values():
            for ptr in lst:
                _lib.call("nqk_free", ctypes.c_void_p(ptr))
        self.free.clear()
        self.cached_bytes = 0


POOL = _Pool()


class _Block:
    __slots__ = ("ptr", "size", "__weakref__")

    def __init__(self, nbytes: int):
        _lib.ensure_init()
        self.ptr, self.size = POOL.alloc(max(1, nbytes))
        weakref.finalize(self, POOL.release, self.ptr, self.size)
        if POOL.capture is not None:
            POOL.capture.append(self)


class DeviceArray:
    """Contiguous device buffer with numpy shape/dtype.  `base` keeps a parent
    block alive for views (reshape, offset slices)."""

    __slots__ = ("block", "ptr", "shape", "dtype")

    def __init__(self, shape: Sequence[int], dtype, block: _Block | None = None, ptr: int | None = None):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        if block is None:
            block = _Block(self.nbytes)
        self.block = block
        self.ptr = block.ptr if ptr is None else ptr

    # ---------------------------------------------------------------- properties
    @property
    def size(self) -> int:
        return int(math.prod(self.shape))

    @property
    def nbytes(self) -> int:
        return self.size * self.dtype.itemsize

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def vp(self) -> ctypes.c_void_p:
        return ctypes.c_void_p(self.ptr)

    @property
    def code(self) -> int:
        return dtype_code(self.dtype)

    def strides(self) -> tuple[int, ...]:
        return contiguous_strides(self.shape)

    # ---------------------------------------------------------------- transfers
    @classmethod
    def from_host(cls, arr: np.ndarray, dtype=None) -> "DeviceArray":
        a = np.ascontiguousarray(arr, dtype=dtype)
        d = cls(a.shape, a.dtype)
        if a.nbytes:
            _lib.call("nqk_memcpy_h2d", d.vp, ctypes.c_void_p(a.ctypes.data), a.nbytes)
        return d

    def to_host(self) -> np.ndarray:
        out = np.empty(self.shape, dtype=self.dtype)
        if out.nbytes:
            _lib.call("nqk_memcpy_d2h", ctypes.c_void_p(out.ctypes.data), self.vp, out.nbytes)
        return out

    def reshape(self, shape: Sequence[int]) -> "DeviceArray":
        shape = tuple(int(s) for s in shape)
        if math.prod(shape) != self.size:
            raise ValueError(f"cannot reshape array of size {self.size} into shape {shape}")
        return DeviceArray(shape, self.dtype, self.block, self.ptr)

    def offset_view(self, elem_offset: int, shape: Sequence[int]) -> "DeviceArray":
        return DeviceArray(shape, self.dtype, self.block, self.ptr + elem_offset * self.dtype.itemsize)

    def copy(self) -> "DeviceArray":
        d = DeviceArray(self.shape, self.dtype)
        _lib.call("nqk_memcpy_d2d", d.vp, self.vp, self.nbytes)
        return d

    def fill_zero(self) -> "DeviceArray":
        _lib.call("nqk_memset", self.vp, 0, self.nbytes)
        return self

    def __repr__(self):
        return f"DeviceArray(shape={self.shape}, dtype={self.dtype})"


def empty(shape, dtype) -> DeviceArray:
    return DeviceArray(shape, dtype)


def zeros(shape, dtype) -> DeviceArray:
    return DeviceArray(shape, dtype).fill_zero()


def contiguous_strides(shape: Sequence[int]) -> tuple[int, ...]:
    st = []
    acc = 1
    for s in reversed(shape):
        st.append(acc)
        acc *= int(s)
    return tuple(reversed(st))


def collapse(shape, *stride_sets):
    """Drop size-1 dims and merge adjacent dims that are contiguous in every
    stride set (keeps the kernels' index arithmetic short)."""
    dims = [(int(s), [int(st[k]) for st in stride_sets]) for k, s in enumerate(shape) if int(s) != 1]
    if not dims:
        return [1], [[0] for _ in stride_sets]
    out = [dims[0]]
    for s, sts in dims[1:]:
        ps, psts = out[-1]
        if all(psts[j] == sts[j] * s for j in range(len(stride_sets))):
            out[-1] = (ps * s, sts)
        else:
            out.append((s, sts))
    shp = [d[0] for d in out]
    strides = [[d[1][j] for d in out] for j in range(len(stride_sets))]
    return shp, strides


def _check_range(arr: DeviceArray, elem_offset: int, shape, strides, what: str) -> None:
    """Host-side bounds check of a strided access against the array's block: a bad
    view must raise here, never reach the GPU as an out-of-bounds access."""
    if any(int(s) == 0 for s in shape):
        return
    lo = elem_offset + sum((int(n) - 1) * int(st) for n, st in zip(shape, strides) if int(st) < 0)
    hi = elem_offset + sum((int(n) - 1) * int(st) for n, st in zip(shape, strides) if int(st) > 0)
    if lo < 0 or hi + 1 > arr.size:
        raise ValueError(f"{what}: strided access [{lo}, {hi}] outside the buffer of {arr.shape} {arr.dtype}")


def copy_strided(src: DeviceArray, dst: DeviceArray, shape, src_strides, dst_strides,
                 src_offset: int = 0, dst_offset: int = 0) -> None:
    _check_range(src, src_offset, shape, src_strides, "copy source")
    _check_range(dst, dst_offset, shape, dst_strides, "copy destination")
    shp, (ss, ds) = collapse(shape, src_strides, dst_strides)
    if len(shp) > 6:
        raise ValueError("copy of more than 6 non-mergeable dimensions")
    isz = src.dtype.itemsize
    _lib.call("nqk_copy_strided", ctypes.c_void_p(src.ptr + src_offset * isz),
              ctypes.c_void_p(dst.ptr + dst_offset * isz), isz, len(shp),
              _lib.i64arr(shp), _lib.i64arr(ss), _lib.i64arr(ds))


def permute(src: DeviceArray, perm: Sequence[int]) -> DeviceArray:
    perm = [p % src.ndim for p in perm] if src.ndim else []
    out_shape = [src.shape[p] for p in perm]
    sst = src.strides()
    out = DeviceArray(out_shape, src.dtype)
    copy_strided(src, out, out_shape, [sst[p] for p in perm], contiguous_strides(out_shape))
    return out


def broadcast_strides(shape, out_shape) -> list[int]:
    """Strides of a contiguous array of `shape` broadcast to `out_shape`."""
    st = contiguous_strides(shape)
    nd = len(out_shape)
    pad = nd - len(shape)
    res = []
    for k in range(nd):
        if k < pad:
            res.append(0)
        else:
            s = shape[k - pad]
            if s == out_shape[k]:
                res.append(st[k - pad])
            elif s == 1:
                res.append(0)
            else:
                raise ValueError(f"operands could not be broadcast together with shapes {tuple(shape)} {tuple(out_shape)}")
    return res


def materialize_broadcast(src: DeviceArray, out_shape) -> DeviceArray:
    out = DeviceArray(out_shape, src.dtype)
    copy_strided(src, out, out_shape, broadcast_strides(src.shape, out_shape), contiguous_strides(out_shape))
    return out


def sync() -> None:
    _lib.call("nqk_sync")
