"""Typed wrappers around the libnqk.so entry points, on DeviceArrays.

One function per kernel family; argument checking (shapes the kernels and their
grids assume) happens here, on the host, before anything is launched.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

from . import _lib
from .device import (DeviceArray, broadcast_strides, collapse, contiguous_strides, copy_strided,
                     materialize_broadcast)

VP = ctypes.c_void_p


def storage_dtype(bit_width: int) -> np.dtype:
    """Narrowest integer storage for values in [-2^(bw-1), 2^(bw-1)-1]."""
    if bit_width <= 8:
        return np.dtype(np.int8)
    if bit_width <= 16:
        return np.dtype(np.int16)
    if bit_width <= 32:
        return np.dtype(np.int32)
    return np.dtype(np.int64)


# ----------------------------------------------------------------------------- quantization
def quantize(x: DeviceArray, bit_width: int, scale: float, zp: int | None, out_dtype=None,
             rowsum: bool = False):
    """numpy_quantization.py:24-34 on device.  Returns (q, rowsum | None)."""
    if x.dtype != np.float32:
        raise ValueError("quantize expects float32 input")
    dt = np.dtype(out_dtype) if out_dtype is not None else storage_dtype(bit_width)
    q = DeviceArray(x.shape, dt)
    rs = None
    row_len = x.shape[-1] if x.ndim else 1
    if rowsum:
        rs = DeviceArray(x.shape[:-1] if x.ndim else (), np.int64)
    _lib.call("nqk_quantize", x.vp, q.vp, q.code, x.size, float(np.float32(scale)),
              0 if zp is None else int(zp), 0 if zp is None else 1, int(bit_width),
              rs.vp if rs is not None else None, row_len)
    return q, rs


class ZpTerm:
    """Zero-point term of a q_matmul output (numpy_quantization.py:49-61), kept as
    row sums of A and column sums of B instead of an int64 (..., M, N) array."""

    __slots__ = ("flags", "zpa", "zpb", "K", "row", "col", "bmap", "a_batch", "b_batch", "M", "N")

    def __init__(self, flags, zpa, zpb, K, row, col, bmap, a_batch, b_batch, M, N):
        self.flags, self.zpa, self.zpb, self.K = flags, zpa, zpb, K
        self.row, self.col, self.bmap = row, col, bmap
        self.a_batch, self.b_batch, self.M, self.N = tuple(a_batch), tuple(b_batch), M, N

    def to_host(self) -> np.ndarray:
        """The reference's int64 zero_point array (same shape and values)."""
        term = None
        if self.flags & _lib.ZP_ROW:
            term = self.row.to_host().reshape(self.a_batch + (self.M, 1)) * np.int64(self.zpb)
        if self.flags & _lib.ZP_COL:
            c = self.col.to_host().reshape(self.b_batch + (1, self.N)) * np.int64(self.zpa)
            term = c if term is None else term + c
        if self.flags & _lib.ZP_KCONST:
            term = term - np.int64(self.zpa) * np.int64(self.zpb) * np.int64(self.K)
        return term


def _zp_args(zp):
    """(flags, zp, zpa, zpb, K, row, col, bmap) for dequantize / requantize."""
    if zp is None:
        return _lib.ZP_NONE, 0, 0, 0, 0, None, None, None
    if isinstance(zp, ZpTerm):
        return (zp.flags, 0, zp.zpa, zp.zpb, zp.K, zp.row.vp if zp.row is not None else None,
                zp.col.vp if zp.col is not None else None, _lib.i64arr(zp.bmap))
    return _lib.ZP_SCALAR, int(zp), 0, 0, 0, None, None, None


def _bmn(shape):
    if isinstance(shape, tuple) and len(shape) >= 2:
        return int(math.prod(shape[:-2])), int(shape[-2]), int(shape[-1])
    return 1, 1, int(math.prod(shape))


def dequantize(q: DeviceArray, scale, zp) -> DeviceArray:
    """f32( f64(q - zp) * f64(s) )  (numpy_quantization.py:37-41, tensor.py:261-265)."""
    out = DeviceArray(q.shape, np.float32)
    flags, z, zpa, zpb, K, row, col, bmap = _zp_args(zp)
    if isinstance(zp, ZpTerm):
        b, m, n = _bmn(q.shape)
    else:
        b, m, n = 1, 1, q.size
    _lib.call("nqk_dequantize", q.vp, q.code, out.vp, b, m, n, float(np.float32(scale)), flags, z, zpa, zpb,
              K, row, col, bmap)
    return out


def requantize(acc: DeviceArray, scale, zp, bias: DeviceArray | None, res_scale, res_zp,
               bit_width: int) -> DeviceArray:
    """numpy_quantization.py:64-72 with the Gemm bias add (tensor.py:255-259) fused."""
    out = DeviceArray(acc.shape, storage_dtype(bit_width))
    flags, z, zpa, zpb, K, row, col, bmap = _zp_args(zp)
    b, m, n = _bmn(acc.shape) if acc.ndim >= 2 else (1, 1, acc.size)
    if bias is not None and bias.size != n:
        raise ValueError(f"bias of {bias.size} elements cannot broadcast over rows of {n}")
    _lib.call("nqk_requantize", acc.vp, acc.code, bias.vp if bias is not None else None,
              bias.code if bias is not None else _lib.NQK_I64, out.vp, out.code, b, m, n,
              float(np.float32(scale)), flags, z, zpa, zpb, K, row, col, bmap,
              float(np.float32(res_scale)), 0 if res_zp is None else int(res_zp),
              0 if res_zp is None else 1, int(bit_width))
    return out


def rowsum(a: DeviceArray, batch: int, rows: int, k: int, ld: int, bstride: int) -> DeviceArray:
    out = DeviceArray((batch * rows,), np.int64)
    _lib.call("nqk_rowsum", a.vp, a.code, out.vp, batch, rows, k, ld, bstride)
    return out


# ----------------------------------------------------------------------------- batch maps
def batch_map(a_batch, b_batch):
    """Express np.matmul batch broadcasting as (out_batch, [inner, ao, ai, bo, bi])
    or None when it cannot be split into two uniform groups."""
    nd = max(len(a_batch), len(b_batch))
    a = (1,) * (nd - len(a_batch)) + tuple(a_batch)
    b = (1,) * (nd - len(b_batch)) + tuple(b_batch)
    out = []
    for x, y in zip(a, b):
        if x != y and x != 1 and y != 1:
            raise ValueError(f"matmul batch shapes {a_batch} and {b_batch} do not broadcast")
        out.append(max(x, y))
    out = tuple(out)

    def group_kind(src, lo, hi):
        full = all(src[k] == out[k] for k in range(lo, hi))
        one = all(src[k] == 1 for k in range(lo, hi))
        return "full" if full else ("one" if one else None)

    for p in range(nd + 1):
        ka_o, ka_i = group_kind(a, 0, p), group_kind(a, p, nd)
        kb_o, kb_i = group_kind(b, 0, p), group_kind(b, p, nd)
        if None in (ka_o, ka_i, kb_o, kb_i):
            continue
        inner = int(math.prod(out[p:]))
        a_inner = int(math.prod(a[p:]))
        b_inner = int(math.prod(b[p:]))
        ao = a_inner if ka_o == "full" else 0
        ai = 1 if ka_i == "full" and a_inner > 1 else 0
        bo = b_inner if kb_o == "full" else 0
        bi = 1 if kb_i == "full" and b_inner > 1 else 0
        return out, [max(inner, 1), ao, ai, bo, bi]
    return out, None


# ----------------------------------------------------------------------------- integer GEMM
MFMA_MIN_WORK = 1 << 15


class KernelTimer:
    """Brackets selected kernel launches with stream events (bench.py roofline):
    `records` collects (tag, start_event, stop_event, work) tuples."""

    def __init__(self):
        self.records = []
        self._free = []

    def _event(self):
        if self._free:
            return self._free.pop()
        e = ctypes.c_void_p()
        _lib.call("nqk_event_create", ctypes.byref(e))
        return e

    def begin(self):
        e = self._event()
        _lib.call("nqk_event_record", e)
        return e

    def end(self, tag, start, work, unit="int8"):
        """work = (ops, algorithmic bytes); unit: what the ops count ("int8" MFMA ops,
        "flop32" f32 MFMA flops)."""
        e = self._event()
        _lib.call("nqk_event_record", e)
        self.records.append((tag, start, e, work, unit))

    def collect(self):
        """[(tag, ms, work, unit)] and recycle the events."""
        out = []
        for tag, a, b, w, unit in self.records:
            ms = ctypes.c_float()
            _lib.call("nqk_event_elapsed", a, b, ctypes.byref(ms))
            out.append((tag, ms.value, w, unit))
            self._free += [a, b]
        self.records = []
        return out


TIMER: KernelTimer | None = None


def _pad_k(x: DeviceArray, rows_shape, k: int, kp: int) -> DeviceArray:
    """Copy [..., rows, k] into a zero-filled [..., rows, kp] (kp % 16 == 0)."""
    out = DeviceArray(tuple(rows_shape) + (kp,), x.dtype).fill_zero()
    shape = tuple(rows_shape) + (k,)
    copy_strided(x, out, shape, contiguous_strides(shape), contiguous_strides(tuple(rows_shape) + (kp,)))
    return out


def qmatmul(a: DeviceArray, b: DeviceArray, zpa, zpb, b_transposed: DeviceArray | None = None,
            b_colsum: DeviceArray | None = None):
    """q_matmul (numpy_quantization.py:44-61): returns (acc, ZpTerm | None).

    a: [..., M, K] and b: [..., K, N] integer DeviceArrays (contiguous).  The int8
    path needs Bt[..., N, Kp]; `b_transposed` (and its column sums) may be passed in
    pre-computed for constant weights.
    """
    if a.ndim < 2 or b.ndim < 2:
        raise ValueError("q_matmul operands must have at least 2 dimensions")
    M, K = a.shape[-2:]
    K2, N = b.shape[-2:]
    if K != K2:
        raise ValueError(f"matmul: mismatch in core dimension ({K} vs {K2})")
    a_batch, b_batch = a.shape[:-2], b.shape[:-2]
    out_batch, bmap = batch_map(a_batch, b_batch)
    if bmap is None:  # exotic broadcast: materialise both operands
        a = materialize_broadcast(a, out_batch + (M, K))
        b = materialize_broadcast(b, out_batch + (K, N))
        a_batch = b_batch = out_batch
        b_transposed = b_colsum = None
        _, bmap = batch_map(a_batch, b_batch)
    nb = int(math.prod(out_batch))
    na, nbb = int(math.prod(a_batch)), int(math.prod(b_batch))
    use_mfma = (a.dtype == np.int8 and b.dtype == np.int8 and M * N * K >= MFMA_MIN_WORK and nb <= 65535)
    if use_mfma:
        kp = (K + 15) // 16 * 16
        ap = a if K == kp else _pad_k(a, a.shape[:-1], K, kp)
        if b_transposed is None:
            bt = DeviceArray(b_batch + (N, kp), np.int8)
            if K != kp:
                bt.fill_zero()
            shape = b_batch + (N, K)
            bst = contiguous_strides(b.shape)
            src_st = list(bst[:-2]) + [bst[-1], bst[-2]]
            copy_strided(b, bt, shape, src_st, contiguous_strides(b_batch + (N, kp)))
        else:
            bt = b_transposed
        acc = DeviceArray(out_batch + (M, N), np.int32)
        t0 = TIMER.begin() if TIMER is not None else None
        _lib.call("nqk_qgemm_i8", ap.vp, bt.vp, acc.vp, nb, M, N, kp, kp, kp, N, _lib.i64arr(bmap),
                  M * kp, N * kp, M * N)
        if t0 is not None:
            TIMER.end("qgemm_i8", t0, (2 * nb * M * N * K, nb * (M * K + N * K + 4 * M * N)))
    else:
        acc = DeviceArray(out_batch + (M, N), np.int64)
        _lib.call("nqk_qgemm_generic", a.vp, a.code, b.vp, b.code, acc.vp, nb, M, N, K, K, 1, N, 1, N,
                  _lib.i64arr(bmap), M * K, K * N, M * N)
        bt = None
    if zpa is None and zpb is None:
        return acc, None
    row = col = None
    flags = 0
    if zpb is not None:
        row = rowsum(a, na, M, K, K, M * K)
        flags |= _lib.ZP_ROW
    if zpa is not None:
        if b_colsum is not None:
            col = b_colsum
        elif bt is not None and use_mfma:
            kp = bt.shape[-1]
            col = rowsum(bt, nbb, N, kp, kp, N * kp)
        else:
            btt = DeviceArray(b_batch + (N, K), b.dtype)
            bst = contiguous_strides(b.shape)
            copy_strided(b, btt, b_batch + (N, K), list(bst[:-2]) + [bst[-1], bst[-2]],
                         contiguous_strides(b_batch + (N, K)))
            col = rowsum(btt, nbb, N, K, K, N * K)
        flags |= _lib.ZP_COL
    if zpa is not None and zpb is not None:
        flags |= _lib.ZP_KCONST
    zt = ZpTerm(flags, 0 if zpa is None else int(zpa), 0 if zpb is None else int(zpb), K, row, col, bmap,
                a_batch, b_batch, M, N)
    return acc, zt


def weight_bt(b: DeviceArray):
    """Pre-transposed, K-padded int8 copy of a constant [K, N] weight and its
    column sums (used for every call instead of per-call transposes)."""
    K, N = b.shape[-2:]
    kp = (K + 15) // 16 * 16
    bt = DeviceArray(b.shape[:-2] + (N, kp), b.dtype)
    if kp != K:
        bt.fill_zero()
    bst = contiguous_strides(b.shape)
    copy_strided(b, bt, b.shape[:-2] + (N, K), list(bst[:-2]) + [bst[-1], bst[-2]],
                 contiguous_strides(b.shape[:-2] + (N, kp)))
    nb = int(math.prod(b.shape[:-2]))
    col = rowsum(bt, nb, N, kp, kp, N * kp)
    return bt, col


# ----------------------------------------------------------------------------- float GEMM
def sgemm(a: DeviceArray, a_sm, a_sk, b: DeviceArray, b_sk, b_sn, M, N, K, batch=1, bmap=None,
          a_ms=0, b_ms=0) -> DeviceArray:
    c = DeviceArray((batch, M, N) if batch > 1 else (M, N), np.float32)
    _lib.call("nqk_sgemm", a.vp, b.vp, c.vp, batch, M, N, K, a_sm, a_sk, b_sk, b_sn, N,
              _lib.i64arr(bmap) if bmap is not None else None, a_ms, b_ms, M * N)
    return c


# OpenBLAS thread count of the NumPy whose GEMV order is reproduced (its column split
# depends on it, oracle/openblas_order.py): NQK_BLAS_THREADS, else what OpenBLAS itself
# reads (OPENBLAS_NUM_THREADS, GOTO_NUM_THREADS, OMP_NUM_THREADS, else the CPUs this
# process may run on), at most 64 (scipy-openblas MAX_THREADS)
BLAS_THREADS = None


def openblas_threads() -> int:
    if BLAS_THREADS is not None:
        return int(BLAS_THREADS)
    for v in ("NQK_BLAS_THREADS", "OPENBLAS_NUM_THREADS", "GOTO_NUM_THREADS", "OMP_NUM_THREADS"):
        s = os.environ.get(v, "").strip()
        if s.isdigit() and int(s) > 0:
            return min(int(s), 64)
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 64))


def gemv_t_applies(M: int, N: int, K: int) -> bool:
    """NumPy sends a one-row product x[1, K] @ B[K, N] (N > 1) whose B has unit stride
    along K to OpenBLAS GEMV-T; nqk_sgemv_t reproduces its order for every K (the regular
    kernels, and for K <= 8 the small-m kernels of each thread chunk of at most 16 384
    columns: oracle/openblas_order.py, pinned against np.matmul)."""
    return M == 1 and N > 1


def small_one_row(N: int, K: int) -> bool:
    """A one-row product with a 1 x 1 result: NumPy calls cblas_sdot (nqk_sgemv_small)."""
    return N == 1


def one_row_restated(N: int, K: int) -> bool:
    """Whether x[1, K] @ B[K, N] with B's columns contiguous (a Gemm's w.T) is computed in
    NumPy's exact order (pinned against np.matmul, tests/test_host.py): since round 6 every
    such product is — sdot at every length, GEMV-T's regular and small-m kernels at every K.
    (A one-row product against a row-major B — a MatMul's weight — is GEMV-N: nqk_sgemv_n.)"""
    return N >= 1 and K >= 1


def sgemv_small(x: DeviceArray, bt: DeviceArray) -> DeviceArray:
    """y[1, 1] = x[1, K] . bt[1, K]^T in cblas_sdot's order (nqk_sgemv_small)."""
    N, Kb = bt.shape
    K = x.shape[-1]
    if Kb != K or x.size != K:
        raise ValueError(f"matmul: mismatch in core dimension ({K} vs {Kb})")
    y = DeviceArray((1, N), np.float32)
    _lib.call("nqk_sgemv_small", x.vp, bt.vp, y.vp, N, K, K)
    return y


def sgemv_t(x: DeviceArray, bt: DeviceArray) -> DeviceArray:
    """y[1, N] = x[1, K] . bt[N, K]^T in OpenBLAS GEMV-T order (nqk_sgemv_t)."""
    N, Kb = bt.shape
    K = x.shape[-1]
    if Kb != K or x.size != K:
        raise ValueError(f"matmul: mismatch in core dimension ({K} vs {Kb})")
    y = DeviceArray((1, N), np.float32)
    _lib.call("nqk_sgemv_t", x.vp, bt.vp, y.vp, N, K, K, openblas_threads())
    return y


def matmul_f32(a: DeviceArray, b: DeviceArray) -> DeviceArray:
    """np.matmul for float32 (batched, broadcast), BLAS summation order."""
    M, K = a.shape[-2:]
    K2, N = b.shape[-2:]
    if K != K2:
        raise ValueError(f"matmul: mismatch in core dimension ({K} vs {K2})")
    if (M == 1 or N == 1) and K > 1:
        return _matmul_level2(a, b, M, N, K)
    out_batch, bmap = batch_map(a.shape[:-2], b.shape[:-2])
    if bmap is None:
        a = materialize_broadcast(a, out_batch + (M, K))
        b = materialize_broadcast(b, out_batch + (K, N))
        _, bmap = batch_map(out_batch, out_batch)
    nb = int(math.prod(out_batch))
    c = sgemm(a, K, 1, b, N, 1, M, N, K, batch=nb, bmap=bmap, a_ms=M * K, b_ms=K * N)
    return c.reshape(out_batch + (M, N))


def _matmul_level2(a: DeviceArray, b: DeviceArray, M: int, N: int, K: int) -> DeviceArray:
    """np.matmul where one side of each product is a vector: NumPy's matmul (matmul.cpp special
    cases, per matrix of a stack) calls cblas_sdot for a 1 x 1 result, and cblas_sgemv for
    vector @ matrix — OpenBLAS GEMV-N on a row-major matrix (nqk_sgemv_n) — and for matrix @
    vector — GEMV-T over the matrix's rows (nqk_sgemv_t); each restated bit for bit
    (oracle/openblas_order.py, round 6).  (K = 1 stays on the GEMM path: NumPy's own loop, one
    product per output.)"""
    out_batch = tuple(np.broadcast_shapes(a.shape[:-2], b.shape[:-2]))
    if a.shape[:-2] != out_batch:
        a = materialize_broadcast(a, out_batch + (M, K))
    if b.shape[:-2] != out_batch:
        b = materialize_broadcast(b, out_batch + (K, N))
    c = DeviceArray(out_batch + (M, N), np.float32)
    t = openblas_threads()
    for i in range(int(math.prod(out_batch))):
        ai, bi, ci = a.offset_view(i * M * K, (M, K)), b.offset_view(i * K * N, (K, N)), c.offset_view(i * M * N, (M, N))
        if M == 1 and N == 1:
            _lib.call("nqk_sgemv_small", ai.vp, bi.vp, ci.vp, 1, K, K)
        elif M == 1:
            _lib.call("nqk_sgemv_n", ai.vp, bi.vp, ci.vp, N, K, N, t)
        else:
            _lib.call("nqk_sgemv_t", bi.vp, ai.vp, ci.vp, M, K, K, t)
    return c


def sgemv_n(x: DeviceArray, b: DeviceArray) -> DeviceArray:
    """y[1, N] = x[1, K] . b[K, N] (b row-major) in OpenBLAS GEMV-N order (nqk_sgemv_n)."""
    K, N = b.shape
    if x.size != K:
        raise ValueError(f"matmul: mismatch in core dimension ({x.size} vs {K})")
    y = DeviceArray((1, N), np.float32)
    _lib.call("nqk_sgemv_n", x.vp, b.vp, y.vp, N, K, N, openblas_threads())
    return y


# ----------------------------------------------------------------------------- float ops
def binary(op: int, a: DeviceArray, b: DeviceArray) -> DeviceArray:
    out_shape = tuple(np.broadcast_shapes(a.shape, b.shape))
    out = DeviceArray(out_shape, np.float32)
    sa = broadcast_strides(a.shape, out_shape)
    sb = broadcast_strides(b.shape, out_shape)
    shp, (sa, sb) = collapse(out_shape, sa, sb)
    if len(shp) > 6:
        raise ValueError("elementwise op over more than 6 non-mergeable dimensions")
    _lib.call("nqk_binary_f32", op, a.vp, b.vp, out.vp, len(shp), _lib.i64arr(shp), _lib.i64arr(sa),
              _lib.i64arr(sb))
    return out


def unary(op: int, x: DeviceArray) -> DeviceArray:
    out = DeviceArray(x.shape, np.float32)
    _lib.call("nqk_unary_f32", op, x.vp, out.vp, x.size)
    return out


def add_scalar(x: DeviceArray, s: float) -> DeviceArray:
    out = DeviceArray(x.shape, np.float32)
    _lib.call("nqk_add_scalar_f32", x.vp, float(np.float32(s)), out.vp, x.size)
    return out


def _move_last(x: DeviceArray, axis: int):
    axis %= x.ndim
    if axis == x.ndim - 1:
        return x, None
    perm = [k for k in range(x.ndim) if k != axis] + [axis]
    from .device import permute
    return permute(x, perm), perm


def _move_back(y: DeviceArray, perm):
    if perm is None:
        return y
    inv = [0] * len(perm)
    for i, p in enumerate(perm):
        inv[p] = i
    from .device import permute
    return permute(y, inv)


def softmax(x: DeviceArray, axis: int) -> DeviceArray:
    xt, perm = _move_last(x, axis)
    cols = xt.shape[-1]
    out = DeviceArray(xt.shape, np.float32)
    _lib.call("nqk_softmax_lastdim", xt.vp, out.vp, xt.size // max(cols, 1), cols)
    return _move_back(out, perm)


def layernorm(x: DeviceArray, g: DeviceArray, b: DeviceArray, axis: int, eps: float) -> DeviceArray:
    xt, perm = _move_last(x, axis)
    cols = xt.shape[-1]
    if g.size != cols or b.size != cols:
        g = materialize_broadcast(g, (cols,)) if g.size == 1 else g
        b = materialize_broadcast(b, (cols,)) if b.size == 1 else b
    if g.size != cols or b.size != cols:
        raise ValueError("LayerNormalization scale/bias must cover the normalised axis")
    out = DeviceArray(xt.shape, np.float32)
    _lib.call("nqk_layernorm_lastdim", xt.vp, g.vp, b.vp, out.vp, xt.size // cols, cols, float(np.float32(eps)))
    return _move_back(out, perm)


def mean_lastdim(x: DeviceArray) -> DeviceArray:
    cols = x.shape[-1]
    out = DeviceArray(x.shape[:-1] + (1,), np.float32)
    _lib.call("nqk_mean_lastdim", x.vp, out.vp, x.size // cols, cols)
    return out


def minmax(x: DeviceArray) -> tuple[np.float32, np.float32]:
    scratch = DeviceArray((4096,), np.float32)
    res = DeviceArray((2,), np.float32)
    _lib.call("nqk_minmax_f32", x.vp, x.size, res.vp, scratch.vp, 4096)
    h = res.to_host()
    return h[0], h[1]


def where(cond: np.ndarray, a: DeviceArray, b: DeviceArray) -> DeviceArray:
    c = DeviceArray.from_host(np.asarray(cond).astype(np.int64))
    out_shape = tuple(np.broadcast_shapes(c.shape, a.shape, b.shape))
    out = DeviceArray(out_shape, np.float32)
    sc, sa, sb = (broadcast_strides(t.shape, out_shape) for t in (c, a, b))
    shp, (sc, sa, sb) = collapse(out_shape, sc, sa, sb)
    _lib.call("nqk_where_f32", c.vp, a.vp, b.vp, out.vp, len(shp), _lib.i64arr(shp), _lib.i64arr(sc),
              _lib.i64arr(sa), _lib.i64arr(sb))
    return out


def im2col(x: DeviceArray, kh, kw, pads, strides):
    n, c, h, w = x.shape
    ph0, pw0, ph1, pw1 = pads
    sh, sw = strides
    ho = int(np.ceil((h - kh + ph0 + ph1 + 1) / sh))
    wo = int(np.ceil((w - kw + pw0 + pw1 + 1) / sw))
    cols = DeviceArray((n * ho * wo, kh * kw * c), np.float32)
    _lib.call("nqk_im2col", x.vp, cols.vp, n, c, h, w, kh, kw, ph0, pw0, sh, sw, ho, wo)
    return cols, ho, wo
