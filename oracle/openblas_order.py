"""ORACLE — test infrastructure only, never part of the product path.

Summation order of OpenBLAS 0.3.29's single-precision GEMV-T, the routine NumPy's
`matmul` calls for a one-row product `x[1, K] @ B[K, N]` whose B has unit stride along
K (numpy/_core/src/umath/matmul.cpp, vector_matrix -> cblas_sgemv(ColMajor, Trans)):
the reference's classifier Gemm on the CLS token at batch 1 (numpy_quant/model.py:75-92
Gemm, tensor.py:100-101 FTensor.matmul -> np.matmul).

Restated from OpenBLAS's published sources (kernel/x86_64/sgemv_t_4.c with the Haswell
micro-kernel used by the Haswell / Zen / SkylakeX targets; driver/level2/gemv_thread.c;
interface/gemv.c) and PINNED against np.matmul in this container
(tests/test_host.py::test_sgemv_order_matches_numpy_matmul, shapes and thread counts
swept): OpenBLAS is a third-party dependency of the reference's NumPy (scipy-openblas
0.3.29), not part of /root/reference.

The order:
  * threads: when K * N >= 460800 the N columns are split over T threads (T =
    OpenBLAS's thread count) in chunks of ceil(remaining / threads left), at least 4;
  * K is cut into blocks of 4096 rows (the last K & 4095, less K % 4); each block's
    dot products are added to y in block order (y starts at +0);
  * per chunk, columns in groups of 4 go to the AVX2 4x4 kernel: 8 lanes, lane l takes
    rows l, l+8, ... of the block as a k-ordered fma chain (a block whose length is
    4 mod 8 starts with 4 rows in lanes 0-3), then lanes (l + l+4), then ((0+1) + (2+3));
  * 2 leftover columns: SSE kernel, 4 lanes (row r -> lane r % 4), separate multiply and
    add, then ((0+1) + (2+3));
  * 1 leftover column: SSE kernel, two 4-lane accumulators (rows 8i..8i+3 and
    8i+4..8i+7; a leading 4-row piece goes to the first), summed lane-wise, then
    ((0+1) + (2+3));
  * K % 4 trailing rows in scalar C (GCC fma contraction): one row y = fma(a0, x0, y);
    two or three y + fma(a0, x0, RN(a1 x1)) [then fma(a2, x2, .)].
"""
from __future__ import annotations

import os

import numpy as np

LD = np.longdouble
NBMAX = 4096


def openblas_threads() -> int:
    """OpenBLAS's default thread count: OPENBLAS_NUM_THREADS, GOTO_NUM_THREADS,
    OMP_NUM_THREADS, else the CPUs this process may run on; at most 64 (MAX_THREADS of
    scipy-openblas)."""
    for v in ("OPENBLAS_NUM_THREADS", "GOTO_NUM_THREADS", "OMP_NUM_THREADS"):
        s = os.environ.get(v)
        if s and s.strip().isdigit() and int(s) > 0:
            return min(int(s), 64)
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 64))


def _f(v):
    return np.asarray(v, dtype=np.float32)


def _fma(a, b, c):
    # a * b is exact in 80-bit long double (48-bit product); the sum rounds once to 64
    # bits and then to f32 (a double rounding only on an exact f32 midpoint: never seen
    # in the sweeps)
    return _f(a.astype(LD) * b.astype(LD) + c.astype(LD))


def _mul(a, b):
    return _f(a.astype(LD) * b.astype(LD))


def _k4x4(a, x):
    """a [nb, c] rows of the block, x [nb]: AVX2 kernel, 8 lanes."""
    nb = a.shape[0]
    acc = np.zeros((8,) + a.shape[1:], np.float32)
    i = 0
    if nb & 4:
        for r in range(4):
            acc[r] = _fma(np.broadcast_to(x[r], a.shape[1:]), a[r], acc[r])
        i = 4
    while i < nb:
        for r in range(8):
            acc[r] = _fma(np.broadcast_to(x[i + r], a.shape[1:]), a[i + r], acc[r])
        i += 8
    h = _f(acc[0:4] + acc[4:8])
    return _f(_f(h[0] + h[1]) + _f(h[2] + h[3]))


def _k4x2(a, x):
    nb = a.shape[0]
    acc = np.zeros((4,) + a.shape[1:], np.float32)
    for i in range(0, nb, 4):
        for r in range(4):
            acc[r] = _f(acc[r] + _mul(np.broadcast_to(x[i + r], a.shape[1:]), a[i + r]))
    return _f(_f(acc[0] + acc[1]) + _f(acc[2] + acc[3]))


def _k4x1(a, x):
    nb = a.shape[0]
    acc = np.zeros((2, 4) + a.shape[1:], np.float32)
    i = 0
    if nb & 4:
        for r in range(4):
            acc[0, r] = _f(acc[0, r] + _mul(np.broadcast_to(x[r], a.shape[1:]), a[r]))
        i = 4
    while i < nb:
        for s in range(2):
            for r in range(4):
                k = i + 4 * s + r
                acc[s, r] = _f(acc[s, r] + _mul(np.broadcast_to(x[k], a.shape[1:]), a[k]))
        i += 8
    c = _f(acc[0] + acc[1])
    return _f(_f(c[0] + c[1]) + _f(c[2] + c[3]))


def _chunk(a, x, y):
    """Columns a[:, j0:j1] of one thread (a: [K, n] with the K rows of each column)."""
    m, n = a.shape
    m3 = m & 3
    m1 = m & -4
    m2 = (m & (NBMAX - 1)) - m3
    n4 = n & -4
    k0 = 0
    nb = NBMAX
    while nb == NBMAX:
        m1 -= nb
        if m1 < 0:
            if m2 == 0:
                break
            nb = m2
        blk = a[k0:k0 + nb]
        xb = x[k0:k0 + nb]
        if n4:
            y[:n4] = _f(y[:n4] + _k4x4(blk[:, :n4], xb))
        if (n - n4) & 2:
            y[n4:n4 + 2] = _f(y[n4:n4 + 2] + _k4x2(blk[:, n4:n4 + 2], xb))
        if (n - n4) & 1:
            if m == 4:  # K = 4: the single leftover column is one multiply-add chain
                y[n - 1:n] = _f(y[n - 1:n] + _chain(xb, blk[:, n - 1:n].T, False))
            else:
                y[n - 1:n] = _f(y[n - 1:n] + _k4x1(blk[:, n - 1:n], xb))
        k0 += nb
    if m3:
        # K % 4 trailing rows in C with GCC's fma contraction: one row is
        # y = fma(a0, x0, y); two or three are y + fma(a0, x0, RN(a1 x1)) [fma(a2, x2, .)]
        xb = lambda r: np.broadcast_to(x[k0 + r], (n,))
        if m3 == 1:
            y[:] = _fma(xb(0), a[k0], y)
        else:
            t = _fma(xb(0), a[k0], _mul(xb(1), a[k0 + 1]))
            if m3 == 3:
                t = _fma(xb(2), a[k0 + 2], t)
            y[:] = _f(y + t)


def thread_ranges(n: int, m: int, threads: int) -> list[tuple[int, int]]:
    """Column chunks of gemv_thread.c (one chunk when m * n < 115200 * 4)."""
    if m * n < 115200 * 4 or threads <= 1:
        return [(0, n)]
    out, j, t = [], 0, 0
    rem = n
    while rem > 0:
        w = (rem + threads - t - 1) // (threads - t) if threads - t > 0 else rem
        w = max(w, 4)
        w = min(w, rem)
        out.append((j, j + w))
        j += w
        rem -= w
        t += 1
    return out


def sgemv_t(b_t: np.ndarray, x: np.ndarray, threads: int | None = None) -> np.ndarray:
    """y[j] = sum_k b_t[j, k] * x[k] in OpenBLAS's order (b_t: [N, K] float32, the
    columns of B stored contiguously; x: [K])."""
    b_t = np.asarray(b_t, np.float32)
    x = np.asarray(x, np.float32)
    n, m = b_t.shape
    threads = openblas_threads() if threads is None else threads
    y = np.zeros(n, np.float32)
    a = np.ascontiguousarray(b_t.T)  # [K, N]
    for j0, j1 in thread_ranges(n, m, threads):
        yc = y[j0:j1].copy()
        _chunk(a[:, j0:j1], x, yc)
        y[j0:j1] = yc
    return y


# --------------------------------------------------------------------------------------
# The one-row products outside the GEMV-T kernels above, identified against np.matmul in
# this container (tests/test_host.py::test_small_one_row_orders_match_numpy_matmul):
#  * a 1 x 1 result goes to cblas_sdot: below 32 rows the f32 products are summed in double
#    in order and the sum rounded once (sdot's scalar tail; from 32 rows a vector kernel
#    whose order is not restated);
#  * K in 2..8 except 4 goes to OpenBLAS's small-m GEMV-T kernels: columns in blocks of 16
#    (K = 2), 4 (K = 5) or 8 (K = 3, 6, 7) are k-ordered fma chains, leftover columns
#    multiply-add chains, except a leftover 4-column block (K = 3, 6, 7) and a last odd
#    column (K = 3), and K = 8 altogether, whose orders are not restated;
#  * K = 4: the GEMV-T kernels above, except a single leftover column (N odd), which is a
#    multiply-add chain.


def sdot(x: np.ndarray, w: np.ndarray) -> np.float32:
    """x . w for a 1 x 1 matmul result (len < 32)."""
    p = (np.asarray(x, np.float32) * np.asarray(w, np.float32)).astype(np.float32)
    d = 0.0
    for v in p:
        d += float(v)
    return np.float32(d)


def _chain(x, w, fma: bool):
    acc = np.zeros(w.shape[0], np.float32)
    for k in range(w.shape[1]):
        xk = np.broadcast_to(np.float32(x[k]), acc.shape)
        acc = _fma(xk, w[:, k], acc) if fma else _f(acc + _mul(xk, w[:, k]))
    return acc


def small_modes(N: int, K: int) -> str:
    """Per column: 'F' fma chain, 'M' multiply-add chain, '?' not restated (K in 2..8, not 4)."""
    blk = 16 if K == 2 else (4 if K == 5 else 8)
    f_end = N // blk * blk
    if K == 8:
        return "?" * N
    tail = ""
    r = N - f_end
    if K in (3, 6, 7) and r >= 4:
        tail, r = "????", r - 4
    if K == 3:
        tail += ("MM" if r & 2 else "") + ("?" if r & 1 else "")
    else:
        tail += "M" * r
    return "F" * f_end + tail


def sgemv_small(b_t: np.ndarray, x: np.ndarray) -> np.ndarray:
    """y = b_t . x for K in 2..8 except 4 ('?' columns computed as fma chains)."""
    b_t = np.asarray(b_t, np.float32)
    x = np.asarray(x, np.float32)
    modes = small_modes(*b_t.shape)
    fm = np.array([m != "M" for m in modes])
    return np.where(fm, _chain(x, b_t, True), _chain(x, b_t, False)).astype(np.float32)
