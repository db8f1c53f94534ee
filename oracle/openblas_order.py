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
        if 2 <= m <= SMALL_M and j1 - j0 <= SMALL_N:  # OpenBLAS's small-m kernels (below)
            y[j0:j1] = _small_chunk(b_t[j0:j1], x)
            continue
        yc = y[j0:j1].copy()
        _chunk(a[:, j0:j1], x, yc)
        y[j0:j1] = yc
    return y


# --------------------------------------------------------------------------------------
# The one-row products outside the kernels above (round 6: every class identified against
# np.matmul in this container by probing the summation tree of single outputs — which pairs of
# products meet before a third, with exactly representable inputs — and then which nodes fuse
# the product into an fma, on random inputs; pinned by tests/test_host.py
# ::test_small_one_row_orders_match_numpy_matmul and ::test_sdot_order_matches_numpy_matmul):
#  * a 1 x 1 result goes to cblas_sdot (kernel/x86_64/sdot.c + its SkylakeX micro-kernel): the
#    first n & -32 elements by the vector kernel — four 16-lane fma accumulators over 64-element
#    steps, each folded to 8 lanes (low half + high half), four 8-lane fma accumulators over the
#    remaining 32-element steps, ((a0 + a1) + a2) + a3, low + high 4 lanes, two horizontal adds
#    — then the f32 products of the tail added in double and the sum rounded once;
#  * GEMV-T with K = m <= 8 rows and contiguous columns: per thread chunk of at most 16 384
#    columns (wider chunks: the regular kernels above), OpenBLAS's small-m kernels, whose
#    column classes (by the column's place in its chunk) are, with p_k = RN(x_k w_k):
#      F  k-ordered fma chain;  M  multiply-add chain ((p0 + p1) + p2) + ...;
#      K = 2: F in blocks of 16, the rest M;   K = 5: F in blocks of 4, the rest M;
#      K = 4: (p0 + p1) + (p2 + p3), a last odd column M;
#      K = 3: F in blocks of 8; then a 4-column block and a last odd column
#             fma(x2, w2, fma(x0, w0, p1)); two leftover columns M;
#      K = 6: F in blocks of 8; a 4-column block (p0 + fma(x1, w1, p2)) + (p3 + fma(x4, w4, p5)); rest M;
#      K = 7: F in blocks of 8; a 4-column block (fma(x0, w0, p1) + fma(x4, w4, p5)) +
#             (fma(x2, w2, p3) + p6); rest M;
#      K = 8: blocks of 4 ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)); two leftover columns
#             ((p0 + p1) + (p4 + p5)) + ((p2 + p3) + (p6 + p7)); a last odd column
#             (((p0 + p4) + (p1 + p5)) + (p2 + p6)) + (p3 + p7).
SMALL_M, SMALL_N = 8, 16384


def sdot(x: np.ndarray, w: np.ndarray) -> np.float32:
    """x . w for a 1 x 1 matmul result (cblas_sdot's order, any length)."""
    x = np.asarray(x, np.float32)
    w = np.asarray(w, np.float32)
    n = x.size
    n1 = n & -32
    d = 0.0
    if n1:
        acc = np.zeros((4, 16), np.float32)
        i, n64 = 0, n & ~63
        while i < n64:
            for q in range(4):
                acc[q] = _fma(x[i + 16 * q:i + 16 * q + 16], w[i + 16 * q:i + 16 * q + 16], acc[q])
            i += 64
        a8 = _f(acc[:, :8] + acc[:, 8:])
        while i < n1:
            for q in range(4):
                a8[q] = _fma(x[i + 8 * q:i + 8 * q + 8], w[i + 8 * q:i + 8 * q + 8], a8[q])
            i += 32
        s8 = _f(_f(_f(a8[0] + a8[1]) + a8[2]) + a8[3])
        h = _f(s8[:4] + s8[4:])
        d = float(_f(_f(h[0] + h[1]) + _f(h[2] + h[3])))
    for k in range(n1, n):
        d += float(_mul(x[k:k + 1], w[k:k + 1])[0])
    return np.float32(d)


def _chain(x, w, fma: bool):
    acc = np.zeros(w.shape[0], np.float32)
    for k in range(w.shape[1]):
        xk = np.broadcast_to(np.float32(x[k]), acc.shape)
        acc = _fma(xk, w[:, k], acc) if fma else _f(acc + _mul(xk, w[:, k]))
    return acc


def small_modes(N: int, K: int) -> str:
    """Per column of a chunk of N columns, the small-m kernel's class for K in 2..8: 'F' fma
    chain, 'M' multiply-add chain, 'P' K = 4's pairs, 'b' the 4-column block of K = 3, 6, 7
    (and K = 3's last odd column), 'c' / 'a' / 'e' K = 8's 4-column blocks / two leftover
    columns / last odd column."""
    if K == 4:
        return "P" * (N & ~1) + ("M" if N & 1 else "")
    if K == 8:
        n4 = N & ~3
        return "c" * n4 + ("aa" if N & 2 else "") + ("e" if N & 1 else "")
    blk = {2: 16, 5: 4}.get(K, 8)
    f_end = N // blk * blk
    r = N - f_end
    tail = ""
    if K in (3, 6, 7) and r >= 4:
        tail, r = "bbbb", r - 4
    if K == 3:
        tail += ("MM" if r & 2 else "") + ("b" if r & 1 else "")
    else:
        tail += "M" * r
    return "F" * f_end + tail


def _small_class(c: str, x, W) -> np.ndarray:
    K = x.size
    p = [_mul(np.broadcast_to(x[k], W.shape[:1]), W[:, k]) for k in range(K)]
    F = lambda k, acc: _fma(np.broadcast_to(x[k], W.shape[:1]), W[:, k], acc)
    if c == "F":
        return _chain(x, W, True)
    if c == "M":
        return _chain(x, W, False)
    if c == "P":
        return _f(_f(p[0] + p[1]) + _f(p[2] + p[3]))
    if c == "b":
        if K == 3:
            return F(2, F(0, p[1]))
        if K == 6:
            return _f(_f(p[0] + F(1, p[2])) + _f(p[3] + F(4, p[5])))
        return _f(_f(F(0, p[1]) + F(4, p[5])) + _f(F(2, p[3]) + p[6]))
    if c == "c":
        return _f(_f(_f(p[0] + p[1]) + _f(p[2] + p[3])) + _f(_f(p[4] + p[5]) + _f(p[6] + p[7])))
    if c == "a":
        return _f(_f(_f(p[0] + p[1]) + _f(p[4] + p[5])) + _f(_f(p[2] + p[3]) + _f(p[6] + p[7])))
    return _f(_f(_f(_f(p[0] + p[4]) + _f(p[1] + p[5])) + _f(p[2] + p[6])) + _f(p[3] + p[7]))


def _small_chunk(b_t: np.ndarray, x: np.ndarray) -> np.ndarray:
    """The small-m kernel over one thread chunk b_t [n, K] (K in 2..8)."""
    modes = small_modes(*b_t.shape)
    y = np.zeros(b_t.shape[0], np.float32)
    for c in set(modes):
        sel = np.array([m == c for m in modes])
        y[sel] = _small_class(c, x, b_t[sel])
    return y


def sgemv_small(b_t: np.ndarray, x: np.ndarray, threads: int | None = None) -> np.ndarray:
    """y = b_t . x for K in 2..8 (= sgemv_t, which dispatches the small-m kernels)."""
    return sgemv_t(b_t, x, threads)


# --------------------------------------------------------------------------------------
# GEMV-N (round 6): a one-row product x[1, K] @ B[K, N] with B row-major — NumPy's matmul
# vector_matrix -> cblas_sgemv on the row-major matrix, which OpenBLAS runs as its "N" kernel
# (kernel/x86_64/sgemv_n_4.c with the SkylakeX micro-kernels, driver/level2/gemv_thread.c);
# identified against np.matmul in this container as the small-m classes above and pinned by
# tests/test_host.py::test_sgemv_n_order_matches_numpy_matmul:
#  * K <= 48: every output a k-ordered fma chain;
#  * N < 4 (the matrix is its own 1-3 trailing rows, lda == m): t = t + fma(x_k, b_k,
#    RN(x_{k+1} b_{k+1})) over k = 0, 2, ... below K & -4, then an fma chain over the rest;
#  * else: the N outputs split over the threads like GEMV-T's columns (thread_ranges); per chunk
#    of w outputs the last w & 3 are fma chains; the others go in blocks of 4096 outputs (the
#    last (w & 4095) - (w & 3)); in a block of NB the first NB % 16 outputs take the 8- / 4-row
#    kernel — per group of 8 products two fma chains (even, odd positions) added, y += a + b;
#    a leftover group of 4 the same; of 2 or 1 one chain — and the rest the 16-row kernel: per
#    group of 8, 4, 2, 1 products one fma chain, y += chain.


def _bx(x, k, n):
    return np.broadcast_to(np.float32(x[k]), (n,))


def _chain_n(x, b, k0, k1, init=None):
    acc = np.zeros(b.shape[1], np.float32) if init is None else init
    for k in range(k0, k1):
        acc = _fma(_bx(x, k, b.shape[1]), b[k], acc)
    return acc


def _two_acc(x, b, k0, size):
    n = b.shape[1]
    a = np.zeros(n, np.float32)
    e = np.zeros(n, np.float32)
    for q in range(size):
        if q & 1:
            e = _fma(_bx(x, k0 + q, n), b[k0 + q], e)
        else:
            a = _fma(_bx(x, k0 + q, n), b[k0 + q], a)
    return _f(a + e)


def _gemv_n_rows(x, b, two: bool):
    K, n = b.shape
    y = np.zeros(n, np.float32)
    for g in range(0, K - K % 8, 8):
        y = _f(y + (_two_acc(x, b, g, 8) if two else _chain_n(x, b, g, g + 8)))
    k = K - K % 8
    for size in (4, 2, 1):
        if (K % 8) & size:
            y = _f(y + (_two_acc(x, b, k, size) if (two and size == 4) else _chain_n(x, b, k, k + size)))
            k += size
    return y


def sgemv_n(b: np.ndarray, x: np.ndarray, threads: int | None = None) -> np.ndarray:
    """y = x @ b in OpenBLAS GEMV-N's order (b: [K, N] float32 row-major; x: [K])."""
    b = np.asarray(b, np.float32)
    x = np.asarray(x, np.float32)
    K, N = b.shape
    threads = openblas_threads() if threads is None else threads
    if K <= 48:
        return _chain_n(x, b, 0, K)
    if N < 4:
        t = np.zeros(N, np.float32)
        k = 0
        while k < (K & -4):
            t = _f(t + _fma(_bx(x, k, N), b[k], _mul(_bx(x, k + 1, N), b[k + 1])))
            k += 2
        return _chain_n(x, b, k, K, init=t)
    y = np.zeros(N, np.float32)
    for r0, r1 in thread_ranges(N, K, threads):
        w = r1 - r0
        m3 = w & 3
        m1 = w & -4
        m2 = (w & (NBMAX - 1)) - m3
        nb, p = NBMAX, r0
        while nb == NBMAX:
            m1 -= nb
            if m1 < 0:
                if m2 == 0:
                    break
                nb = m2
            r = nb % 16
            y[p:p + r] = _gemv_n_rows(x, b[:, p:p + r], True)
            y[p + r:p + nb] = _gemv_n_rows(x, b[:, p + r:p + nb], False)
            p += nb
        if m3:
            y[r1 - m3:r1] = _chain_n(x, b[:, r1 - m3:r1], 0, K)
    return y
