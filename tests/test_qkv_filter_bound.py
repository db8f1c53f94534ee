"""The QKV epilogue's rounding filter (nqk_pgemm_kernel.h, k_pg EPI QKV, NQK_PG_QK1 / NQK_PG_QKC2),
restated in NumPy f32 arithmetic and checked on elements placed next to rounding boundaries
(ADVICE r4).  Fast side: u = fma(v, c1, c2) with c1 = RN(sacc rsf), c2 = RN(bias rsf),
rsf = RN(1 / s_out); it passes when fma(|v|, k1, |u - rint(u)|) < lim, k1 = |c1| 6.25 2^-24,
lim = (Q_LIM - |c2| 5.25 2^-24) - 2^-22, and then outputs rint(u) + zp.  Reference chain
(numpy_quantization.py:37-41 dequantize, model.py Add, numpy_quantization.py:24-34 quantize):
t = RN(RN(RN(v sacc) + bias) / s_out), q = rint(clip(zp + t, lo, hi)).  Every passing element
must equal the reference; with zero margins the same inputs show mismatches, so the check has
teeth."""
import numpy as np
import pytest

U = 2.0 ** -24
Q_LIM = np.float32(float.fromhex("0x1.fffffcp-2"))


def _f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def _fma32(a, b, c):
    # f32 fma: the f32 x f32 product is exact in f64; one rounding to f32 after the add
    return _f32(a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64))


def _cases(n, seed):
    rng = np.random.default_rng(seed)
    s_out = _f32(10.0 ** rng.uniform(-3.0, -1.0, n))
    # sacc / s_out >= 2^-16: |v| stays far below 2^24 (the F32X condition)
    sacc = _f32(s_out.astype(np.float64) * 10.0 ** rng.uniform(-4.5, -2.5, n))
    bias = _f32(rng.standard_normal(n) * s_out.astype(np.float64) * 20.0)
    zp = rng.integers(-128, 128, n)
    k = rng.integers(-250, 250, n).astype(np.float64)
    target = (k + 0.5) * s_out.astype(np.float64) - bias.astype(np.float64)
    v = np.rint(target / sacc.astype(np.float64)) + rng.integers(-2, 3, n)
    assert np.abs(v).max() < 2 ** 24
    vf = _f32(v)
    # the reference chain: dequantize (one rounding of the exact product), bias add, divide
    d = _f32(v * sacc.astype(np.float64))
    y = _f32(d.astype(np.float64) + bias.astype(np.float64))
    t = _f32(y.astype(np.float64) / s_out.astype(np.float64))  # a correctly rounded f32 division
    q_ref = np.rint(np.clip(zp + t.astype(np.float64), -128, 127)).astype(np.int64)
    return vf, sacc, bias, s_out, zp, q_ref


def _fast(vf, sacc, bias, s_out, zp, qk1, qkc2):
    rsf = _f32(1.0 / s_out.astype(np.float64))
    c1 = _f32(sacc.astype(np.float64) * rsf.astype(np.float64))
    c2 = _f32(bias.astype(np.float64) * rsf.astype(np.float64))
    k1 = _f32(np.abs(c1).astype(np.float64) * qk1)
    u = _fma32(vf, c1, c2)
    rr = np.rint(u)
    dd = _f32(u.astype(np.float64) - rr.astype(np.float64))
    meas = _fma32(np.abs(vf), k1, np.abs(dd))
    lim = _f32(_f32(Q_LIM.astype(np.float64) - _f32(np.abs(c2).astype(np.float64) * qkc2).astype(np.float64))
               - 2.0 ** -22)
    q = np.clip(rr.astype(np.int64) + zp, -128, 127)
    return meas < lim, q


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_qkv_filter_margins(seed):
    vf, sacc, bias, s_out, zp, q_ref = _cases(1_000_000, seed)
    ok, q = _fast(vf, sacc, bias, s_out, zp, 6.25 * U, 5.25 * U)
    assert ok.mean() > 0.5
    assert np.array_equal(q[ok], q_ref[ok]), int((q[ok] != q_ref[ok]).sum())
    # without the margins the filter passes wrong bytes on the same inputs
    ok0, q0 = _fast(vf, sacc, bias, s_out, zp, 0.0, 0.0)
    assert int((q0[ok0] != q_ref[ok0]).sum()) > 0
