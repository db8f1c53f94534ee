"""The attention's P-quantize filter margins (nqk_attn.hip NQK_ATTN_PM_R / NQK_ATTN_PM_T /
NQK_ATTN_PKL), restated in NumPy f32 arithmetic and checked on elements placed next to rounding
boundaries: whenever the fast path's measure passes its limit, its byte equals the reference
chain's (numpy_helper.py softmax, then numpy_quantization.py:24-34 quantize:
t = RN(RN(e / tot) / s_p), q = rint(clip(zp + t, lo, hi))).  A margin below the proven bound
must show mismatches on the same inputs, so the check has teeth."""
import numpy as np
import pytest

U = 2.0 ** -24
LIMIT = np.float32(0.5 - 2.0 ** -23)  # 0x1.fffff8p-2


def _f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def _fma32(a, b, c):
    # f32 fma: the product of two f32 values is exact in f64; one rounding to f32 after the add
    return _f32(a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64))


def _cases(n, seed, zp=-142):
    rng = np.random.default_rng(seed)
    tot = _f32(rng.uniform(1.0, 200.0, n))
    s_p = _f32(10.0 ** rng.uniform(-5.5, -2.0, n))
    lo, hi = -128, 127
    # targets next to half-integers inside (and around) the unclamped range
    k = rng.integers(-20, 400, n).astype(np.float64)
    delta = rng.uniform(-1, 1, n) * np.abs(k + 0.5) * 2.0 ** -19
    x = k + 0.5 + delta
    e = _f32(np.clip(x * tot.astype(np.float64) * s_p.astype(np.float64), 0, 1))
    # the reference chain (f32 divisions are correctly rounded in NumPy)
    p = e / tot
    t = p / s_p
    q_ref = np.rint(np.clip(zp + t.astype(np.float64), lo, hi)).astype(np.int64)
    kd = (1.0 / tot.astype(np.float64)) * (1.0 / s_p.astype(np.float64))
    kpf = _f32(kd)
    kpl = _f32(kd - kpf.astype(np.float64))
    pqlo, pqhi = np.float32(lo - zp), np.float32(hi - zp)
    return e, kpf, kpl, q_ref, pqlo, pqhi, zp


def _clamped_path(e, kpf, kpl, pqlo, pqhi, zp, margin, pkl):
    if pkl:
        tf = _f32(e.astype(np.float64) * kpf.astype(np.float64) + _f32(e.astype(np.float64) * kpl.astype(np.float64)))
    else:
        tf = e * kpf
    c = np.clip(tf, pqlo, pqhi)
    r = np.rint(c)
    dd = c - r
    meas = _fma32(np.abs(tf), np.full_like(tf, margin), np.abs(dd))
    return meas < LIMIT, r.astype(np.int64) + zp


def _clampfree_path(e, kpf, zp, margin):
    prod = e.astype(np.float64) * kpf.astype(np.float64)  # exact
    r = np.rint(prod)
    dd = _f32(prod - r)
    meas = _fma32(np.abs(_f32(r)), np.full_like(dd, margin), np.abs(dd))
    return meas < LIMIT, r.astype(np.int64) + zp


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_clamped_path_margin(seed):
    e, kpf, kpl, q_ref, pqlo, pqhi, zp = _cases(400_000, seed)
    ok, q = _clamped_path(e, kpf, kpl, pqlo, pqhi, zp, np.float32(4.125 * U), False)
    assert ok.mean() > 0.3
    assert np.array_equal(q[ok], q_ref[ok])
    ok, q = _clamped_path(e, kpf, kpl, pqlo, pqhi, zp, np.float32(3.125 * U), True)
    assert np.array_equal(q[ok], q_ref[ok])
    # without a margin the filter passes wrong bytes on these inputs
    ok, q = _clamped_path(e, kpf, kpl, pqlo, pqhi, zp, np.float32(0.0), False)
    assert not np.array_equal(q[ok], q_ref[ok])


@pytest.mark.parametrize("seed", [3, 4])
def test_clampfree_path_margin(seed):
    e, kpf, kpl, q_ref, pqlo, pqhi, zp = _cases(400_000, seed, zp=0)
    inside = (q_ref > -128) & (q_ref < 127)  # the clamp-free path runs only where no clamp is reached
    e, kpf, q_ref = e[inside], kpf[inside], q_ref[inside]
    ok, q = _clampfree_path(e, kpf, 0, np.float32(4.75 * U))
    assert ok.mean() > 0.3
    assert np.array_equal(q[ok], q_ref[ok])
    ok, q = _clampfree_path(e, kpf, 0, np.float32(0.0))
    assert not np.array_equal(q[ok], q_ref[ok])
