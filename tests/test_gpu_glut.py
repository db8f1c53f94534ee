"""The FFN-up epilogue's GELU chain as a table (round 4; nqk_glut.hip, the k_pg PG_GLUT
epilogue).  The reference chain is model.py Div -> Erf -> Add -> Mul -> Mul on f32
(numpy_helper.py:95-112 erf) followed by numpy_quantization.py:24-34 quantize.

* nqk_gelu_lut_build derives every entry from the exact chain and checks the whole table on
  all finite f32 inputs; nqk_gelu_lut_check repeats that check and must find a single altered
  threshold or output byte;
* the GEMM with the table epilogue equals the filtered-chain epilogue (itself pinned to the
  reference through k_qgemm_big, tests/test_gpu_pgemm.py) bit for bit, at the ViT-Base and
  ViT-Ti shapes, with small output scales that put many values next to rounding boundaries."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SQRT2_F32 = float(np.float32(1.4142135381698608))


def _build(s_out, zp, bw=8):
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    lut = DeviceArray((8192,), np.uint8)
    k = (ctypes.c_float * 5)()
    n = ctypes.c_int32(-1)
    _lib.call("nqk_gelu_lut_build", float(np.float32(s_out)), int(zp), bw, SQRT2_F32, 1.0, 0.5, lut.vp, k, ctypes.byref(n))
    return lut, k, n.value


def _check(lut, k, n, s_out, zp, bw=8):
    from numpy_quant import _lib
    bad = ctypes.c_uint64(0)
    _lib.call("nqk_gelu_lut_check", float(np.float32(s_out)), int(zp), bw, SQRT2_F32, 1.0, 0.5, lut.vp, k, n,
              ctypes.byref(bad))
    return bad.value


# (s_out, zp, bit width): the ViT-Base calibration's GELU outputs (tests/golden/api.json:
# s ~ 0.0109 .. 0.0124, zp -112 .. -114), ViT-Ti's (s ~ 0.0052 .. 0.0058, zp -95 .. -99: more
# than 512 buckets at the finest widths), the k_pg tests' parameters, other zero points and int4
CASES = [(0.012436897, -114, 8), (0.010944091, -112, 8), (0.0165, -118, 8), (0.0027, -9, 8), (0.0125, 0, 8),
         (0.05, -128, 8), (0.2, -7, 4), (0.05, 3, 4), (0.0123, -113, 7), (0.00566313, -98, 8), (0.00521903, -95, 8)]


@pytest.mark.parametrize("s_out,zp,bw", CASES)
@pytest.mark.parametrize("no1", [False, True])
def test_gelu_table_is_exact_on_every_float(s_out, zp, bw, no1, monkeypatch):
    """no1: NQK_GLUT_NO1=1, two-line bucket coordinates only (round 5 tries a single line first:
    k[2] == 0, the k_pg<PG_GLUT1> epilogue)."""
    if no1:
        monkeypatch.setenv("NQK_GLUT_NO1", "1")
    else:
        monkeypatch.delenv("NQK_GLUT_NO1", raising=False)
    lut, k, n = _build(s_out, zp, bw)
    if no1:
        assert k[2] != 0.0
    # small scales need more than the 128 x 256-tile kernel's 512 buckets: up to 1024 (the
    # 256 x 256-tile kernel's LDS)
    assert 0 < n <= (1024 if s_out < 0.006 else 512), n
    assert _check(lut, k, n, s_out, zp, bw) == 0


def test_gelu_table_check_finds_an_altered_entry():
    s_out, zp = 0.012436897, -114
    lut, k, n = _build(s_out, zp)
    assert n > 0
    tab = lut.to_host().view(np.uint32).reshape(-1, 2).copy()
    # the first entry with a threshold: move the threshold by one ulp, then swap its bytes
    i = int(np.nonzero(tab[:n, 0] != 0x7F800000)[0][n // 8 if n > 8 else 0])
    for mod in ("ulp", "bytes"):
        t = tab.copy()
        if mod == "ulp":
            t[i, 0] += 1
        else:
            t[i, 1] = ((t[i, 1] & 0xFFFF) << 16) | (t[i, 1] >> 16)
        from numpy_quant.device import DeviceArray
        alt = DeviceArray.from_host(t.reshape(-1).view(np.uint8))
        assert _check(alt, k, n, s_out, zp) > 0, mod


def test_gelu_table_refuses_other_chains():
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    lut = DeviceArray((8192,), np.uint8)
    k = (ctypes.c_float * 5)()
    n = ctypes.c_int32(-1)
    _lib.call("nqk_gelu_lut_build", 0.0124, -114, 8, 2.0, 1.0, 0.5, lut.vp, k, ctypes.byref(n))
    assert n.value == 0
    _lib.call("nqk_gelu_lut_build", 0.0124, -114, 16, SQRT2_F32, 1.0, 0.5, lut.vp, k, ctypes.byref(n))
    assert n.value == 0


def _gelu_gemm(M, N, K, s_out, zp, seed, table, monkeypatch, wm=0, wbits=8):
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, _gemm, _pack_b, _pack_pg
    rng = np.random.default_rng(seed)
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-24, 25, size=(N, K), dtype=np.int8) if wbits == 8 else rng.integers(-8, 8, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col_h = bt_h.astype(np.int64).sum(axis=1)
    col = DeviceArray.from_host(col_h)
    bias = DeviceArray.from_host((0.05 * rng.standard_normal(N)).astype(np.float32))
    packed, kind = _pack_b(bt, wbits)
    pg = _pack_pg(bt, wbits, 0, nibbles=kind == 2)
    zpa = -5
    colterm = DeviceArray.from_host((col_h * zpa).astype(np.int32))
    for v in ("NQK_NO_PROJ", "NQK_NO_F32X", "NQK_NO_PG", "NQK_NO_GLUT", "NQK_PG_WM"):
        monkeypatch.delenv(v, raising=False)
    if wm:
        monkeypatch.setenv("NQK_PG_WM", str(wm))
    e = _lib.Epilogue()
    obits = 8 if wbits == 8 else 4  # int4 weights come with 4-bit outputs (the int4 model)
    e.zp_flags, e.bit_width = _lib.ZP_COL, obits
    e.zpa, e.col, e.col_absmax = zpa, col.ptr, int(np.abs(col_h).max())
    e.bias, e.b_packed, e.colterm, e.bt_pg = bias.ptr, kind, colterm.ptr, pg.ptr
    e.group_cols = 1 << 30
    out = DeviceArray((M, N), np.int8)
    out.fill_zero()
    e.s_acc[0], e.s_out[0], e.zp_out[0], e.out[0] = float(np.float32(1.3e-4)), float(np.float32(s_out)), zp, out.ptr
    e.div, e.add1, e.mul2 = SQRT2_F32, 1.0, 0.5
    keep = None
    if table:
        lut, k, n = _build(s_out, zp, obits)
        assert n > 0
        e.gelu_lut, e.lut_n = lut.ptr, n
        for j in range(5):
            e.lut_k[j] = k[j]
        keep = lut
    _gemm(EPI_GELU, a, packed, 1, M, N, K, K, K, None, 0, 0, e)
    del keep
    return _lib.load().nqk_qgemm_last_kernel(), out.to_host()


@pytest.mark.parametrize("M,N,K,s_out,zp", [
    (128 * 197, 3072, 768, 0.012436897, -114), (300, 3072, 768, 0.0165, -118), (256 * 50, 3072, 768, 0.0125, 0),
    (128 * 197, 768, 192, 0.012436897, -114), (300, 768, 192, 0.05, -128),
    # ViT-Ti's GELU outputs: tables of more than 512 entries, which only the 256 x 256-tile kernel holds
    (256 * 197, 768, 192, 0.00521903, -95), (128 * 50 + 77, 3072, 768, 0.0027, -9),
])
@pytest.mark.parametrize("wm", [1, 2])
@pytest.mark.parametrize("no1", [False, True])
def test_pg_gelu_table_equals_filtered_chain(M, N, K, s_out, zp, wm, no1, monkeypatch):
    """wm 2: the 256 x 256-tile form of k_pg (both sides; K = 192 and M < 256 stay 128-row),
    and a table of more than 512 entries takes that form whatever wm says.  no1: two-line tables
    only (else a single-line table, k_pg<PG_GLUT1>, where one fits first)."""
    if no1:
        monkeypatch.setenv("NQK_GLUT_NO1", "1")
    else:
        monkeypatch.delenv("NQK_GLUT_NO1", raising=False)
    k0, ref = _gelu_gemm(M, N, K, s_out, zp, M + N, False, monkeypatch, wm)
    k1, got = _gelu_gemm(M, N, K, s_out, zp, M + N, True, monkeypatch, wm)
    two = wm == 2 and K != 192 and M >= 256
    big = _build(s_out, zp)[2] > 512
    assert (k0, k1) == (5 if two else 4, 7 if (two or big) else 6), (k0, k1)
    np.testing.assert_array_equal(ref, got)


@pytest.mark.parametrize("M", [128 * 197, 300])
def test_pg_gelu_table_int4_weights(M, monkeypatch):
    """the table epilogue on nibble-packed int4 weights (k_pg<PG_GLUT, B4>, the int4
    B = 256 forward's FFN-up) equals the filtered chain on the same weights, bit for bit."""
    s_out, zp = 0.05, 3  # 4-bit outputs (the table of CASES' (0.05, 3, 4))
    k0, ref = _gelu_gemm(M, 3072, 768, s_out, zp, M + 4, False, monkeypatch, wbits=4)
    k1, got = _gelu_gemm(M, 3072, 768, s_out, zp, M + 4, True, monkeypatch, wbits=4)
    assert (k0, k1) == (4, 6), (k0, k1)
    np.testing.assert_array_equal(ref, got)
