"""The persistent 16x16x64 projection GEMM (k_pg, nqk_pgemm.hip) against the
one-tile-per-workgroup 32x32x32 kernel (k_qgemm_big) on the same operands: bit-identical
outputs for every epilogue (QKV head split + quantize, GELU + quantize, bias + residual
with the f32 and the f64 dequantize), with many tiles per workgroup, with one, and with
ragged last tile rows.  Small output scales put many values next to rounding boundaries, so
the rounding filters' exact fallbacks run.  Reference: numpy_quantization.py:44-61 (q_matmul)
and the consumer chains of model.py:486-565, pinned to the reference's fixtures through
k_qgemm_big (tests/test_gpu_models.py, tests/test_gpu_b256.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _last_kernel():
    from numpy_quant import _lib
    return _lib.load().nqk_qgemm_last_kernel()


def _run(epi_name, M, N, K, s_out_scale, use_pg, no_f32x, monkeypatch, seed, kernel=2, bw=8, l1=False, proj=False):
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, EPI_QKV, EPI_RESID, _gemm, _pack_b, _pack_pg
    epi = {"qkv": EPI_QKV, "resid": EPI_RESID, "gelu": EPI_GELU}[epi_name]
    rng = np.random.default_rng(seed)
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    lim = {8: 24, 6: 32, 4: 8}[bw]  # weights inside the bit width's range
    bt_h = rng.integers(-lim, lim + (1 if bw == 8 else 0), size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col_h = bt_h.astype(np.int64).sum(axis=1)
    col = DeviceArray.from_host(col_h)
    bias = DeviceArray.from_host((0.05 * rng.standard_normal(N)).astype(np.float32))
    resid = DeviceArray.from_host(rng.standard_normal((M, N)).astype(np.float32))
    packed, kind = _pack_b(bt, bw)
    pg = _pack_pg(bt, bw, 1 if epi == EPI_RESID else 0, nibbles=kind == 2)
    assert pg is not None
    zpa = -5
    colterm = DeviceArray.from_host((col_h * zpa).astype(np.int32))
    for k in ("NQK_NO_PROJ", "NQK_NO_F32X", "NQK_NO_PG", "NQK_PG_NORESID"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.delenv("NQK_PROJ_RESID", raising=False)
    if proj:  # the round-2 persistent 256 x 256 kernel (k_proj) for the residual epilogue
        monkeypatch.setenv("NQK_PROJ_RESID", "1")
    else:
        monkeypatch.setenv("NQK_NO_PROJ", "1")
    monkeypatch.setenv("NQK_PG_WM", str(kernel))
    if no_f32x:
        monkeypatch.setenv("NQK_NO_F32X", "1")
    e = _lib.Epilogue()
    e.zp_flags, e.bit_width = _lib.ZP_COL, bw
    e.zpa, e.col, e.col_absmax = zpa, col.ptr, int(np.abs(col_h).max())
    e.bias, e.b_packed, e.colterm = bias.ptr, kind, colterm.ptr
    if l1:  # the weights' largest column L1 norm: the tighter |acc| bound of the f32 proof
        e.col_l1max = int(np.abs(bt_h.astype(np.int64)).sum(axis=1).max())
    e.bt_pg = pg.ptr if use_pg else None
    sa = 1.3e-4
    if epi == EPI_QKV:
        T, H, Dh = 197, N // 3 // 64, 64
        e.group_cols, e.tokens, e.heads, e.hdim = N // 3, T, H, Dh
        bufs = [DeviceArray((-(-M // T) * H * T, Dh), np.int8) for _ in range(3)]
        for g in range(3):
            e.s_acc[g] = float(np.float32(sa * (g + 1)))
            e.s_out[g] = (0.0021, 0.0173, 0.05)[g] * s_out_scale
            e.zp_out[g], e.out[g] = (3, -140, 0)[g] if bw == 8 else (3, -20, 0)[g], bufs[g].ptr
    elif epi == EPI_RESID:
        e.group_cols = 1 << 30
        bufs = [DeviceArray((M, N), np.float32)]
        e.s_acc[0], e.out[0], e.resid = float(np.float32(sa * 2)), bufs[0].ptr, resid.ptr
    else:
        e.group_cols = 1 << 30
        bufs = [DeviceArray((M, N), np.int8)]
        e.s_acc[0], e.s_out[0], e.zp_out[0], e.out[0] = float(np.float32(sa)), 0.0027 * s_out_scale, -9, bufs[0].ptr
        e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
    for b in bufs:
        b.fill_zero()
    _gemm(epi, a, packed, 1, M, N, K, K, K, None, 0, 0, e)
    host = dict(a=a.to_host(), bt=bt_h, colterm=col_h * zpa, bias=bias.to_host(), resid=resid.to_host(), e=e)
    return _last_kernel(), [b.to_host() for b in bufs], host


def _numpy_ref(epi_name, M, N, K, host):
    """The reference chain in NumPy (numpy_quantization.py:37-41 dequantize, model.py Add,
    numpy_quantization.py:24-34 quantize) for small cases."""
    e = host["e"]
    acc = host["a"].astype(np.int64) @ host["bt"].astype(np.int64).T - host["colterm"][None, :]
    if epi_name == "qkv":
        T, H, Dh, G = e.tokens, e.heads, e.hdim, e.group_cols
        outs = []
        for g in range(3):
            v = acc[:, g * G:(g + 1) * G]
            d = (v.astype(np.float64) * np.float64(np.float32(e.s_acc[g]))).astype(np.float32)
            y = d + host["bias"][g * G:(g + 1) * G]
            t = y / np.float32(e.s_out[g])
            q = np.rint(np.clip(np.float64(e.zp_out[g]) + t.astype(np.float64), -128, 127)).astype(np.int8)
            nimg = -(-M // T)
            o = np.zeros((nimg, H, T, Dh), np.int8)
            qq = np.zeros((nimg * T, G), np.int8)
            qq[:M] = q
            o[:] = qq.reshape(nimg, T, H, Dh).transpose(0, 2, 1, 3)
            outs.append(o.reshape(nimg * H * T, Dh))
        return outs
    return None


@pytest.mark.parametrize("epi_name,M,N,K,s_out_scale,no_f32x", [
    ("qkv", 256 * 197, 2304, 768, 1.0, False), ("qkv", 128 * 197, 2304, 768, 1.0, False),
    ("qkv", 197, 2304, 768, 1.0, False), ("qkv", 512, 2304, 768, 0.05, False),
    ("gelu", 128 * 50, 3072, 768, 1.0, False), ("gelu", 128 * 197, 3072, 768, 1.0, False),
    ("gelu", 300, 3072, 768, 0.1, False),
    ("resid", 128 * 200, 768, 768, 1.0, False), ("resid", 128 * 200, 768, 3072, 1.0, False),
    ("resid", 128 * 197, 768, 3072, 1.0, True), ("resid", 300, 768, 768, 1.0, False),
    ("resid", 256 * 197, 768, 3072, 1.0, False),
    # ragged last tile rows with more tiles than workgroup slots
    ("gelu", 128 * 50 + 77, 3072, 768, 1.0, False), ("resid", 128 * 200 + 50, 768, 768, 1.0, False),
    ("qkv", 128 * 197 + 64, 2304, 768, 1.0, False), ("resid", 256 * 97 + 128, 768, 3072, 1.0, False),
])
@pytest.mark.parametrize("kernel", [1, 2])
def test_pg_gemm_equals_big_tile(epi_name, M, N, K, s_out_scale, no_f32x, kernel, monkeypatch):
    """kernel 1: k_pg on 128 x 256 tiles (two 256-thread workgroups per CU); 2: k_pg on
    256 x 256 tiles (NQK_PG_WM=2: one 512-thread workgroup per CU, both row halves reading the
    same B stage; below 256 rows, or ragged in place, the launcher keeps the 128-row form)."""
    seed = M + N + K
    k0, ref, host = _run(epi_name, M, N, K, s_out_scale, False, no_f32x, monkeypatch, seed, kernel)
    k1, got, _ = _run(epi_name, M, N, K, s_out_scale, True, no_f32x, monkeypatch, seed, kernel)
    wm2 = kernel == 2 and M >= 256
    assert (k0, k1) == (1, 5 if wm2 else 4), (k0, k1)
    if M <= 1024:
        npref = _numpy_ref(epi_name, M, N, K, host)
        if npref is not None:
            bad_old = [int((x != r).sum()) for x, r in zip(ref, npref)]
            bad_new = [int((y != r).sum()) for y, r in zip(got, npref)]
            assert bad_old == [0] * len(npref) and bad_new == [0] * len(npref), (bad_old, bad_new)
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("epi_name,M,N,K,s_out_scale,no_f32x", [
    ("qkv", 256 * 197, 576, 192, 1.0, False), ("qkv", 197 * 3, 576, 192, 0.05, False),
    ("gelu", 128 * 197, 768, 192, 1.0, False), ("gelu", 300, 768, 192, 0.1, False),
    # ragged last 64-row tiles, more tiles than workgroup slots
    ("qkv", 197 * 13, 576, 192, 1.0, False), ("gelu", 64 * 1100 + 5, 768, 192, 1.0, False),
])
@pytest.mark.parametrize("rows", [64, 128])
def test_pg_gemm_vit_tiny_shapes(epi_name, M, N, K, s_out_scale, no_f32x, rows, monkeypatch):
    """ViT-Ti/16 widths (D = 192, 3 heads, MLP 768): K = 192 (a 3-step k loop) and N % 256 != 0
    (QKV 576: the last column tile's waves past N store through zero-size descriptors) — k_pg
    equals the one-tile-per-workgroup kernel bit for bit, and the NumPy chain for the small
    QKV case.  rows: the 64-row tile form (WM = 0, round 5, opt-in NQK_PG_WM0=1) and the
    128-row one.  (Residual epilogues at N = 192 stay on the other kernel.)"""
    monkeypatch.setenv("NQK_PG_WM0", "1" if rows == 64 else "0")
    seed = M + N + K + 1
    k0, ref, host = _run(epi_name, M, N, K, s_out_scale, False, no_f32x, monkeypatch, seed, 1)
    k1, got, _ = _run(epi_name, M, N, K, s_out_scale, True, no_f32x, monkeypatch, seed, 1)
    assert k0 in (0, 1) and k1 == 4, (k0, k1)
    if M <= 1024:
        npref = _numpy_ref(epi_name, M, N, K, host)
        if npref is not None:
            bad = [int((y != r).sum()) for y, r in zip(got, npref)]
            assert bad == [0] * len(npref), bad
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("epi_name,M,N,K,s_out_scale,no_f32x", [
    ("qkv", 128 * 197, 2304, 768, 1.0, False), ("qkv", 300, 2304, 768, 0.05, False),
    ("gelu", 128 * 50, 3072, 768, 1.0, False), ("gelu", 300, 3072, 768, 0.1, False),
    ("resid", 128 * 200, 768, 768, 1.0, False), ("resid", 128 * 197, 768, 3072, 1.0, False),
    ("resid", 300, 768, 3072, 1.0, True), ("resid", 256 * 197, 768, 3072, 1.0, False),
])
def test_pg_gemm_int4_equals_big_tile(epi_name, M, N, K, s_out_scale, no_f32x, monkeypatch):
    """BASELINE configs[4]: int4 weights as the nqk_pack_pg4 nibble image on k_pg (B operand
    unpacked after the LDS stage, 16 x the products accumulated, >> 4 in the epilogue), 4-bit
    output clamps: equal to k_qgemm_big on its own nibble image (nqk_pack_b4), bit for bit."""
    seed = M + N + K + 4
    k0, ref, _ = _run(epi_name, M, N, K, s_out_scale, False, no_f32x, monkeypatch, seed, 1, bw=4)
    k1, got, _ = _run(epi_name, M, N, K, s_out_scale, True, no_f32x, monkeypatch, seed, 1, bw=4)
    assert (k0, k1) == (1, 4), (k0, k1)
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("M,seed", [(128 * 197, 11), (256 * 197, 12), (300, 13)])
def test_pg_resid_k3072_f32_dequant_from_column_l1_bound(M, seed, monkeypatch):
    """FFN-down (K = 3072): 2^14 K exceeds 2^24, so without more information the residual
    epilogue dequantizes in f64; with the weights' largest column L1 norm (col_l1max) the
    bound 128 L1 + |zpa| cmax < 2^24 proves the f32 dequantize exact.  Both runs of k_pg
    (the f32 one by the L1 bound, the f64 one with NQK_NO_F32X=1) are bit-identical."""
    k1, f32, _ = _run("resid", M, 768, 3072, 1.0, True, False, monkeypatch, seed, 1, l1=True)
    k2, f64, _ = _run("resid", M, 768, 3072, 1.0, True, True, monkeypatch, seed, 1, l1=True)
    assert (k1, k2) == (4, 4), (k1, k2)
    for x, y in zip(f32, f64):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("epi_name,M,N,K,s_out_scale", [
    ("qkv", 128 * 197, 2304, 768, 1.0), ("qkv", 300, 2304, 768, 0.05),
    ("gelu", 128 * 50, 3072, 768, 1.0), ("gelu", 300, 3072, 768, 0.1),
])
def test_pg_gemm_bw6_equals_big_tile(epi_name, M, N, K, s_out_scale, monkeypatch):
    """bit widths below 8 (here 6: int8 storage, the 6-bit output clamps of the QKV
    blo/bhi and the GELU qlo/qhi) on k_pg equal k_qgemm_big bit for bit."""
    seed = M + N + K + 6
    k0, ref, _ = _run(epi_name, M, N, K, s_out_scale, False, False, monkeypatch, seed, 1, bw=6)
    k1, got, _ = _run(epi_name, M, N, K, s_out_scale, True, False, monkeypatch, seed, 1, bw=6)
    assert (k0, k1) == (1, 4), (k0, k1)
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("M,seed", [(256 * 197, 21), (256 * 4, 22)])
def test_proj_resid_k3072_f32_dequant_equals_f64(M, seed, monkeypatch):
    """the round-2 persistent residual kernel (k_proj, NQK_PROJ_RESID=1) at K = 3072,
    reachable in f32 through the column-L1 bound (col_l1max), equals its f64-dequantize run
    (NQK_NO_F32X=1) bit for bit."""
    k1, f32, _ = _run("resid", M, 768, 3072, 1.0, False, False, monkeypatch, seed, 1, l1=True, proj=True)
    k2, f64, _ = _run("resid", M, 768, 3072, 1.0, False, True, monkeypatch, seed, 1, l1=True, proj=True)
    assert (k1, k2) == (3, 3), (k1, k2)
    for x, y in zip(f32, f64):
        np.testing.assert_array_equal(x, y)
