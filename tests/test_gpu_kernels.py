"""GPU parity, kernels: numpy-exact float building blocks and the integer GEMMs on
shapes beyond the golden vectors (odd sizes, batches, broadcasts, ViT shapes),
against NumPy on the same seeded inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def init():
    from numpy_quant import _lib
    _lib.ensure_init()


def test_exp_matches_numpy_on_64M_floats():
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant import kernels as K
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2 ** 32, size=1 << 24, dtype=np.uint64).astype(np.uint32)
    dense = np.linspace(-110, 100, 1 << 22, dtype=np.float32)
    for x in (bits.view(np.float32), dense):
        y = K.unary(_lib.EXP, DeviceArray.from_host(x)).to_host()
        with np.errstate(all="ignore"):
            ref = np.exp(x)
        same = (y.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(y) & np.isnan(ref))
        assert same.all(), (x[~same][:5], y[~same][:5], ref[~same][:5])


def test_fast_division_exp_erf_exhaustive():
    """The fused kernels use exp / erf with a 4-instruction division (v_rcp_f32 + one
    residual correction).  That division is not correctly rounded in general, so the
    fast functions are used only because they equal the IEEE-division ones bit for bit
    on every one of the 2^32 float inputs, which this test establishes on the device."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    counts = DeviceArray.from_host(np.zeros(5, np.uint64))
    ex = DeviceArray.from_host(np.zeros(5, np.uint32))
    _lib.call("nqk_selftest_fastmath", counts.vp, ex.vp)
    c, e = counts.to_host(), ex.to_host()
    assert c[0] == 0, f"fast exp differs on {c[0]} inputs, e.g. {e[0:1].view(np.float32)}"
    assert c[1] == 0, f"fast erf differs on {c[1]} inputs, e.g. {e[1:2].view(np.float32)}"
    assert c[2] == 0, f"non-positive exp differs on {c[2]} inputs, e.g. {e[2:3].view(np.float32)}"
    assert c[3] == 0, f"packed non-positive exp differs on {c[3]} inputs, e.g. {e[3:4].view(np.float32)}"
    assert c[4] == 0, f"exp on [-86.5, 0] by exponent add differs on {c[4]} inputs, e.g. {e[4:5].view(np.float32)}"


def test_gelu_filter_bound_exhaustive():
    """The GELU epilogue computes a cheap approximation first and falls back to the
    exact chain wherever the approximation's error bound could change the quantized
    value.  This test proves the bound |fast - exact| <= 2^-21 |h| + 2^-60 on every
    f32 input with |h| < 2^64 (the others always take the exact chain)."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    st = DeviceArray.from_host(np.zeros(258, np.uint64))
    _lib.call("nqk_selftest_gelu_filter", st.vp)
    s = st.to_host()
    worst = {e - 127: int(v) for e, v in enumerate(s[2:]) if v}
    print("max error per exponent (units of |h| 2^-24):", worst)
    assert s[0] == 0, f"{s[0]} inputs exceed the bound, e.g. h = {np.uint32(s[1]).view(np.float32)}"


@pytest.mark.parametrize("rows,cols", [(7, 5), (33, 128), (64, 197), (17, 768), (9, 3072), (3, 1000), (2, 129)])
def test_pairwise_softmax_layernorm(rows, cols):
    from numpy_quant.tensor import FTensor
    from numpy_quant.model import onnx_operator_implementation as op
    rng = np.random.default_rng(rows * cols)
    x = (rng.standard_normal((rows, cols)) * 3).astype(np.float32)
    g = (1 + 0.02 * rng.standard_normal(cols)).astype(np.float32)
    b = (0.02 * rng.standard_normal(cols)).astype(np.float32)
    sm = op("Softmax", [FTensor(x)], {"axis": -1})[0].data
    m = x + (-x.max(axis=-1, keepdims=True))
    e = np.exp(m)
    np.testing.assert_array_equal(sm, e / e.sum(axis=-1, keepdims=True))
    ln = op("LayerNormalization", [FTensor(x), FTensor(g), FTensor(b)], {"axis": -1, "epsilon": 1e-12})[0].data
    mean = x.mean(axis=-1, keepdims=True)
    d = x + (-mean)
    var = (d * d).mean(axis=-1, keepdims=True)
    ref = d * (np.float32(1) / np.sqrt(var + np.float32(1e-12))) * g + b
    np.testing.assert_array_equal(ln, ref)
    np.testing.assert_array_equal(FTensor(x).mean(-1, keepdims=True).data, x.mean(-1, keepdims=True))


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (5, 3, 2), (100, 5, 2), (197, 768, 768), (256, 100, 700),
                                   (130, 70, 500), (64, 300, 384), (3, 1000, 768)])
def test_sgemm_matches_blas(M, N, K):
    from numpy_quant.tensor import FTensor
    rng = np.random.default_rng(M + N + K)
    a = rng.standard_normal((M, K), dtype=np.float32)
    b = rng.standard_normal((K, N), dtype=np.float32)
    got = FTensor(a).matmul(FTensor(b)).data
    ref = np.matmul(a, b)
    if M == 1 or N == 1:  # NumPy uses gemv there: not the gemm summation order
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    else:
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("shape_a,shape_b", [((197, 768), (768, 768)), ((2, 197, 768), (768, 3072)),
                                             ((4, 12, 197, 64), (4, 12, 64, 197)), ((4, 12, 197, 197), (4, 12, 197, 64)),
                                             ((33, 17), (17, 45)), ((2, 1, 40, 48), (1, 2, 48, 40)),
                                             ((129, 3072), (3072, 130))])
@pytest.mark.parametrize("zps", [(None, None), (-9, None), (None, 5), (-138, 11)])
def test_int8_gemm_and_zero_point_terms(shape_a, shape_b, zps):
    from numpy_quant import numpy_quantization as nq
    rng = np.random.default_rng(sum(shape_a) + sum(shape_b))
    a = rng.integers(-128, 128, size=shape_a, dtype=np.int64)
    b = rng.integers(-128, 128, size=shape_b, dtype=np.int64)
    za = None if zps[0] is None else np.array(zps[0], np.int64)
    zb = None if zps[1] is None else np.array(zps[1], np.int64)
    acc, s, z = nq.q_matmul(a, np.float32(0.5), za, b, np.float32(0.25), zb)
    np.testing.assert_array_equal(acc, np.matmul(a, b))
    if za is None and zb is None:
        assert z is None
    else:
        ra = a.sum(axis=-1, keepdims=True)
        cb = b.sum(axis=-2, keepdims=True)
        if za is None:
            ref = ra * zb
        elif zb is None:
            ref = cb * za
        else:
            ref = ra * zb + cb * za - za * zb * a.shape[-1]
        np.testing.assert_array_equal(z, ref)
        d = nq.dequantize(acc, np.float32(0.125), z)
        np.testing.assert_array_equal(d, ((acc - ref) * np.float32(0.125)).astype(np.float32))


def test_wide_bit_width_gemm():
    from numpy_quant import numpy_quantization as nq
    rng = np.random.default_rng(3)
    a = rng.integers(-2 ** 15, 2 ** 15, size=(37, 50), dtype=np.int64)
    b = rng.integers(-2 ** 15, 2 ** 15, size=(50, 29), dtype=np.int64)
    acc, _, z = nq.q_matmul(a, np.float32(1), np.array(7, np.int64), b, np.float32(1), None)
    np.testing.assert_array_equal(acc, a @ b)
    np.testing.assert_array_equal(z, b.sum(axis=-2, keepdims=True) * 7)


def test_quantize_rowsum_and_graph_capture():
    from numpy_quant import _lib, kernels as K
    from numpy_quant.device import DeviceArray
    import ctypes
    rng = np.random.default_rng(11)
    x = (rng.standard_normal((300, 197)) * 4).astype(np.float32)
    dx = DeviceArray.from_host(x)
    q, rs = K.quantize(dx, 8, np.float32(0.05), -3, rowsum=True)
    qh = q.to_host().astype(np.int64)
    from oracle import nq_oracle as O
    ref = O.quantize(x, 8, np.array(0.05, np.float32), np.array(-3, np.int64))
    np.testing.assert_array_equal(qh, ref)
    np.testing.assert_array_equal(rs.to_host(), ref.sum(axis=-1))
    # capture the same quantize into a hipGraph and replay it
    out = DeviceArray(x.shape, np.int8)
    _lib.call("nqk_graph_begin")
    _lib.call("nqk_quantize", dx.vp, out.vp, out.code, x.size, float(np.float32(0.05)), -3, 1, 8, None, 197)
    g = ctypes.c_void_p()
    _lib.call("nqk_graph_end", ctypes.byref(g))
    _lib.call("nqk_graph_launch", g)
    np.testing.assert_array_equal(out.to_host().astype(np.int64), ref)
    _lib.call("nqk_graph_destroy", g)


@pytest.mark.parametrize("batch,M,N,K", [(1, 50176 // 8, 768, 768), (1, 197, 768, 768), (3, 130, 257, 1000),
                                         (2, 256, 200, 386), (1, 129, 131, 2)])
def test_sgemm_mfma_equals_fma_chain_kernel(batch, M, N, K, monkeypatch):
    """v_mfma_f32_32x32x2_f32 path vs the VALU fmaf-chain kernel (both in the BLAS K
    blocking, nqk_sgemm): bit-identical, including batched and ragged tiles."""
    from numpy_quant import kernels as KM
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(M * N + K)
    a = DeviceArray.from_host(rng.standard_normal((batch, M, K), dtype=np.float32))
    b = DeviceArray.from_host(rng.standard_normal((batch, K, N), dtype=np.float32))
    bmap = [1, 1, 0, 1, 0]
    got = KM.sgemm(a, K, 1, b, N, 1, M, N, K, batch=batch, bmap=bmap, a_ms=M * K, b_ms=K * N).to_host()
    monkeypatch.setenv("NQK_SGEMM_VALU", "1")
    ref = KM.sgemm(a, K, 1, b, N, 1, M, N, K, batch=batch, bmap=bmap, a_ms=M * K, b_ms=K * N).to_host()
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("K,N,threads", [(768, 1000, 8), (768, 1000, 3), (768, 1000, 16), (772, 1001, 8),
                                         (780, 2001, 8), (770, 1000, 4), (771, 37, 1), (5000, 30, 1),
                                         (8200, 17, 1), (4100, 130, 8), (9, 300, 1), (4, 2304, 1), (1, 50, 1),
                                         (3072, 300, 64)])
def test_sgemv_t_matches_openblas_order(K, N, threads):
    """nqk_sgemv_t (one-row float product against a transposed weight: the reference's
    classifier Gemm at batch 1, model.py:122-131 -> np.matmul -> OpenBLAS GEMV-T) equals
    the oracle's restatement of OpenBLAS's order (oracle/openblas_order.py, pinned to
    np.matmul by tests/test_host.py) bit for bit, at several OpenBLAS thread counts."""
    from numpy_quant import kernels as KM
    from numpy_quant.device import DeviceArray
    from oracle.openblas_order import sgemv_t
    rng = np.random.default_rng(K + 3 * N)
    x = rng.standard_normal(K).astype(np.float32)
    w = (0.05 * rng.standard_normal((N, K))).astype(np.float32)
    old = KM.BLAS_THREADS
    KM.BLAS_THREADS = threads
    try:
        got = KM.sgemv_t(DeviceArray.from_host(x[None, :]), DeviceArray.from_host(w)).to_host()[0]
    finally:
        KM.BLAS_THREADS = old
    want = sgemv_t(w, x, threads)
    np.testing.assert_array_equal(got.view(np.int32), want.view(np.int32))


def test_one_row_gemm_takes_gemv_order():
    """Model-level: a float Gemm(transB=1) on one row (model.py:122-131) goes through the
    GEMV-T order, a two-row one through the GEMM order: both bit-exact vs the oracle's
    restatements of what NumPy does there."""
    from numpy_quant.model import onnx_operator_implementation
    from numpy_quant.tensor import FTensor
    from oracle.openblas_order import sgemv_t
    rng = np.random.default_rng(5)
    w = (0.05 * rng.standard_normal((1000, 768))).astype(np.float32)
    b = rng.standard_normal(1000).astype(np.float32)
    x1 = rng.standard_normal((1, 768)).astype(np.float32)
    y1 = onnx_operator_implementation("Gemm", [FTensor(x1), FTensor(w), FTensor(b)], {"transB": 1})[0].data
    np.testing.assert_array_equal(y1, (sgemv_t(w, x1[0], 8) + b)[None, :])


@pytest.mark.parametrize("K,N,threads", [(49, 2, 8), (64, 3, 1), (3072, 2, 8), (16, 4100, 8), (48, 9000, 8),
                                         (49, 4100, 1), (64, 9000, 3), (768, 4095, 8), (49, 12289, 8), (768, 700, 2),
                                         (768, 3072, 8), (3072, 768, 8), (57, 8191, 1), (200, 4099, 8), (5000, 7, 1),
                                         (100, 5, 8), (59, 36, 1), (63, 28, 8), (2, 40, 8), (1025, 3000, 64)])
def test_sgemv_n_matches_openblas_order(K, N, threads):
    """nqk_sgemv_n (one-row float product against a row-major matrix: a MatMul on one row,
    tensor.py:100-101 -> np.matmul -> OpenBLAS GEMV-N; round 6) equals the oracle's restatement
    (oracle/openblas_order.py sgemv_n, pinned to np.matmul by tests/test_host.py) bit for bit:
    every regime (K <= 48 chains, N < 4 pairs, 8- / 16-row kernels, 4096-output blocks, trailing
    outputs, thread chunks)."""
    from numpy_quant import kernels as KM
    from numpy_quant.device import DeviceArray
    from oracle.openblas_order import sgemv_n
    rng = np.random.default_rng(K + 7 * N)
    x = rng.standard_normal(K).astype(np.float32)
    b = rng.standard_normal((K, N)).astype(np.float32)
    old = KM.BLAS_THREADS
    KM.BLAS_THREADS = threads
    try:
        got = KM.sgemv_n(DeviceArray.from_host(x[None, :]), DeviceArray.from_host(b)).to_host()[0]
    finally:
        KM.BLAS_THREADS = old
    np.testing.assert_array_equal(got.view(np.int32), sgemv_n(b, x, threads).view(np.int32))


def test_matmul_level2_products_take_blas2_orders():
    """FTensor.matmul (tensor.py:100-101 -> np.matmul) where a product has a vector side: vector
    @ matrix (GEMV-N), matrix @ vector (GEMV-T over the matrix's rows), vector @ vector (sdot),
    2-D and stacked (a batch of one-row products against one broadcast weight) — each equal to
    the oracle's restatement of NumPy's BLAS call, bit for bit."""
    from numpy_quant import kernels as KM
    from numpy_quant.device import DeviceArray
    from oracle.openblas_order import sdot, sgemv_n, sgemv_t
    rng = np.random.default_rng(12)
    t = KM.openblas_threads()
    for K, N in ((768, 3072), (64, 10), (33, 5), (100, 2)):
        x = rng.standard_normal((1, K)).astype(np.float32)
        b = rng.standard_normal((K, N)).astype(np.float32)
        got = KM.matmul_f32(DeviceArray.from_host(x), DeviceArray.from_host(b)).to_host()
        np.testing.assert_array_equal(got[0].view(np.int32), sgemv_n(b, x[0], t).view(np.int32), err_msg=f"{K} {N}")
        a = rng.standard_normal((N, K)).astype(np.float32)
        v = rng.standard_normal((K, 1)).astype(np.float32)
        got = KM.matmul_f32(DeviceArray.from_host(a), DeviceArray.from_host(v)).to_host()
        np.testing.assert_array_equal(got[:, 0].view(np.int32), sgemv_t(a, v[:, 0], t).view(np.int32), err_msg=f"mv {K} {N}")
        got = KM.matmul_f32(DeviceArray.from_host(x), DeviceArray.from_host(v)).to_host()
        assert got.shape == (1, 1) and got[0, 0].view(np.int32) == sdot(x[0], v[:, 0]).view(np.int32)
    xs = rng.standard_normal((3, 1, 96)).astype(np.float32)
    b = rng.standard_normal((96, 40)).astype(np.float32)
    got = KM.matmul_f32(DeviceArray.from_host(xs), DeviceArray.from_host(b)).to_host()
    assert got.shape == (3, 1, 40)
    for i in range(3):
        np.testing.assert_array_equal(got[i, 0].view(np.int32), sgemv_n(b, xs[i, 0], t).view(np.int32))


@pytest.mark.parametrize("M,N,K", [(1000, 768, 768), (197, 192, 768), (130, 260, 64), (50176 // 16, 768, 768)])
def test_sgemm_vector_loads_equal_scalar_loads(M, N, K, monkeypatch):
    """k_sgemm_mfma's 16-byte operand loads (unit-stride A rows and B rows) give the same
    bits as its scalar-load form (NQK_SGEMM_SCALAR=1), plain and patch-embedding paths."""
    from numpy_quant import kernels as KM
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(M + N + K)
    a = DeviceArray.from_host(rng.standard_normal((M, K), dtype=np.float32))
    b = DeviceArray.from_host(rng.standard_normal((K, N), dtype=np.float32))
    got = KM.sgemm(a, K, 1, b, N, 1, M, N, K).to_host()
    hw = M  # one image of M patches through the embedding epilogue
    bias = DeviceArray.from_host(rng.standard_normal(N, dtype=np.float32))
    cls = DeviceArray.from_host(rng.standard_normal(N, dtype=np.float32))
    pos = DeviceArray.from_host(rng.standard_normal((hw + 1, N), dtype=np.float32))
    out = DeviceArray((1, hw + 1, N), np.float32)
    _lib.call("nqk_sgemm_embed", a.vp, b.vp, bias.vp, cls.vp, pos.vp, out.vp, 1, hw, N, K)
    emb = out.to_host()
    monkeypatch.setenv("NQK_SGEMM_SCALAR", "1")
    ref = KM.sgemm(a, K, 1, b, N, 1, M, N, K).to_host()
    _lib.call("nqk_sgemm_embed", a.vp, b.vp, bias.vp, cls.vp, pos.vp, out.vp, 1, hw, N, K)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(emb, out.to_host())
