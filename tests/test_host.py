"""Host-side logic that needs no GPU: the ONNX reader, batch maps, dimension
collapsing, reshape targets, the pairwise-sum plan and the BLAS K blocking."""
import os

import numpy as np
import pytest

from conftest import ROOT
from numpy_quant import onnx_proto
from numpy_quant.kernels import batch_map
from numpy_quant.device import collapse, contiguous_strides, broadcast_strides, _Pool
from numpy_quant.tensor import _reshape_target

MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")


def test_mlp_graph_matches_reference_summary():
    # test/test_mlp.py:82-103 (IR summary of models/mlp.onnx)
    m = onnx_proto.load(os.path.join(MODELS, "mlp.onnx"))
    g = m.graph
    rows = [(n.name, n.op_type, list(n.input), list(n.output)) for n in g.node]
    assert rows == [
        ("/fc1/Gemm", "Gemm", ["input", "fc1.weight", "fc1.bias"], ["/fc1/Gemm_output_0"]),
        ("/relu/Relu", "Relu", ["/fc1/Gemm_output_0"], ["/relu/Relu_output_0"]),
        ("/fc2/Gemm", "Gemm", ["/relu/Relu_output_0", "fc2.weight", "fc2.bias"], ["/fc2/Gemm_output_0"]),
        ("/sigmoid/Sigmoid", "Sigmoid", ["/fc2/Gemm_output_0"], ["output"]),
    ]
    attrs = {a.name: onnx_proto.attribute_value(a) for a in g.node[0].attribute}
    assert attrs == {"alpha": 1.0, "beta": 1.0, "transB": 1}
    w = {t.name: t.to_array() for t in g.initializer}
    assert w["fc1.weight"].shape == (5, 2) and w["fc1.weight"].dtype == np.float32
    assert sum(v.size for v in w.values()) == 27


def test_vit_graph_and_rebatch():
    m = onnx_proto.load(os.path.join(MODELS, "vit_image_classifier_no_weights.onnx"), synthetic_weights=True)
    ops = {}
    for n in m.graph.node:
        ops[n.op_type] = ops.get(n.op_type, 0) + 1
    assert len(m.graph.node) == 516
    assert ops["MatMul"] == 96 and ops["LayerNormalization"] == 25 and ops["Gemm"] == 1 and ops["Conv"] == 1
    assert sum(int(np.prod(t.dims)) for t in m.graph.initializer) == 86567656
    assert onnx_proto.rebatch(m, 4) == 49
    with pytest.raises(FileNotFoundError):
        onnx_proto.load(os.path.join(MODELS, "vit_image_classifier_no_weights.onnx"))


def test_synthetic_weights_deterministic():
    a = onnx_proto.synthetic_array("x.weight", (4, 5))
    b = onnx_proto.synthetic_array("x.weight", (4, 5))
    c = onnx_proto.synthetic_array("layernorm.weight", (8,))
    assert np.array_equal(a, b) and a.dtype == np.float32
    assert abs(float(c.mean()) - 1.0) < 0.1 and c.min() != c.max()


@pytest.mark.parametrize("a,b", [((2, 1), (1, 2)), ((8, 12), (8, 12)), ((8,), ()), ((), (3,)), ((3, 1, 5), (1, 4, 5)),
                                 ((2, 3), (3,))])
def test_batch_map_reproduces_numpy_broadcast(a, b):
    out, bm = batch_map(a, b)
    assert out == np.broadcast_shapes(a, b)
    ia = np.arange(int(np.prod(a))).reshape(a) if a else np.array(0)
    ib = np.arange(int(np.prod(b))).reshape(b) if b else np.array(0)
    ea, eb = np.broadcast_arrays(ia, ib)
    if bm is None:
        pytest.skip("materialised broadcast")
    inner, ao, ai, bo, bi = bm
    for k in range(int(np.prod(out))):
        assert (k // inner) * ao + (k % inner) * ai == ea.reshape(-1)[k]
        assert (k // inner) * bo + (k % inner) * bi == eb.reshape(-1)[k]


def test_collapse_and_broadcast_strides():
    shp, (s1, s2) = collapse((2, 3, 4), contiguous_strides((2, 3, 4)), contiguous_strides((2, 3, 4)))
    assert shp == [24] and s1 == [1] and s2 == [1]
    st = broadcast_strides((3, 1), (2, 3, 4))
    assert st == [0, 1, 0]
    shp, (sa, sb) = collapse((256, 197, 768), broadcast_strides((256, 197, 768), (256, 197, 768)),
                             broadcast_strides((768,), (256, 197, 768)))
    assert shp == [256 * 197, 768] and sb == [0, 1]


def test_reshape_target_and_pool_rounding():
    assert _reshape_target((1, 197, 768), np.array([1, 197, 12, 64])) == (1, 197, 12, 64)
    assert _reshape_target((4, 768, 14, 14), np.array([4, 768, -1])) == (4, 768, 196)
    with pytest.raises(ValueError):
        _reshape_target((2, 3), np.array([4, -1]))
    assert _Pool.round(1) == 256 and _Pool.round(257) == 512
    assert _Pool.round(3 << 20) >= 3 << 20


def blas_blocks(K, Q=448, U=2):
    out, ls = [], 0
    while ls < K:
        m = K - ls
        if m >= 2 * Q:
            m = Q
        elif m > Q:
            m = ((m // 2 + U - 1) // U) * U
        out.append(m)
        ls += m
    return out


def test_blas_blocking_rule_matches_numpy_dot():
    """The block structure nqk_sgemm uses (OpenBLAS level-3 K loop, GEMM_Q = 448)."""
    assert blas_blocks(768) == [384, 384]
    assert blas_blocks(500) == [250, 250]
    assert blas_blocks(700) == [350, 350]
    assert blas_blocks(64) == [64]
    assert blas_blocks(3072) == [448] * 5 + [416, 416]
    assert blas_blocks(1536) == [448, 448, 320, 320]


def _fma_chain_blocks(a, w, K):
    """Per output element: a k-ordered f32 fma chain from 0 in every BLAS block, block
    results added in order (a*b is exact in f64 for f32 operands; one f64 add then the
    f32 rounding stands in for the fused rounding)."""
    f32 = lambda x: x.astype(np.float32).astype(np.float64)  # noqa: E731
    acc = np.zeros((a.shape[0], w.shape[1]))
    ls = 0
    for m in blas_blocks(K):
        c = np.zeros_like(acc)
        for k in range(ls, ls + m):
            c = f32(a[:, k:k + 1] * w[k:k + 1, :] + c)
        acc = f32(acc + c)
        ls += m
    return acc


@pytest.mark.parametrize("K", [384, 768, 1000, 3072])
def test_blas_order_matches_numpy_matmul(K):
    """nqk_sgemm's summation order (GEMM_Q = 448 K blocks, k-ordered fma chains) is the
    order of the NumPy the reference runs on (scipy-openblas 0.3.29, SkylakeX kernels):
    an emulation of it equals np.matmul bit for bit on the FFN-down shape (K = 3072) and
    the others.  Skipped where OpenBLAS picks other kernels."""
    threadpoolctl = pytest.importorskip("threadpoolctl")
    info = [i for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"]
    if not info or info[0].get("architecture") != "SkylakeX":
        pytest.skip("OpenBLAS does not run its SkylakeX kernels on this host")
    rng = np.random.default_rng(K)
    A = np.maximum(rng.standard_normal((40, K)).astype(np.float32), -0.17)
    W = (0.02 * rng.standard_normal((K, 64))).astype(np.float32)
    C = A @ W
    rows, cols = np.arange(0, 40, 5), np.arange(0, 64, 9)
    got = _fma_chain_blocks(A[rows].astype(np.float64), W[:, cols].astype(np.float64), K)
    np.testing.assert_array_equal(got.astype(np.float32), C[np.ix_(rows, cols)])


def _proto_view(m):
    """onnx_proto's decode in _onnx_walk's shape."""
    def val(a):
        if a.type == onnx_proto.ATTR_TENSOR:
            return ("tensor", tuple(a.t.dims), a.t.data_type)
        v = onnx_proto.attribute_value(a)
        if isinstance(v, bytes):
            return v.decode()
        if isinstance(v, list):
            return tuple(v)
        return v
    g = m.graph
    nodes = [(n.name, n.op_type, tuple(n.input), tuple(n.output), {a.name: val(a) for a in n.attribute}) for n in g.node]
    inits = [(t.name, tuple(t.dims), t.data_type) for t in g.initializer]
    return nodes, inits, [v.name for v in g.input], [v.name for v in g.output]


@pytest.mark.parametrize("fname", ["mlp.onnx", "vit_image_classifier_no_weights.onnx",
                                   "vit_image_classifier_encoder_layer_no_weights.onnx",
                                   "vit_image_classifier_self_attention_no_weights.onnx"])
def test_onnx_decode_matches_independent_reader(fname):
    """The product's ONNX decoder against a separately written wire-format reader
    (tests/_onnx_walk.py) on every graph the fixtures use: every node's name, op type,
    inputs, outputs and attribute values, every initializer's name, shape and element
    type, the graph inputs and outputs (the fixtures and the product
    share onnx_proto, so it needs a pin of its own)."""
    import _onnx_walk
    path = os.path.join(MODELS, fname)
    want = _onnx_walk.read(path)
    got = _proto_view(onnx_proto.load(path, synthetic_weights="no_weights" in fname))
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2] and got[3] == want[3]


_GEMV_CASES = [(768, 1000, 8), (768, 1000, 3), (768, 1000, 4), (768, 1001, 8), (772, 1001, 8), (780, 2001, 8),
               (770, 1000, 8), (771, 37, 1), (769, 60, 1), (5000, 30, 1), (8200, 17, 1), (4100, 130, 8),
               (100, 90, 1), (9, 300, 1), (12, 64, 1), (4, 2304, 1), (1, 50, 1), (3072, 300, 8), (256, 2001, 8)]


@pytest.mark.parametrize("K,N,threads", _GEMV_CASES)
def test_sgemv_order_matches_numpy_matmul(K, N, threads):
    """oracle/openblas_order.py (OpenBLAS 0.3.29 GEMV-T: thread split of the columns, the
    4x4 / 4x2 / 4x1 kernels' lane orders, K blocks, trailing rows) equals np.matmul of a
    one-row product against a transposed weight, the reference's classifier Gemm at batch
    1 (model.py:122-131), bit for bit, at OpenBLAS thread counts 1..8.  Skipped where
    OpenBLAS runs other kernel families."""
    threadpoolctl = pytest.importorskip("threadpoolctl")
    info = [i for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"]
    if not info or info[0].get("architecture") not in ("Haswell", "Zen", "SkylakeX", "Cooperlake", "SapphireRapids"):
        pytest.skip("OpenBLAS does not run its Haswell-family GEMV kernels on this host")
    from oracle.openblas_order import sgemv_t
    rng = np.random.default_rng(K * 7 + N)
    x = rng.standard_normal(K).astype(np.float32)
    w = (0.05 * rng.standard_normal((N, K))).astype(np.float32)
    with threadpoolctl.threadpool_limits(limits=threads, user_api="blas"):
        ref = (x[None, :] @ w.T)[0]
    np.testing.assert_array_equal(sgemv_t(w, x, threads).view(np.int32), ref.view(np.int32))


def _openblas_haswell_family():
    threadpoolctl = pytest.importorskip("threadpoolctl")
    info = [i for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"]
    if not info or info[0].get("architecture") not in ("Haswell", "Zen", "SkylakeX", "Cooperlake", "SapphireRapids"):
        pytest.skip("OpenBLAS does not run its Haswell-family GEMV kernels on this host")
    return threadpoolctl


@pytest.mark.parametrize("K", [1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 31])
def test_small_one_row_orders_match_numpy_matmul(K):
    """oracle/openblas_order.py's GEMV-T for K <= 8 (OpenBLAS's small-m kernels per thread chunk
    of at most 16 384 columns, the regular kernels for wider chunks; round 6 identified every
    column class) equals np.matmul bit for bit on every column: N = 2..70 and chunks around
    16 384 columns at OpenBLAS thread counts 1, 3 and 8; kernels.one_row_restated says so."""
    threadpoolctl = _openblas_haswell_family()
    from oracle.openblas_order import sgemv_t
    from numpy_quant.kernels import one_row_restated
    rng = np.random.default_rng(1000 + K)
    big = [16383, 16384, 16385, 57601, 70001, 131075] if K <= 8 else [20001]
    for threads in (1, 3, 8):
        for N in (list(range(2, 71)) if threads == 8 else [2, 5, 37, 70]) + big:
            x = rng.standard_normal(K).astype(np.float32)
            w = rng.standard_normal((N, K)).astype(np.float32)
            with threadpoolctl.threadpool_limits(limits=threads, user_api="blas"):
                ref = (x[None, :] @ w.T)[0]
            np.testing.assert_array_equal(sgemv_t(w, x, threads).view(np.int32), ref.view(np.int32),
                                          err_msg=f"K={K} N={N} threads={threads}")
            assert one_row_restated(N, K)


def test_sdot_order_matches_numpy_matmul():
    """oracle/openblas_order.py sdot (cblas_sdot: the SkylakeX vector kernel's accumulators
    from 32 elements, the tail in double) equals np.matmul's 1 x 1 product bit for bit at every
    length class (below 32, 32-element steps, 64-element steps, ragged tails, 4 M elements)."""
    threadpoolctl = _openblas_haswell_family()
    from oracle.openblas_order import sdot
    rng = np.random.default_rng(77)
    for n in list(range(1, 200)) + [255, 256, 257, 768, 3072, 4099, 65537, 1 << 22]:
        x = rng.standard_normal(n).astype(np.float32)
        w = rng.standard_normal(n).astype(np.float32)
        for threads in ((1, 8) if n > 10000 else (8,)):
            with threadpoolctl.threadpool_limits(limits=threads, user_api="blas"):
                ref = np.matmul(x[None, :], w[:, None])[0, 0]
            assert sdot(x, w).view(np.int32) == ref.view(np.int32), (n, threads)


_GEMV_N_CASES = [(49, 2), (64, 3), (3072, 2), (16, 4100), (48, 9000), (49, 4100), (64, 9000), (768, 4095),
                 (49, 12289), (768, 700), (768, 3072), (3072, 768), (57, 8191), (200, 4099), (5000, 7), (100, 5),
                 (50, 16), (59, 36), (63, 28), (2, 40), (9, 33)]


@pytest.mark.parametrize("K,N", _GEMV_N_CASES)
def test_sgemv_n_order_matches_numpy_matmul(K, N):
    """oracle/openblas_order.py sgemv_n (round 6: OpenBLAS GEMV-N for a one-row product against
    a row-major matrix — K <= 48 fma chains, N < 4 pairs, the 8- / 16-row kernels' groups of 8
    per block of 4096 outputs, trailing outputs, the thread split) equals np.matmul bit for bit
    at OpenBLAS thread counts 1, 3 and 8; and matrix @ vector equals GEMV-T over the matrix's
    rows (sgemv_t)."""
    threadpoolctl = _openblas_haswell_family()
    from oracle.openblas_order import sgemv_n, sgemv_t
    rng = np.random.default_rng(K * 131 + N)
    for threads in (1, 3, 8):
        b = rng.standard_normal((K, N)).astype(np.float32)
        x = rng.standard_normal(K).astype(np.float32)
        with threadpoolctl.threadpool_limits(limits=threads, user_api="blas"):
            ref = np.matmul(x[None, :], b)[0]
            ref_mv = np.matmul(b.T.copy(), x[:, None])[:, 0]  # matrix [N, K] @ vector
        np.testing.assert_array_equal(sgemv_n(b, x, threads).view(np.int32), ref.view(np.int32),
                                      err_msg=f"K={K} N={N} threads={threads}")
        np.testing.assert_array_equal(sgemv_t(b.T.copy(), x, threads).view(np.int32), ref_mv.view(np.int32),
                                      err_msg=f"matrix @ vector K={K} N={N} threads={threads}")


def test_redimension_vit_base_to_tiny():
    """onnx_proto.redimension (the metric's ViT-tiny from the reference's ViT-Base graph):
    every width-768 / MLP-3072 initializer dimension and the head / width Reshape
    constants follow (192, 3 heads of 64, 768), the oracle's float forward runs and the
    synthetic weights stay deterministic."""
    from oracle import nq_oracle as O
    path = os.path.join(MODELS, "vit_image_classifier_no_weights.onnx")
    m = onnx_proto.load(path, synthetic_weights=True)
    n = onnx_proto.redimension(m, 192, 3, 768)
    dims = {tuple(t.dims) for t in m.graph.initializer}
    assert not any(768 in d and d != (192, 768) and d != (768, 192) and d != (768,) for d in dims)
    assert (192, 3, 16, 16) in dims and (1000, 192) in dims and (192, 768) in dims and (768, 192) in dims
    consts = [tuple(onnx_proto.to_array(a.t).tolist()) for nd in m.graph.node if nd.op_type == "Constant"
              for a in nd.attribute if a.name == "value" and onnx_proto.to_array(a.t).dtype == np.int64
              and onnx_proto.to_array(a.t).ndim == 1 and onnx_proto.to_array(a.t).size in (3, 4)]
    assert (1, 197, 3, 64) in consts and (1, 197, 192) in consts and (1, 197, 12, 64) not in consts
    assert n == 247
    x = np.random.default_rng(0).standard_normal((1, 3, 224, 224)).astype(np.float32)
    g = O.Graph(m)
    out = O.outputs_of(g, O.float_forward(g, [x]))[0]
    assert out.shape == (1, 1000) and np.isfinite(out).all()
    m2 = onnx_proto.load(path, synthetic_weights=True)
    onnx_proto.redimension(m2, 192, 3, 768)
    a = {t.name: onnx_proto.to_array(t) for t in m.graph.initializer}
    for t in m2.graph.initializer:
        np.testing.assert_array_equal(onnx_proto.to_array(t), a[t.name])
    with pytest.raises(ValueError):
        onnx_proto.redimension(onnx_proto.load(path, synthetic_weights=True), 192, 4, 768)


def test_embed_fold_guard_per_stream_part():
    """nqk_embed_q's 32-bit output offsets need (images x 197) x 768 < 2^31 per call
    (one call per stream part); past that the plan keeps the patchify path instead of failing."""
    from numpy_quant.plan import Streams, embed_q_fits
    two, one = Streams(True, 2), Streams(False)
    assert two.max_part(256) == 128 and two.max_part(257) == 129 and one.max_part(257) == 257
    assert embed_q_fits(two.max_part(256), 196, 768)
    assert embed_q_fits(14_000, 196, 768) and not embed_q_fits(14_200, 196, 768)
    assert embed_q_fits(two.max_part(28_000), 196, 768)       # 14 000 per part
    assert not embed_q_fits(two.max_part(28_500), 196, 768)   # 14 250 per part: past 2^31
    assert not embed_q_fits(one.max_part(20_000), 196, 768)   # one stream: the whole batch in one call
    assert not embed_q_fits(45_000, 196, 64)                  # 65535 row tiles


def test_fused_away_value_raises_on_read():
    """reading a value that a fused step never materialised raises a RuntimeError
    (FusedAwayError), also through NumPy's array conversion; protocol probes see a missing
    attribute."""
    from numpy_quant.plan import FusedAway, FusedAwayError
    v = FusedAway("x")
    with pytest.raises(FusedAwayError):
        v.data
    with pytest.raises(FusedAwayError):
        np.asarray(v)
    assert not isinstance(FusedAwayError("m"), AttributeError)
    assert getattr(v, "__array_interface__", None) is None


@pytest.mark.parametrize("bw", [2, 4, 8])
def test_ln_magic_quantize_equals_f64_chain(bw):
    """The LayerNorm kernels' output quantize (nqk_fused.hip ln_quant4, round 5) restated in NumPy
    f32 arithmetic: c = med3(t, lo - zp, hi - zp), s = RN32(c + 1.5 2^23 + zp), the low byte of
    bits(s) — equal to the reference's rint(clip(zp + t, lo, hi)) in f64 (numpy_quantization.py:
    24-34) for every t tried: exact half-integers (ties to even with odd and even zero points),
    their neighbouring floats, the clamp bounds, infinities and random values, |zp| <= 2^20."""
    lo, hi = -(2 ** (bw - 1)), 2 ** (bw - 1) - 1
    rng = np.random.default_rng(bw)
    for zp in (-(1 << 20), -300, -129, -128, -7, -1, 0, 1, 2, 3, 127, 140, 1 << 20):
        k = np.arange(lo - zp - 3, hi - zp + 4, dtype=np.float64)
        half = (k + 0.5).astype(np.float32)
        t = np.concatenate([half, np.nextafter(half, np.float32(np.inf)), np.nextafter(half, np.float32(-np.inf)),
                            k.astype(np.float32), (rng.standard_normal(20000) * (hi - lo)).astype(np.float32) - zp,
                            np.array([np.inf, -np.inf, 3e38, -3e38], np.float32)]).astype(np.float32)
        ref = np.rint(np.clip(np.float64(zp) + t.astype(np.float64), lo, hi)).astype(np.int64)
        qlo, qhi = np.float32(lo - zp), np.float32(hi - zp)
        magic = np.float32(1.5 * 2 ** 23) + np.float32(zp)
        c = np.minimum(np.maximum(t, qlo), qhi)
        s = (c + magic).astype(np.float32)
        got = (s.view(np.uint32) & 0xFF).astype(np.int64)
        got = np.where(got >= 128, got - 256, got)
        np.testing.assert_array_equal(got, ref, err_msg=f"zp {zp}")


def test_ln_dma_swizzle_conflict_free():
    """k_ln_quant_lds with NQK_LN_DMA (nqk_fused.hip ln_swz): the row image loaded by LDS-DMA is
    XOR-swizzled so that the tree reads (lane (row, leaf, grp) reads 16-B chunk 24 leaf + 2 i + grp
    of its row) put the 16 lanes of every ds_read_b128 lane group (MI355X_MICROARCH.md, LDS table)
    on 16 different 4-bank slots, for 8, 4 and 2 leaves; the swizzle is a permutation of each row
    that stays inside the leaf (its own inverse), so the loader can use it both ways."""
    groups = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32))]
    groups += [[g + 32 for g in grp] for grp in groups]

    def swz(nl, r, c):  # nqk_fused.hip ln_swz
        return c ^ (((((c // 24) >> 1) & 3) if nl == 8 else (r & 3)) << 1)

    for nl in (8, 4, 2):
        ch, lpr = 24 * nl, 2 * nl
        for r in range(64 // lpr):
            row = [swz(nl, r, c) for c in range(ch)]
            assert sorted(row) == list(range(ch))
            assert all(swz(nl, r, swz(nl, r, c)) == c and swz(nl, r, c) // 24 == c // 24 for c in range(ch))
        for i in range(12):
            for grp in groups:
                slots = set()
                for lane in grp:
                    r, u = lane // lpr, lane % lpr
                    leaf, g = u >> 1, u & 1
                    slots.add((r * ch + swz(nl, r, 24 * leaf + 2 * i + g)) % 16)
                assert len(slots) == 16, (nl, i, grp)
