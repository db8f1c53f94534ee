"""GPU parity of the fused-plan element kernels against NumPy / the oracle on the same
seeded inputs: nqk_ln_quant (LayerNormalization model.py:134-152 -> quantize
numpy_quantization.py:24-34), both the register-tree path (rows of 2, 4 or 8 leaves
of 96 columns) and the LDS path.  Integer outputs: bit-exact."""
import ctypes

import numpy as np
import pytest

from oracle import nq_oracle as O

pytestmark = pytest.mark.gpu


def _ln_ref(x, g, b, eps):
    mean = x.mean(axis=-1, keepdims=True)
    d = x + (-mean)
    var = (d * d).mean(axis=-1, keepdims=True)
    return d * (np.float32(1) / np.sqrt(var + np.float32(eps))) * g + b


@pytest.mark.parametrize("rows,cols", [(1, 768), (257, 768), (1000, 192), (33, 384), (64, 197), (5, 1000),
                                       (3, 96), (7, 3072)])
@pytest.mark.parametrize("bw,zp", [(8, -3), (8, 140), (4, 2)])
@pytest.mark.parametrize("path", ["lds", "reg"])
def test_ln_quant(rows, cols, bw, zp, path, monkeypatch):
    from numpy_quant import _lib
    if path == "reg":
        monkeypatch.setenv("NQK_LN_REG", "1")
    else:
        monkeypatch.delenv("NQK_LN_REG", raising=False)
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(rows * cols + bw)
    x = (rng.standard_normal((rows, cols)) * 2 + 0.3).astype(np.float32)
    g = (1 + 0.02 * rng.standard_normal(cols)).astype(np.float32)
    b = (0.02 * rng.standard_normal(cols)).astype(np.float32)
    eps = np.float32(1e-12)
    s = np.float32(0.031) if bw == 8 else np.float32(0.6)
    ref = O.quantize(_ln_ref(x, g, b, eps), bw, s, np.int64(zp))
    dx, dg, db = DeviceArray.from_host(x), DeviceArray.from_host(g), DeviceArray.from_host(b)
    out = DeviceArray((rows, cols), np.int8)
    _lib.call("nqk_ln_quant", dx.vp, dg.vp, db.vp, out.vp, rows, cols, float(eps), float(s), zp, bw)
    np.testing.assert_array_equal(out.to_host().astype(np.int64), ref)


@pytest.mark.parametrize("rows,cols", [(4109, 768), (40000, 192), (9001, 384)])
@pytest.mark.parametrize("variant", ["NQK_LN_WPB=1", "NQK_LN_WPB=2", "NQK_LN_WPB=4", "NQK_LN_PERS=1", "NQK_LN_PERS=4",
                                     "NQK_LN_PERS=6"])
def test_ln_quant_workgroup_forms_match_oracle(rows, cols, variant, monkeypatch):
    """Every launch form of the LDS LayerNorm (nqk_fused.hip: 1 / 2 / 4 row groups per workgroup;
    the persistent double-buffered k_ln_quant_pers at 1 / 4 / 6 waves per CU, whose waves walk
    many row groups with the next group's LDS-DMA in flight — 40 000 x 192 at one wave per CU is
    ~10 groups per wave; ragged last groups) against the oracle, bit for bit."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    monkeypatch.delenv("NQK_LN_REG", raising=False)
    k, v = variant.split("=")
    monkeypatch.setenv(k, v)
    rng = np.random.default_rng(rows + cols)
    x = (rng.standard_normal((rows, cols)) * 3 - 0.7).astype(np.float32)
    g = (1 + 0.05 * rng.standard_normal(cols)).astype(np.float32)
    b = (0.05 * rng.standard_normal(cols)).astype(np.float32)
    s, zp = np.float32(0.0021), 5
    dx, dg, db = DeviceArray.from_host(x), DeviceArray.from_host(g), DeviceArray.from_host(b)
    out = DeviceArray((rows, cols), np.int8)
    _lib.call("nqk_ln_quant", dx.vp, dg.vp, db.vp, out.vp, rows, cols, 1e-5, float(s), zp, 8)
    ref = O.quantize(_ln_ref(x, g, b, np.float32(1e-5)), 8, s, np.int64(zp))
    np.testing.assert_array_equal(out.to_host().astype(np.int64), ref)


@pytest.mark.parametrize("s,zp,bw", [(0.031, -3, 8), (0.0021, 5, 8), (0.0007, -120, 8), (0.45, 1, 4), (0.031, 1 << 20, 8)])
def test_ln_quant_lds_small_scales_match_oracle(s, zp, bw, monkeypatch):
    """The LDS LayerNorm + quantize on ViT-Base rows (4109 x 768: a ragged last workgroup)
    with small output scales (many values next to rounding boundaries), 4-bit outputs and
    a zero point of 2^20, against the oracle's LayerNorm chain and quantize, bit for bit."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    monkeypatch.delenv("NQK_LN_REG", raising=False)
    rng = np.random.default_rng(int(s * 1e4) + bw)
    rows, cols = 4096 + 13, 768
    x = (rng.standard_normal((rows, cols)) * 3 - 0.7).astype(np.float32)
    g = (1 + 0.05 * rng.standard_normal(cols)).astype(np.float32)
    b = (0.05 * rng.standard_normal(cols)).astype(np.float32)
    dx, dg, db = DeviceArray.from_host(x), DeviceArray.from_host(g), DeviceArray.from_host(b)
    out = DeviceArray((rows, cols), np.int8)
    _lib.call("nqk_ln_quant", dx.vp, dg.vp, db.vp, out.vp, rows, cols, 1e-5, float(np.float32(s)), zp, bw)
    ref = O.quantize(_ln_ref(x, g, b, np.float32(1e-5)), bw, np.float32(s), np.int64(zp))
    np.testing.assert_array_equal(out.to_host().astype(np.int64), ref)


@pytest.mark.parametrize("s_out,zp,bw", [(0.041, -7, 8), (0.0023, 0, 8), (0.31, -3, 4), (1e-5, 100, 8)])
def test_gelu_epilogue_filter_matches_exact_chain(s_out, zp, bw, monkeypatch):
    """FFN-up GEMM with the GELU epilogue (model.py MatMul -> Add -> Div -> Erf -> Add ->
    Mul -> Mul -> quantize): the filtered epilogue (cheap GELU where its proven error
    bound cannot change the rounding, exact chain elsewhere) equals the exact chain
    everywhere.  Small output scales put many values next to rounding boundaries."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, _gemm
    rng = np.random.default_rng(int(s_out * 1e6) + bw)
    M, N, K = 1024 + 77, 3072, 768
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-20, 21, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col = DeviceArray.from_host(bt_h.astype(np.int64).sum(axis=1))
    bias = DeviceArray.from_host((0.02 * rng.standard_normal(N)).astype(np.float32))
    outs = []
    for flag in (None, "1"):
        if flag:
            monkeypatch.setenv("NQK_NO_GELU_FILTER", flag)
        out = DeviceArray((M, N), np.int8)
        e = _lib.Epilogue()
        e.zp_flags, e.bit_width, e.group_cols = _lib.ZP_COL, bw, 1 << 30
        e.zpa, e.col = 5, col.ptr
        e.s_acc[0] = float(np.float32(1.3e-4))
        e.s_out[0], e.zp_out[0], e.out[0] = s_out, zp, out.ptr
        e.bias = bias.ptr
        e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
        _gemm(EPI_GELU, a, bt, 1, M, N, K, K, K, None, 0, 0, e)
        outs.append(out.to_host())
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("n,c,h,w,kh,kw,zp", [(2, 3, 224, 224, 16, 16, -5), (1, 3, 32, 48, 16, 16, 0),
                                             (3, 2, 12, 15, 4, 5, 7), (1, 1, 8, 8, 2, 2, -128)])
def test_patchify_dequant_equals_dequantize_then_im2col(n, c, h, w, kh, kw, zp):
    """Conv input path of the fused patch embedding: dequantize (numpy_quantization.py:37-41)
    then numpy_helper.py:18-70 sliding windows, in one pass over the int8 input."""
    from numpy_quant import _lib
    from numpy_quant import kernels as KM
    from numpy_quant.device import DeviceArray
    rng = np.random.default_rng(h * w + c)
    q = rng.integers(-128, 128, size=(n, c, h, w), dtype=np.int8)
    s = np.float32(0.0173)
    x = O.dequantize(q.astype(np.int64), s, np.int64(zp) if zp else None)
    ref_cols, _, _ = KM.im2col(DeviceArray.from_host(x), kh, kw, (0, 0, 0, 0), (kh, kw))
    cols = DeviceArray(ref_cols.shape, np.float32)
    _lib.call("nqk_patchify_dequant", DeviceArray.from_host(q).vp, cols.vp, n, c, h, w, kh, kw, float(s), zp)
    np.testing.assert_array_equal(cols.to_host(), ref_cols.to_host())


@pytest.mark.parametrize("n,h,w,N,zp", [(3, 224, 224, 768, -5), (2, 224, 224, 192, 0), (1, 32, 48, 64, 17),
                                        (5, 64, 32, 128, -128)])
@pytest.mark.parametrize("mfma", ["32", "16"])
def test_embed_q_equals_patchify_then_sgemm_embed(n, h, w, N, zp, mfma, monkeypatch):
    """nqk_embed_q (patchify + dequantize folded into the GEMM's A-operand load, round 3)
    gives the bits of nqk_patchify_dequant + nqk_sgemm_embed (the im2col path, pinned to the
    reference's fconv2d by test_gpu_kernels / vit_b1): bias, position embedding and the
    class-token rows included; ragged last row tile (n * hw % 128 != 0) and N = 64 / 192;
    both kernel forms (v_mfma_f32_32x32x2_f32 and, round 6, 16x16x4), each with its weight
    order (plan.embed_weight_image)."""
    monkeypatch.setenv("NQK_EMBED_MFMA", mfma)
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray, permute
    from numpy_quant.plan import embed_weight_image
    rng = np.random.default_rng(n * 1000 + N)
    q = rng.integers(-128, 128, size=(n, 3, h, w), dtype=np.int8)
    s = np.float32(0.0173)
    W = (0.05 * rng.standard_normal((N, 3, 16, 16))).astype(np.float32)
    hw = (h // 16) * (w // 16)
    bias = DeviceArray.from_host((0.1 * rng.standard_normal(N)).astype(np.float32))
    cls = DeviceArray.from_host(rng.standard_normal(N).astype(np.float32))
    pos = DeviceArray.from_host(rng.standard_normal((hw + 1, N)).astype(np.float32))
    Wd = DeviceArray.from_host(W)
    wm = permute(Wd, [2, 3, 1, 0]).reshape((768, N))
    cols = DeviceArray((n * hw, 768), np.float32)
    qd = DeviceArray.from_host(q)
    _lib.call("nqk_patchify_dequant", qd.vp, cols.vp, n, 3, h, w, 16, 16, float(s), zp)
    ref = DeviceArray((n, hw + 1, N), np.float32)
    _lib.call("nqk_sgemm_embed", cols.vp, wm.vp, bias.vp, cls.vp, pos.vp, ref.vp, n, hw, N, 768)
    assert _lib.load().nqk_embed_weight_order() == int(mfma)
    wt = embed_weight_image(Wd, N, 768)
    out = DeviceArray((n, hw + 1, N), np.float32)
    _lib.call("nqk_embed_q", qd.vp, float(s), zp, wt.vp, bias.vp, cls.vp, pos.vp, out.vp, n, 3, h, w, 16, 16, N)
    np.testing.assert_array_equal(out.to_host().view(np.int32), ref.to_host().view(np.int32))


_VARIANTS = [{}, {"NQK_GEMM_PP": "1"}, {"NQK_NO_F32X": "1"}, {"NQK_NO_F32X": "1", "NQK_GEMM_PP": "1"},
             {"NQK_NO_GELU_FILTER": "1", "NQK_NO_F32X": "1"}, {"PACK": "1"}, {"PACK": "1", "NQK_NO_F32X": "1"}]


@pytest.mark.parametrize("epi_name,M,N,K,zpa,s_out,zp", [
    ("qkv", 4 * 197, 2304, 768, -7, (0.021, 0.0173, 0.05), (3, -140, 0)),
    ("qkv", 2 * 197, 2304, 192, 131, (0.9, 0.0011, 2.5e-3), (0, 17, -3)),
    ("resid", 1024 + 77, 772, 768, 5, (1, 1, 1), (0, 0, 0)),
    ("resid", 512, 768, 3072, -120, (1, 1, 1), (0, 0, 0)),
    ("gelu", 1024 + 77, 3072, 768, -3, (0.0027, 1, 1), (-9, 0, 0)),
    ("gelu", 300, 772, 192, 140, (0.05, 1, 1), (2, 0, 0)),
    ("resid", 77, 256, 192, 3, (1, 1, 1), (0, 0, 0)),
    ("gelu", 513, 512, 1536, -1, (0.02, 1, 1), (0, 0, 0)),
])
def test_projection_gemm_variants_agree(epi_name, M, N, K, zpa, s_out, zp, monkeypatch):
    """Projection GEMM variants: the 128x256 kernel (k_qgemm_big) with row-major or
    tile-packed weights (nqk_pack_b), the ping-pong 256x256 kernel (k_qgemm_pp), f64 or
    proven-exact f32 epilogue arithmetic with rounding filters,
    GELU filter on or off -- all bit-identical, on ragged tiles and small output scales
    that put many values next to rounding boundaries.  The exact-chain variant is itself
    checked against the reference's node loop by the plan tests."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, EPI_QKV, EPI_RESID, _gemm
    epi = {"qkv": EPI_QKV, "resid": EPI_RESID, "gelu": EPI_GELU}[epi_name]
    rng = np.random.default_rng(M + N + K + zpa)
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-24, 25, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col_h = bt_h.astype(np.int64).sum(axis=1)
    col = DeviceArray.from_host(col_h)
    bias = DeviceArray.from_host((0.05 * rng.standard_normal(N)).astype(np.float32))
    resid = DeviceArray.from_host(rng.standard_normal((M, N)).astype(np.float32))
    from numpy_quant.plan import _pack_b
    packed = _pack_b(bt)  # (image, 1), or None where the big-tile kernel does not take the shape
    packed = None if packed is None else packed[0]
    outs = []
    for var in _VARIANTS:
        if "PACK" in var and packed is None:
            continue
        for k in ("NQK_GEMM_PP", "NQK_NO_F32X", "NQK_NO_GELU_FILTER"):
            monkeypatch.delenv(k, raising=False)
        for k, v in var.items():
            if k != "PACK":
                monkeypatch.setenv(k, v)
        e = _lib.Epilogue()
        e.zp_flags, e.bit_width = _lib.ZP_COL, 8
        e.zpa, e.col, e.col_absmax = zpa, col.ptr, int(np.abs(col_h).max())
        e.bias = bias.ptr
        if epi == EPI_QKV:
            T, H, Dh = 197, N // 3 // 64, 64
            e.group_cols, e.tokens, e.heads, e.hdim = N // 3, T, H, Dh
            bufs = [DeviceArray((M // T * H * T, Dh), np.int8) for _ in range(3)]
            for g in range(3):
                e.s_acc[g] = float(np.float32(1.7e-4 * (g + 1)))
                e.s_out[g], e.zp_out[g], e.out[g] = s_out[g], zp[g], bufs[g].ptr
        elif epi == EPI_RESID:
            e.group_cols = 1 << 30
            bufs = [DeviceArray((M, N), np.float32)]
            e.s_acc[0], e.out[0], e.resid = float(np.float32(3.1e-4)), bufs[0].ptr, resid.ptr
        else:
            e.group_cols = 1 << 30
            bufs = [DeviceArray((M, N), np.int8)]
            e.s_acc[0], e.s_out[0], e.zp_out[0], e.out[0] = float(np.float32(1.3e-4)), s_out[0], zp[0], bufs[0].ptr
            e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
        e.b_packed = 1 if "PACK" in var else 0
        _gemm(epi, a, packed if "PACK" in var else bt, 1, M, N, K, K, K, None, 0, 0, e)
        outs.append([b.to_host() for b in bufs])
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("epi_name,M,N,K", [("qkv", 3 * 197, 2304, 768), ("resid", 1000, 768, 3072),
                                           ("gelu", 1024 + 77, 3072, 768), ("resid", 77, 772, 192)])
def test_int4_packed_weights_equal_int8_path(epi_name, M, N, K, monkeypatch):
    """BASELINE configs[4]: bit width 4, weights nibble-packed (nqk_pack_b4) and unpacked
    in registers after the LDS stage; the outputs equal the int8-stored path bit for bit."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, EPI_QKV, EPI_RESID, _gemm, _pack_b
    epi = {"qkv": EPI_QKV, "resid": EPI_RESID, "gelu": EPI_GELU}[epi_name]
    rng = np.random.default_rng(M + N + K + 4)
    a = DeviceArray.from_host(rng.integers(-8, 8, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-8, 8, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col_h = bt_h.astype(np.int64).sum(axis=1)
    col = DeviceArray.from_host(col_h)
    bias = DeviceArray.from_host((0.05 * rng.standard_normal(N)).astype(np.float32))
    resid = DeviceArray.from_host(rng.standard_normal((M, N)).astype(np.float32))
    p4, kind = _pack_b(bt, 4)
    assert kind == 2
    outs = []
    for b_op, kind in ((bt, 0), (p4, 2)):
        e = _lib.Epilogue()
        e.zp_flags, e.bit_width, e.zpa, e.col, e.col_absmax = _lib.ZP_COL, 4, 3, col.ptr, int(np.abs(col_h).max())
        e.bias, e.b_packed = bias.ptr, kind
        if epi == EPI_QKV:
            T, H, Dh = 197, N // 3 // 64, 64
            e.group_cols, e.tokens, e.heads, e.hdim = N // 3, T, H, Dh
            bufs = [DeviceArray((M // T * H * T, Dh), np.int8) for _ in range(3)]
            for g in range(3):
                e.s_acc[g] = float(np.float32(3e-3 * (g + 1)))
                e.s_out[g], e.zp_out[g], e.out[g] = 0.07 * (g + 1), g - 1, bufs[g].ptr
        elif epi == EPI_RESID:
            e.group_cols = 1 << 30
            bufs = [DeviceArray((M, N), np.float32)]
            e.s_acc[0], e.out[0], e.resid = float(np.float32(3.1e-3)), bufs[0].ptr, resid.ptr
        else:
            e.group_cols = 1 << 30
            bufs = [DeviceArray((M, N), np.int8)]
            e.s_acc[0], e.s_out[0], e.zp_out[0], e.out[0] = float(np.float32(2e-3)), 0.11, -2, bufs[0].ptr
            e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
        _gemm(epi, a, b_op, 1, M, N, K, K, K, None, 0, 0, e)
        outs.append([b.to_host() for b in bufs])
    for x, y in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(x, y)


def _last_kernel():
    from numpy_quant import _lib
    return _lib.load().nqk_qgemm_last_kernel()


@pytest.mark.parametrize("epi_name,M,N,K,bw", [
    ("qkv", 256 * 197, 2304, 768, 8), ("qkv", 256 * 197, 2304, 768, 4),
    ("gelu", 128 * 50, 3072, 768, 8), ("gelu", 128 * 50, 3072, 768, 4), ("gelu", 512, 3072, 768, 8),
    ("resid", 128 * 200, 768, 768, 8), ("resid", 128 * 200, 768, 3072, 8), ("resid", 128 * 200, 768, 3072, 4),
    ("resid", 512, 768, 768, 8), ("qkv", 512 * 197, 2304, 768, 8),
    # ragged last tile rows (the half-batch streams of B = 256: M = 128 x 197)
    ("qkv", 128 * 197, 2304, 768, 8), ("qkv", 128 * 197, 2304, 768, 4), ("gelu", 128 * 197, 3072, 768, 8),
    ("gelu", 300, 3072, 768, 4),
])
def test_persistent_projection_gemm_equals_big_tile(epi_name, M, N, K, bw, monkeypatch):
    """The persistent projection GEMM (k_proj: 256 x 256 tiles, the next tile's first
    stages in flight during the epilogue, stores straight from the MFMA layout, residual /
    column constants by LDS-DMA) against the one-tile-per-workgroup kernel (k_qgemm_big) on the same packed weights:
    bit-identical for every epilogue, int8 and nibble-packed int4 weights, with many
    tiles per workgroup (M up to 100 864 rows) and with one, ragged last tile rows; small output scales put many
    values next to rounding boundaries (the filters' exact fallbacks run)."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_GELU, EPI_QKV, EPI_RESID, _gemm, _pack_b
    epi = {"qkv": EPI_QKV, "resid": EPI_RESID, "gelu": EPI_GELU}[epi_name]
    rng = np.random.default_rng(M + N + K + bw)
    lim = 128 if bw == 8 else 8
    a = DeviceArray.from_host(rng.integers(-lim, lim, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-24 if bw == 8 else -8, 25 if bw == 8 else 8, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col_h = bt_h.astype(np.int64).sum(axis=1)
    col = DeviceArray.from_host(col_h)
    bias = DeviceArray.from_host((0.05 * rng.standard_normal(N)).astype(np.float32))
    resid = DeviceArray.from_host(rng.standard_normal((M, N)).astype(np.float32))
    packed, kind = _pack_b(bt, bw)
    colterm = DeviceArray.from_host((col_h * -5).astype(np.int32))
    variants = [{"NQK_NO_PROJ": "1"}, {}]
    if epi == EPI_RESID:  # opt-in for the residual epilogues
        variants = [{"NQK_NO_PROJ": "1"}, {"NQK_PROJ_RESID": "1"}, {"NQK_PROJ_RESID": "1", "NQK_NO_F32X": "1"}]
    elif epi == EPI_GELU:  # opt-in
        variants = [{"NQK_NO_PROJ": "1"}, {"NQK_PROJ_GELU": "1"}]
    outs, kernels = [], []
    sa = 1.3e-4 if bw == 8 else 4e-3
    for var in variants:
        for k in ("NQK_NO_PROJ", "NQK_NO_F32X", "NQK_PROJ_RESID", "NQK_PROJ_GELU"):
            monkeypatch.delenv(k, raising=False)
        for k, v in var.items():
            monkeypatch.setenv(k, v)
        e = _lib.Epilogue()
        e.zp_flags, e.bit_width = _lib.ZP_COL, bw
        e.zpa, e.col, e.col_absmax = -5, col.ptr, int(np.abs(col_h).max())
        e.bias, e.b_packed, e.colterm = bias.ptr, kind, colterm.ptr
        if epi == EPI_QKV:
            T, H, Dh = 197, N // 3 // 64, 64
            e.group_cols, e.tokens, e.heads, e.hdim = N // 3, T, H, Dh
            bufs = [DeviceArray((M // T * H * T, Dh), np.int8) for _ in range(3)]
            for g in range(3):
                e.s_acc[g] = float(np.float32(sa * (g + 1)))
                e.s_out[g], e.zp_out[g], e.out[g] = (0.0021, 0.0173, 0.05)[g], (3, -140, 0)[g], bufs[g].ptr
        elif epi == EPI_RESID:
            e.group_cols = 1 << 30
            bufs = [DeviceArray((M, N), np.float32)]
            e.s_acc[0], e.out[0], e.resid = float(np.float32(sa * 2)), bufs[0].ptr, resid.ptr
        else:
            e.group_cols = 1 << 30
            bufs = [DeviceArray((M, N), np.int8)]
            e.s_acc[0], e.s_out[0], e.zp_out[0], e.out[0] = float(np.float32(sa)), 0.0027, -9, bufs[0].ptr
            e.div, e.add1, e.mul2 = float(np.float32(1.4142135381698608)), 1.0, 0.5
        _gemm(epi, a, packed, 1, M, N, K, K, K, None, 0, 0, e)
        kernels.append(_last_kernel())
        outs.append([b.to_host() for b in bufs])
    assert kernels[0] == 1 and all(k == 3 for k in kernels[1:]), kernels
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("M,K", [(128 * 197, 192), (128 * 197, 768), (1000, 192), (131, 768), (256 * 197, 768)])
@pytest.mark.parametrize("bw,zp,f64q", [(8, -5, False), (8, 140, False), (4, 2, False), (8, 3, True)])
def test_resid_epilogue_fused_layernorm_equals_ln_quant(M, K, bw, zp, f64q, monkeypatch):
    _fused_ln_case(M, K, bw, zp, f64q, monkeypatch, wbits=8)


@pytest.mark.parametrize("M,K", [(128 * 197, 192), (1000, 768)])
def test_resid_epilogue_fused_layernorm_int4_weights(M, K, monkeypatch):
    """The same with nibble-packed int4 weights (k_qgemm_big<RESID, B4, LN>)."""
    _fused_ln_case(M, K, 4, 1, False, monkeypatch, wbits=4)


def _fused_ln_case(M, K, bw, zp, f64q, monkeypatch, wbits):
    """Round 6: the residual GEMM's epilogue with the consumer LayerNorm fused
    (nqk_epilogue.ln_out, k_qgemm_big<RESID, LN>, N = 192: ViT-Ti's out-projection K = 192 and FFN-down
    K = 768) writes the same f32 rows as without it, and its int8 LayerNorm output equals nqk_ln_quant
    run on those rows, bit for bit (ragged last tiles; the magic-number and the f64 quantize)."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_RESID, _gemm, _pack_b
    if f64q:
        monkeypatch.setenv("NQK_LN_F64Q", "1")
    else:
        monkeypatch.delenv("NQK_LN_F64Q", raising=False)
    N = 192
    rng = np.random.default_rng(M + K + bw + zp)
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-30, 31, size=(N, K), dtype=np.int8) if wbits == 8 else rng.integers(-8, 8, size=(N, K), dtype=np.int8)
    bt = DeviceArray.from_host(bt_h)
    col_h = bt_h.astype(np.int64).sum(axis=1)
    col = DeviceArray.from_host(col_h)
    bias = DeviceArray.from_host((0.05 * rng.standard_normal(N)).astype(np.float32))
    resid = DeviceArray.from_host((rng.standard_normal((M, N)) * 1.5).astype(np.float32))
    g = DeviceArray.from_host((1 + 0.1 * rng.standard_normal(N)).astype(np.float32))
    b = DeviceArray.from_host((0.1 * rng.standard_normal(N)).astype(np.float32))
    eps, s_ln = float(np.float32(1e-12)), float(np.float32(0.021 if bw == 8 else 0.4))
    bp = _pack_b(bt, wbits)
    assert bp is not None and bp[1] == (2 if wbits == 4 else 1)
    outs = []
    for fuse in (False, True):
        e = _lib.Epilogue()
        e.zp_flags, e.bit_width, e.zpa, e.col, e.col_absmax = _lib.ZP_COL, bw, 7, col.ptr, int(np.abs(col_h).max())
        e.bias, e.group_cols = bias.ptr, 1 << 30
        e.b_packed = 0 if bp is None else bp[1]
        y = DeviceArray((M, N), np.float32)
        e.s_acc[0], e.out[0], e.resid = float(np.float32(2.3e-4)), y.ptr, resid.ptr
        lnq = DeviceArray((M, N), np.int8)
        if fuse:
            e.ln_gamma, e.ln_beta, e.ln_out, e.ln_eps, e.ln_scale, e.ln_zp = g.ptr, b.ptr, lnq.ptr, eps, s_ln, zp
        _gemm(EPI_RESID, a, bt if bp is None else bp[0], 1, M, N, K, K, K, None, 0, 0, e)
        if fuse:
            assert _last_kernel() == 1  # the one-tile-per-workgroup kernel
        else:
            _lib.call("nqk_ln_quant", y.vp, g.vp, b.vp, lnq.vp, M, N, eps, s_ln, zp, bw)
        outs.append((y.to_host(), lnq.to_host()))
    np.testing.assert_array_equal(outs[1][0], outs[0][0], err_msg="f32 residual rows")
    np.testing.assert_array_equal(outs[1][1], outs[0][1], err_msg="fused LayerNorm vs nqk_ln_quant")


def test_resid_fused_layernorm_refuses_other_widths():
    """A fused LayerNorm at a width other than 192 fails loudly (no silent unfused path)."""
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_RESID, _gemm
    M, N, K = 256, 768, 768
    rng = np.random.default_rng(5)
    a = DeviceArray.from_host(rng.integers(-128, 128, size=(M, K), dtype=np.int8))
    bt_h = rng.integers(-30, 31, size=(N, K), dtype=np.int8)
    bt, col = DeviceArray.from_host(bt_h), DeviceArray.from_host(bt_h.astype(np.int64).sum(axis=1))
    y, resid, lnq = DeviceArray((M, N), np.float32), DeviceArray((M, N), np.float32), DeviceArray((M, N), np.int8)
    gb = DeviceArray.from_host(np.ones(N, np.float32))
    e = _lib.Epilogue()
    e.zp_flags, e.bit_width, e.zpa, e.col, e.group_cols = _lib.ZP_COL, 8, 1, col.ptr, 1 << 30
    e.s_acc[0], e.out[0], e.resid = 1e-3, y.ptr, resid.ptr
    e.ln_gamma, e.ln_beta, e.ln_out, e.ln_eps, e.ln_scale, e.ln_zp = gb.ptr, gb.ptr, lnq.ptr, 1e-12, 0.02, 0
    with pytest.raises(_lib.NQKError, match="fused LayerNorm"):
        _gemm(EPI_RESID, a, bt, 1, M, N, K, K, K, None, 0, 0, e)
