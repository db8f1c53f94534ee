"""GPU parity of the one-kernel attention (nqk_attention_fused) with the three-launch
chain it replaces (nqk_qgemm_fused SCORES -> nqk_softmax_quant -> nqk_qgemm_fused PV),
which tests/test_gpu_plan.py pins to the eager node loop and the reference.  The
chain is the QModel's MatMul(Q, K^T) -> Div -> Softmax -> MatMul(P, V) -> Transpose
-> Reshape -> quantize (model.py:486-565).  Integer outputs: bit-exact."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["k_attention", "k_attn16", "k_attn16_nw5"])
def attn_kernel(request, monkeypatch):
    """Every case on both T = 197 kernels: round 6's k_attn16 (16x16x64, four lanes per query row,
    NQK_ATTN16=1; four or five waves per workgroup, NQK_ATTN16_NW) and k_attention (other T take
    k_attention either way)."""
    monkeypatch.setenv("NQK_ATTN16", "0" if request.param == "k_attention" else "1")
    monkeypatch.setenv("NQK_ATTN16_NW", "5" if request.param == "k_attn16_nw5" else "4")
    return request.param


def _run_both(B, H, T, zq, zk, zp, zv, zc, bw=8, seed=0, s_p=1.0 / 255, s_qk=(0.031, 0.027)):
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.plan import EPI_PV, EPI_SCORES, _gemm
    rng = np.random.default_rng(seed)
    lo, hi = -(1 << (bw - 1)), (1 << (bw - 1)) - 1
    Dh, D = 64, H * 64
    q = rng.integers(lo, hi + 1, size=(B * H, T, Dh), dtype=np.int8)
    k = rng.integers(lo, hi + 1, size=(B * H, T, Dh), dtype=np.int8)
    v = rng.integers(lo, hi + 1, size=(B * H, T, Dh), dtype=np.int8)
    s_q, s_k, s_v = np.float32(s_qk[0]), np.float32(s_qk[1]), np.float32(0.043)
    s_p = np.float32(s_p)
    s_ctx = np.float32(0.017)
    div = 8.0
    dq, dk, dv = (DeviceArray.from_host(a.reshape(B * H * T, Dh)) for a in (q, k, v))
    # fused
    ctx_f = DeviceArray((B, T, D), np.int8)
    a = _lib.Attention()
    a.heads, a.tokens, a.hdim, a.ld_out, a.bit_width = H, T, Dh, D, bw
    a.zq, a.zk, a.s_qk, a.div = zq, zk, float(np.float32(s_q * s_k)), div
    a.s_p, a.zp_p, a.s_pv, a.zv = float(s_p), zp, float(np.float32(s_p * s_v)), zv
    a.s_ctx, a.zp_ctx = float(s_ctx), zc
    _lib.call("nqk_attention_fused", dq.vp, dk.vp, dv.vp, ctx_f.vp, B * H, ctypes.byref(a))
    # three launches
    Tp = (T + 15) // 16 * 16
    vt = DeviceArray((B * H, Dh, Tp), np.int8)
    s = DeviceArray((B * H, T, T), np.float32)
    p = DeviceArray((B * H, T, Tp), np.int8)
    ctx_u = DeviceArray((B, T, D), np.int8)
    _lib.call("nqk_transpose_pad_i8", dv.vp, vt.vp, None, B * H, T, Dh, Tp)
    e = _lib.Epilogue()
    e.bit_width, e.tokens, e.heads, e.hdim = bw, T, H, Dh
    e.group_cols = 1 << 30
    e.zp_flags = _lib.ZP_ROW | _lib.ZP_COL | _lib.ZP_KCONST
    e.zpa, e.zpb, e.kdim = zq, zk, Dh
    e.s_acc[0] = float(np.float32(s_q * s_k))
    e.out[0] = s.ptr
    e.div, e.add1, e.mul2 = div, 0.0, 1.0
    _gemm(EPI_SCORES, dq, dk, B * H, T, T, Dh, Dh, Dh, None, T * Dh, T * Dh, e)
    _lib.call("nqk_softmax_quant", s.vp, p.vp, None, B * H * T, T, Tp, float(s_p), zp, bw)
    e2 = _lib.Epilogue()
    e2.bit_width, e2.tokens, e2.heads, e2.hdim, e2.ld_out = bw, T, H, Dh, D
    e2.group_cols = 1 << 30
    e2.zp_flags = _lib.ZP_ROW | _lib.ZP_COL | _lib.ZP_KCONST
    e2.zpa, e2.zpb, e2.kdim = zp, zv, T
    e2.s_acc[0] = float(np.float32(s_p * s_v))
    e2.s_out[0], e2.zp_out[0], e2.out[0] = float(s_ctx), zc, ctx_u.ptr
    e2.div, e2.add1, e2.mul2 = 1.0, 0.0, 1.0
    _gemm(EPI_PV, p, vt, B * H, T, Dh, Tp, Tp, Tp, None, T * Tp, Dh * Tp, e2)
    return ctx_f.to_host(), ctx_u.to_host()


@pytest.mark.parametrize("T", [1, 7, 8, 31, 32, 33, 100, 128, 129, 160, 197, 224])
def test_attention_matches_three_launch_chain(T):
    f, u = _run_both(2, 3, T, zq=-5, zk=3, zp=-128, zv=2, zc=-7, seed=T)
    np.testing.assert_array_equal(f, u)


@pytest.mark.parametrize("zq,zk,zp,zv,zc,bw", [(0, 0, 0, 0, 0, 8), (-140, 131, -128, -138, 5, 8),
                                              (4096, -4096, 1024, -1024, 0, 8), (-9, 2, -8, 1, 3, 4)])
def test_attention_zero_points_and_bit_widths(zq, zk, zp, zv, zc, bw):
    f, u = _run_both(1, 12, 197, zq, zk, zp, zv, zc, bw=bw, seed=abs(zq) + bw)
    np.testing.assert_array_equal(f, u)


@pytest.mark.parametrize("s_p,zp,s_qk", [(8.051e-05, -142, (0.02, 0.0225)), (2.3e-4, -131, (0.011, 0.009)),
                                         (1.0 / 255, -128, (0.002, 0.003))])
def test_attention_calibrated_softmax_scales(s_p, zp, s_qk):
    """Parameters like the bench model's calibration (its last layer: s_p 8.05e-5, zp_p -142,
    scores within a few units): the P quantize clamps at the bottom (zp < -128), most P
    values are a few units, so the per-element filter margin decides nearly every element
    on the fast path; small scores keep every exp on the exponent-add path."""
    f, u = _run_both(4, 12, 197, zq=0, zk=-6, zp=zp, zv=-14, zc=-11, seed=int(zp) + 1000, s_p=s_p, s_qk=s_qk)
    np.testing.assert_array_equal(f, u)


def test_attention_vit_base_batch():
    """ViT-Base shape at a larger batch (every (image, head) workgroup)."""
    f, u = _run_both(16, 12, 197, zq=-3, zk=4, zp=-128, zv=-1, zc=2, seed=7)
    np.testing.assert_array_equal(f, u)


@pytest.mark.parametrize("s_p,zp,s_qk,zc", [(8.051e-05, -142, (0.02, 0.0225), -11), (1.0 / 255, -128, (0.031, 0.027), 2),
                                            (3e-3, -120, (0.05, 0.06), 0)])
def test_attn16_equals_k_attention(s_p, zp, s_qk, zc, monkeypatch):
    """k_attn16 against k_attention directly (both FAST, T = 197), many workgroups, peaked and flat
    softmaxes (the clamped and the clamp-free P paths), bit for bit."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("NQK_ATTN16", v)
        outs.append(_run_both(24, 12, 197, zq=2, zk=-6, zp=zp, zv=-14, zc=zc, seed=abs(int(zp)) + 77, s_p=s_p, s_qk=s_qk)[0])
    np.testing.assert_array_equal(outs[1], outs[0])


def test_attention_rejects_unsupported_shapes():
    from numpy_quant import _lib
    a = _lib.Attention()
    a.heads, a.tokens, a.hdim, a.ld_out, a.bit_width = 1, 225, 64, 64, 8
    with pytest.raises(_lib.NQKError):
        _lib.call("nqk_attention_fused", None, None, None, None, 1, ctypes.byref(a))
    a.tokens, a.hdim = 197, 32
    with pytest.raises(_lib.NQKError):
        _lib.call("nqk_attention_fused", None, None, None, None, 1, ctypes.byref(a))
