"""Fused device plan for QModel.__call__ (numpy_quant/model.py:486-565).

`compile_plan(qmodel)` pattern-matches the transformer encoder layers of the
graph (the ViT exports in models/vit/) and replaces each layer's ~40 nodes by
11 fused launches (nqk_ln_quant, nqk_qgemm_fused with QKV / SCORES / PV / RESID /
GELU epilogues, nqk_softmax_quant, row sums and an int8 transpose).  Every other
node runs through the eager node loop.  Each fused launch performs, per element,
the same dequantize -> float ops -> quantize sequence as the node loop, so the
layer output is bit-identical to the eager path (tests/test_gpu_plan.py); the
layer's intermediate values are not materialised (their `.data` stays None).

Matching is strict: any deviation in ops, attributes, wiring or constants leaves
the layer to the eager loop.
"""
from __future__ import annotations

import ctypes
import os
import math
from typing import Optional

import numpy as np

from . import _lib
from . import kernels as KM
from .device import DeviceArray
from .tensor import FTensor, QTensor

EPI_QKV, EPI_SCORES, EPI_PV, EPI_RESID, EPI_GELU = 0, 1, 2, 3, 4

_EPI_NAMES = {EPI_QKV: "qkv", EPI_SCORES: "scores", EPI_PV: "pv", EPI_RESID: "resid", EPI_GELU: "gelu"}

# module switches: the one-kernel attention (nqk_attention_fused) and the one-GEMM
# patch embedding (nqk_sgemm_embed) where they apply
FUSED_ATTENTION = True
FUSED_EMBED = True
LN_GATHER = True
SPLIT_STREAMS = True


Epilogue = _lib.Epilogue


class Streams:
    """Fork / join bookkeeping of Plan.run's HIP streams.

    A split step runs its images in `parts` consecutive parts (2 by default,
    NQK_STREAMS = 2..4), part i on stream i (nqk_set_stream); consecutive split steps
    use the same parts, so each stream only depends on its own earlier work and no
    event is needed between them.  Whole-batch work (eager nodes, a dequantized layer
    input, an unsplit layer) must first `join()` (stream 0 waits for the side streams);
    parts that follow whole-batch work on stream 0 must first `fork()` (the side
    streams wait for stream 0)."""

    def __init__(self, enabled: bool, parts: int = 2):
        self.enabled = enabled
        self.parts = max(1, min(4, int(parts)))
        self.forked = False

    def fork(self):
        if not self.forked:
            _lib.call("nqk_stream_fork")
            self.forked = True

    def join(self):
        if self.forked:
            _lib.call("nqk_stream_join")
            self.forked = False

    def max_part(self, n: int) -> int:
        """The most images one `halves` call hands fn (the first part's)."""
        p = min(self.parts, n)
        return n if (not self.enabled or p < 2) else -(-n // p)

    def halves(self, n: int, fn):
        """fn(stream_index, first_image, images) for the parts of n images on their
        streams (or once, whole batch on stream 0, when splitting is off / n < 2); the
        current stream is back to 0 afterwards, also when fn raises."""
        p = min(self.parts, n)
        if not self.enabled or p < 2:
            self.join()
            fn(0, 0, n)
            return
        self.fork()
        try:
            i0 = 0
            for s_idx in range(p):
                nb = n // p + (1 if s_idx < n % p else 0)
                _lib.call("nqk_set_stream", s_idx)
                fn(s_idx, i0, nb)
                i0 += nb
        finally:
            _lib.call("nqk_set_stream", 0)


_ONE_STREAM = Streams(False)


def _stream_lag():
    v = os.environ.get("NQK_STREAM_LAG", "")
    return v if v in ("ln1", "qkv", "attn") else None


_LAG_EVENTS = {}


def _lag_event(i):
    """The event part i records at its NQK_STREAM_LAG point (one per part, reused every layer:
    part i + 1 waits for it right after part i's layer is issued)."""
    if i not in _LAG_EVENTS:
        e = ctypes.c_void_p()
        _lib.call("nqk_event_create", ctypes.byref(e))
        _LAG_EVENTS[i] = e
    return _LAG_EVENTS[i]


def embed_q_fits(images: int, hw: int, kout: int) -> bool:
    """Whether one nqk_embed_q call over `images` images of hw patches takes the shape: at most
    65535 row tiles of 128 patches, and (images x (hw + 1)) x kout < 2^31 (its 32-bit output
    offsets; nqk_gemm.hip checks the same and refuses larger calls)."""
    return -(-(images * hw) // 128) <= 65535 and images * (hw + 1) * kout < 2147483647


class NoMatch(Exception):
    pass


def _f32(x) -> float:
    return float(np.float32(x))


def _zp(p) -> int:
    if p.zero_point is None:
        raise NoMatch("asymmetric parameters expected")
    return int(p.zero_point)


# ----------------------------------------------------------------------------- matching helpers
def _only(lst, what):
    if len(lst) != 1:
        raise NoMatch(f"{what}: expected one, got {len(lst)}")
    return lst[0]


def _consumer(value, op):
    n = _only(value.outputs, f"consumer of {value.name}")
    if n.op != op:
        raise NoMatch(f"{value.name} feeds {n.op}, expected {op}")
    return n


def _const_node_value(value):
    """Value produced by a Constant node (e.g. the Div by 8.0) -> (numpy array, node)."""
    if value.__class__.__name__ != "Variable" or len(value.inputs) != 1 or value.inputs[0].op != "Constant":
        raise NoMatch(f"{value.name} is not a Constant-node output")
    node = value.inputs[0]
    return node.attrs["value"], node


def _is_const(v):
    return v.__class__.__name__ == "Constant"


def _const_float(qmodel, v):
    """The float value of a LayerNorm parameter: a quantized Constant (dequantized as the
    node loop does), or an Identity of one (the ONNX exporter shares equal tensors that
    way, e.g. the encoder-layer graph's layernorm_after weights)."""
    while not _is_const(v):
        if v.__class__.__name__ != "Variable" or len(v.inputs) != 1 or v.inputs[0].op != "Identity":
            raise NoMatch(f"{v.name}: constant LayerNorm parameter expected")
        v = v.inputs[0].inputs[0]
    return qmodel._dequant_input(v)


def _matmul_weight(node):
    a, w = node.inputs
    if not _is_const(w) or _is_const(a):
        raise NoMatch("MatMul with a constant weight expected")
    return a, w


def _bias_add(mm_out):
    add = _consumer(mm_out, "Add")
    consts = [i for i in add.inputs if _is_const(i)]
    if len(consts) != 1:
        raise NoMatch("bias Add expected")
    return add, consts[0]


class LayerMatch:
    """Values / constants of one encoder layer (names as in the QModel)."""

    def __init__(self, qmodel, ln1):
        self.nodes = set()
        take = self.nodes.add
        take(ln1)
        self.ln1 = ln1
        self.x_in = ln1.inputs[0]
        if ln1.attrs.get("axis", -1) not in (-1, 2):
            raise NoMatch("LayerNorm axis")
        ln1_out = ln1.outputs[0]
        mms = ln1_out.outputs
        if len(mms) != 3 or any(m.op != "MatMul" for m in mms):
            raise NoMatch("LN1 must feed three MatMuls")
        roles = {}
        for mm in mms:
            take(mm)
            _, w = _matmul_weight(mm)
            add, bias = _bias_add(mm.outputs[0])
            take(add)
            rs = _consumer(add.outputs[0], "Reshape")
            take(rs)
            shp_val, shp_node = _const_node_value(rs.inputs[1])
            take(shp_node)
            tr = _consumer(rs.outputs[0], "Transpose")
            take(tr)
            perm = list(tr.attrs["perm"])
            nxt = _only(tr.outputs[0].outputs, "transpose consumer")
            if nxt.op != "MatMul":
                raise NoMatch("head transpose must feed a MatMul")
            idx = nxt.inputs.index(tr.outputs[0])
            if perm == [0, 2, 3, 1] and idx == 1:
                role = "k"
            elif perm == [0, 2, 1, 3] and idx == 0:
                role = "q"
            elif perm == [0, 2, 1, 3] and idx == 1:
                role = "v"
            else:
                raise NoMatch(f"unexpected head layout {perm}/{idx}")
            if role in roles:
                raise NoMatch("duplicate role")
            roles[role] = dict(mm=mm, w=w, bias=bias, shape=np.asarray(shp_val), tr_out=tr.outputs[0], user=nxt)
        if set(roles) != {"q", "k", "v"}:
            raise NoMatch("q/k/v roles")
        self.roles = roles
        scores = roles["q"]["user"]
        if roles["k"]["user"] is not scores:
            raise NoMatch("Q and K must meet in one MatMul")
        take(scores)
        div = _consumer(scores.outputs[0], "Div")
        take(div)
        dval, dnode = _const_node_value(div.inputs[1])
        if div.inputs[0] is not scores.outputs[0] or np.asarray(dval).size != 1:
            raise NoMatch("scores Div")
        take(dnode)
        self.div = _f32(np.asarray(dval).reshape(()))
        sm = _consumer(div.outputs[0], "Softmax")
        take(sm)
        if sm.attrs.get("axis") not in (-1, 3):
            raise NoMatch("softmax axis")
        pv = _consumer(sm.outputs[0], "MatMul")
        if pv is not roles["v"]["user"] or pv.inputs[0] is not sm.outputs[0]:
            raise NoMatch("PV MatMul wiring")
        take(pv)
        tr3 = _consumer(pv.outputs[0], "Transpose")
        take(tr3)
        if list(tr3.attrs["perm"]) != [0, 2, 1, 3]:
            raise NoMatch("context transpose")
        rs3 = _consumer(tr3.outputs[0], "Reshape")
        take(rs3)
        _, rs3c = _const_node_value(rs3.inputs[1])
        take(rs3c)
        dense = _consumer(rs3.outputs[0], "MatMul")
        take(dense)
        _, self.wo = _matmul_weight(dense)
        add_o, self.bo = _bias_add(dense.outputs[0])
        take(add_o)
        res1 = _consumer(add_o.outputs[0], "Add")
        take(res1)
        if self.x_in not in res1.inputs:
            raise NoMatch("attention residual")
        x1 = res1.outputs[0]
        users = x1.outputs
        if len(users) != 2:
            raise NoMatch("x1 must feed LN2 and the second residual")
        ln2 = next((u for u in users if u.op == "LayerNormalization"), None)
        res2_candidates = [u for u in users if u.op == "Add"]
        if ln2 is None or len(res2_candidates) != 1:
            raise NoMatch("LN2 / residual 2")
        take(ln2)
        self.ln2 = ln2
        up = _consumer(ln2.outputs[0], "MatMul")
        take(up)
        _, self.w1 = _matmul_weight(up)
        add_u, self.b1 = _bias_add(up.outputs[0])
        take(add_u)
        h = add_u.outputs[0]
        hu = h.outputs
        gdiv = next((u for u in hu if u.op == "Div"), None)
        gmul = next((u for u in hu if u.op == "Mul"), None)
        if len(hu) != 2 or gdiv is None or gmul is None or gdiv.inputs[0] is not h:
            raise NoMatch("GELU structure")
        take(gdiv)
        v, n = _const_node_value(gdiv.inputs[1])
        take(n)
        self.gelu_div = _f32(np.asarray(v).reshape(()))
        erf = _consumer(gdiv.outputs[0], "Erf")
        take(erf)
        gadd = _consumer(erf.outputs[0], "Add")
        take(gadd)
        other = [i for i in gadd.inputs if i is not erf.outputs[0]]
        v, n = _const_node_value(_only(other, "gelu +1 operand"))
        take(n)
        self.gelu_add = _f32(np.asarray(v).reshape(()))
        if gmul.inputs[0] is not h or gmul.inputs[1] is not gadd.outputs[0]:
            raise NoMatch("GELU Mul operand order")
        take(gmul)
        gmul2 = _consumer(gmul.outputs[0], "Mul")
        take(gmul2)
        if gmul2.inputs[0] is not gmul.outputs[0]:
            raise NoMatch("GELU Mul_1 operand order")
        v, n = _const_node_value(gmul2.inputs[1])
        take(n)
        self.gelu_mul = _f32(np.asarray(v).reshape(()))
        self.h_out = gmul2.outputs[0]
        down = _consumer(self.h_out, "MatMul")
        take(down)
        _, self.w2 = _matmul_weight(down)
        add_d, self.b2 = _bias_add(down.outputs[0])
        take(add_d)
        res2 = _consumer(add_d.outputs[0], "Add")
        if res2 is not res2_candidates[0] or x1 not in res2.inputs:
            raise NoMatch("FFN residual")
        take(res2)
        self.x_out = res2.outputs[0]
        self.ln1_out, self.ln2_out = ln1_out, ln2.outputs[0]
        self.sm_out, self.rs3_out = sm.outputs[0], rs3.outputs[0]
        # every intermediate value must be private to the layer
        for node in self.nodes:
            for o in node.outputs:
                if o is self.x_out:
                    continue
                for u in o.outputs:
                    if u not in self.nodes:
                        raise NoMatch(f"{o.name} escapes the layer")
        shp = roles["q"]["shape"]
        if shp.size != 4 or any((roles[r]["shape"][1:] != shp[1:]).any() for r in "kv"):
            raise NoMatch("head reshape")
        self.tokens, self.heads, self.hdim = int(shp[1]), int(shp[2]), int(shp[3])


# ----------------------------------------------------------------------------- patch embedding
def _const_ints(value):
    arr, _ = _const_node_value(value)
    return np.asarray(arr).reshape(-1).astype(np.int64)


class EmbedMatch:
    """ViT patch embedding (models/vit graphs):
        Conv(x, W, b)  -> Reshape(., Concat(Slice(Shape(.), [0], [2], [0]), [-1]))
        -> Transpose([0, 2, 1]) -> Concat([Expand(cls, .), .], axis=1) -> Add(., pos)
    computed by one im2col GEMM with a fused epilogue (nqk_sgemm_embed).  The Conv
    output is never materialised: its Shape consumer sees a shape-only placeholder."""

    def __init__(self, qmodel, conv):
        self.nodes = set()
        take = self.nodes.add
        if conv.op != "Conv" or len(conv.inputs) != 3:
            raise NoMatch("Conv with bias expected")
        x, w, b = conv.inputs
        if _is_const(x) or not (_is_const(w) and _is_const(b)):
            raise NoMatch("Conv(x, const W, const b) expected")
        a = conv.attrs
        kh, kw = (int(v) for v in a.get("kernel_shape", w.data.dev.shape[2:]))
        if list(a.get("strides", [1, 1])) != [kh, kw] or any(int(p) for p in a.get("pads", [0, 0, 0, 0])):
            raise NoMatch("patchify Conv (stride = kernel, no padding) expected")
        if any(int(d) != 1 for d in a.get("dilations", [1, 1])) or int(a.get("group", 1)) != 1:
            raise NoMatch("plain Conv expected")
        take(conv)
        self.conv, self.x, self.w, self.b = conv, x, w, b
        self.kh, self.kw = kh, kw
        cout = conv.outputs[0]
        users = cout.outputs
        rs = [u for u in users if u.op == "Reshape"]
        shp = [u for u in users if u.op == "Shape"]
        if len(rs) != 1 or len(rs) + len(shp) != len(users):
            raise NoMatch("Conv output must feed one Reshape (+ Shape)")
        rs = rs[0]
        take(rs)
        # reshape target = Concat(Slice(Shape(conv), [0], [2], [0]), [-1])  ->  [B, C, H*W]
        cat = rs.inputs[1].inputs[0] if rs.inputs[1].inputs else None
        if cat is None or cat.op != "Concat" or len(cat.inputs) != 2:
            raise NoMatch("reshape target")
        sl = cat.inputs[0].inputs[0] if cat.inputs[0].inputs else None
        if sl is None or sl.op != "Slice" or sl.inputs[0].inputs[0].op != "Shape" or \
                sl.inputs[0].inputs[0].inputs[0] is not cout:
            raise NoMatch("reshape target slice")
        if list(_const_ints(sl.inputs[1])) != [0] or list(_const_ints(sl.inputs[2])) != [2] or \
                list(_const_ints(sl.inputs[3])) != [0] or list(_const_ints(cat.inputs[1])) != [-1]:
            raise NoMatch("reshape target values")
        tr = _consumer(rs.outputs[0], "Transpose")
        if list(tr.attrs["perm"]) != [0, 2, 1]:
            raise NoMatch("patch transpose")
        take(tr)
        cc = _consumer(tr.outputs[0], "Concat")
        if cc.attrs.get("axis") != 1 or len(cc.inputs) != 2 or cc.inputs[1] is not tr.outputs[0]:
            raise NoMatch("class-token concat")
        take(cc)
        ex = cc.inputs[0].inputs[0] if cc.inputs[0].inputs else None
        if ex is None or ex.op != "Expand" or not _is_const(ex.inputs[0]) or len(cc.inputs[0].outputs) != 1:
            raise NoMatch("class-token expand")
        take(ex)
        self.expand, self.cls = ex, ex.inputs[0]
        add = _consumer(cc.outputs[0], "Add")
        others = [i for i in add.inputs if i is not cc.outputs[0]]
        if len(others) != 1 or not _is_const(others[0]) or add.inputs[0] is not cc.outputs[0]:
            raise NoMatch("position-embedding add")
        take(add)
        self.pos, self.add, self.conv_out = others[0], add, cout
        for node in self.nodes:
            for o in node.outputs:
                if o is add.outputs[0] or o is cout:
                    continue
                for u in o.outputs:
                    if u not in self.nodes:
                        raise NoMatch(f"{o.name} escapes the embedding")


class _ShapeOnly:
    """Stand-in value for a tensor that is never materialised: only its shape is read
    (ONNX Shape node, model.py Shape -> x.shape)."""

    def __init__(self, shape):
        self._shape = tuple(int(s) for s in shape)

    @property
    def shape(self):
        from .tensor import ITensor
        return ITensor(np.array(self._shape, dtype=np.int64))


def embed_weight_image(W: DeviceArray, kout: int, kk: int) -> DeviceArray:
    """The Conv weight [kout][c][16][16] as nqk_embed_q's [kout][K] image: K in (ki, kj, ci) order,
    each 16-k block permuted to the kernel's order (nqk_embed_weight_order, include/nqk.h)."""
    from .device import permute
    order = _lib.load().nqk_embed_weight_order()
    if order == 16:
        wt = permute(W, [0, 2, 3, 1]).reshape((kout, kk // 16, 4, 4))
    else:
        wt = permute(W, [0, 2, 3, 1]).reshape((kout, kk // 16, 8, 2))
    return permute(wt, [0, 1, 3, 2]).reshape((kout, kk))


class FusedEmbed:
    def __init__(self, qmodel, m: EmbedMatch):
        self.m = m
        deq = qmodel._dequant_input
        W = deq(m.w).dev
        self.kout, cin = W.shape[0], W.shape[1]
        self.kk = m.kh * m.kw * cin
        from .device import permute
        # weight matrix [(kh, kw, c), kout] as fconv2d builds it (tensor.py)
        self.wm = permute(W, [2, 3, 1, 0]).reshape((self.kk, self.kout))
        self.bias = deq(m.b).dev
        self.cls = deq(m.cls).dev
        self.posv = deq(m.pos).dev
        if self.kk % 2 or self.bias.size != self.kout or self.cls.size != self.kout:
            raise NoMatch("embedding dimensions")
        self._cols = None
        # nqk_embed_q (no im2col matrix): 3-channel 16 x 16 patches, N % 64 == 0; the
        # weights as [N][K] in (ki, kj, ci) order, each 16-block of k permuted to the kernel's
        # LDS order (nqk_embed_weight_order): p = (k & 1) * 8 + (k >> 1) for the 32x32x2 kernel,
        # p = (k & 3) * 4 + (k >> 2) for the 16x16x4 one
        self.wt = None
        if (cin == 3 and m.kh == 16 and m.kw == 16 and self.kout % 64 == 0 and os.environ.get("NQK_EMBED_Q", "1") != "0"):
            self.wt = embed_weight_image(W, self.kout, self.kk)

    def pre(self, qmodel):
        """at the Conv's position: the shape-only placeholder for the Shape consumer"""
        m = self.m
        n, c, h, w = m.x.data.dev.shape
        m.conv_out.data = _ShapeOnly((n, self.kout, h // m.kh, w // m.kw))

    def run(self, qmodel, streams: Streams = _ONE_STREAM):
        """The embedding of every image; with splitting on, in two halves, one per
        stream (as FusedLayer.run)."""
        m = self.m
        xd = m.x.data
        n, c, h, w = xd.dev.shape
        ho, wo = h // m.kh, w // m.kw
        hw = ho * wo
        zp = xd.zero_point
        fused_in = (isinstance(xd, QTensor) and xd._bias is None and xd.dev.dtype == np.int8 and h % m.kh == 0 and
                    w % m.kw == 0 and (zp is None or (np.ndim(zp) == 0 and abs(int(zp)) <= 1 << 20)))
        if self.posv.size != (hw + 1) * self.kout:
            raise ValueError("position embedding does not match the patch grid")
        eshape = np.asarray(m.expand.inputs[1].data.data).reshape(-1)
        if eshape.size != 3 or int(eshape[0]) != n:
            raise ValueError(f"class-token Expand shape {eshape} does not match the batch {n}")
        out = DeviceArray((n, hw + 1, self.kout), np.float32)
        # (fused_in: the zero point within nqk_patchify_dequant's / nqk_embed_q's 2^20;
        # nqk_embed_q, per call (one per stream part): at most 65535 row tiles of 128 patches and
        # (images x (patches + 1)) x kout < 2^31 (its 32-bit output offsets), else the patchify path)
        folded = fused_in and self.wt is not None and c == 3 and embed_q_fits(streams.max_part(n), hw, self.kout)
        if folded:
            cols = None  # nqk_embed_q reads the int8 image itself
        elif fused_in:
            # dequantize fused into the patch gather (the QTensor is read once, as int8); the
            # patch matrix stays with the step (two streams: see FusedLayer.run)
            if self._cols is None or self._cols.shape != (n * hw, self.kk):
                self._cols = DeviceArray((n * hw, self.kk), np.float32)
            cols = self._cols
        else:
            streams.join()  # whole-batch dequantize / im2col on stream 0
            x = qmodel._dequant_input(m.x) if isinstance(xd, QTensor) else xd
            cols, ho, wo = KM.im2col(x.dev, m.kh, m.kw, (0, 0, 0, 0), (m.kh, m.kw))
            streams = _ONE_STREAM
        t0 = KM.TIMER.begin() if KM.TIMER is not None else None

        if folded:
            def part(s_idx, i0, nb):
                qv = xd.dev.offset_view(i0 * c * h * w, (nb, c, h, w))
                ov = out.offset_view(i0 * (hw + 1) * self.kout, (nb, hw + 1, self.kout))
                _lib.call("nqk_embed_q", qv.vp, float(np.float32(xd.scale)), int(zp) if zp is not None else 0,
                          self.wt.vp, self.bias.vp, self.cls.vp, self.posv.vp, ov.vp, nb, c, h, w, m.kh, m.kw,
                          self.kout)

            if os.environ.get("NQK_EMBED_WHOLE") and embed_q_fits(n, hw, self.kout):
                # A/B variant (round 6): one whole-batch launch on stream 0; the next split step forks
                streams.join()
                part(0, 0, n)
            else:
                streams.halves(n, part)
            if t0 is not None:
                KM.TIMER.end("embed_sgemm", t0, (2 * n * hw * self.kk * self.kout,
                                                 n * c * h * w + 4 * (self.kk * self.kout + n * (hw + 1) * self.kout)),
                             unit="flop32")
            m.add.outputs[0].data = FTensor(out)
            m.conv_out.data = FusedAway(m.conv_out.name)
            return

        def part(s_idx, i0, nb):
            cp = cols.offset_view(i0 * hw * self.kk, (nb * hw, self.kk))
            if fused_in:
                qv = xd.dev.offset_view(i0 * c * h * w, (nb, c, h, w))
                _lib.call("nqk_patchify_dequant", qv.vp, cp.vp, nb, c, h, w, m.kh, m.kw,
                          float(np.float32(xd.scale)), int(zp) if zp is not None else 0)
            ov = out.offset_view(i0 * (hw + 1) * self.kout, (nb, hw + 1, self.kout))
            _lib.call("nqk_sgemm_embed", cp.vp, self.wm.vp, self.bias.vp, self.cls.vp, self.posv.vp, ov.vp,
                      nb, hw, self.kout, self.kk)

        streams.halves(n, part)
        if t0 is not None:
            KM.TIMER.end("embed_sgemm", t0, (2 * n * hw * self.kk * self.kout,
                                             4 * (n * hw * self.kk + self.kk * self.kout + n * (hw + 1) * self.kout)),
                         unit="flop32")
        m.add.outputs[0].data = FTensor(out)
        m.conv_out.data = FusedAway(m.conv_out.name)


# ----------------------------------------------------------------------------- Gather after LN
class LnGather:
    """LayerNormalization (last axis) whose only consumer is a Gather along another axis
    with constant indices (the ViT classifier reads the CLS token only): LayerNorm
    normalises every row on its own, so Gather-then-LN equals LN-then-Gather bit for bit
    and only the gathered rows are normalised.  The LN output is not materialised."""

    def __init__(self, qmodel, ln):
        if ln.op != "LayerNormalization":
            raise NoMatch("LayerNormalization expected")
        out = ln.outputs[0]
        g = _only(out.outputs, "LN consumer")
        if g.op != "Gather" or g.inputs[0] is not out:
            raise NoMatch("Gather consumer expected")
        idx = g.inputs[1]
        if not (idx.inputs and idx.inputs[0].op == "Constant"):
            raise NoMatch("constant Gather indices expected")
        ax = int(ln.attrs.get("axis", -1))
        gax = int(g.attrs.get("axis", 0))
        if ax != -1 or gax in (-1,):
            raise NoMatch("LN over the last axis, Gather over another one")
        self.ln, self.g, self.nodes = ln, g, {ln, g}

    def run(self, qmodel, times=None, profile=False):
        from .model import onnx_operator_implementation
        x = self.ln.inputs[0].data
        if not isinstance(x, FTensor) or int(self.g.attrs.get("axis", 0)) % x.dev.ndim == x.dev.ndim - 1:
            raise ValueError("LN/Gather pushdown needs a float input gathered off the last axis")
        xs = x.take(self.g.inputs[1].data, axis=int(self.g.attrs.get("axis", 0)))
        args = [xs] + [qmodel._dequant_input(v) if isinstance(v.data, QTensor) else v.data for v in self.ln.inputs[1:]]
        self.g.outputs[0].data = onnx_operator_implementation("LayerNormalization", args, self.ln.attrs)[0]
        self.ln.outputs[0].data = FusedAway(self.ln.outputs[0].name)


# ----------------------------------------------------------------------------- fused layer
class FusedLayer:
    def __init__(self, qmodel, m: LayerMatch):
        self.m = m
        self.bw = qmodel.bit_width
        qp = qmodel.quant_params
        deq = qmodel._dequant_input
        cf = lambda v: _const_float(qmodel, v)  # noqa: E731
        self.g1, self.be1 = cf(m.ln1.inputs[1]).dev, cf(m.ln1.inputs[2]).dev
        self.g2, self.be2 = cf(m.ln2.inputs[1]).dev, cf(m.ln2.inputs[2]).dev
        self.eps1 = _f32(m.ln1.attrs.get("epsilon", 1e-5))
        self.eps2 = _f32(m.ln2.attrs.get("epsilon", 1e-5))
        self.p_ln1, self.p_ln2 = qp[m.ln1_out.name], qp[m.ln2_out.name]
        self.p_sm, self.p_ctx, self.p_h = qp[m.sm_out.name], qp[m.rs3_out.name], qp[m.h_out.name]
        self.p_head = {r: qp[m.roles[r]["tr_out"].name] for r in "qkv"}
        # weights: pre-transposed int8 Bt, column sums, dequantized biases
        bts, cols, biases, self.s_w = [], [], [], {}
        for r in "qkv":
            w = m.roles[r]["w"].data
            bt, col = w.weight_operand()
            bts.append(bt)
            cols.append(col)
            biases.append(deq(m.roles[r]["bias"]).dev)
            self.s_w[r] = w.scale
        self.D = bts[0].shape[1]
        if any(b.shape[1] != self.D or b.dtype != np.int8 for b in bts):
            raise NoMatch("int8 weights with a common K expected")
        self.bt_qkv = _cat0(bts)
        self.col_qkv = _cat0(cols)
        self.bias_qkv = _cat0(biases)
        self.bt_o, self.col_o = m.wo.data.weight_operand()
        self.bt_1, self.col_1 = m.w1.data.weight_operand()
        self.bt_2, self.col_2 = m.w2.data.weight_operand()
        self.s_wo, self.s_w1, self.s_w2 = m.wo.data.scale, m.w1.data.scale, m.w2.data.scale
        self.bias_o, self.bias_1, self.bias_2 = deq(m.bo).dev, deq(m.b1).dev, deq(m.b2).dev
        self.F = self.bt_1.shape[0]
        # tile-packed weight images (whole 128-B lines per LDS-DMA piece), when the big-tile
        # GEMM takes the shape
        self.bp = {k: _pack_b(b, self.bw) for k, b in (("qkv", self.bt_qkv), ("o", self.bt_o), ("1", self.bt_1),
                                                        ("2", self.bt_2))}
        # the persistent 16x16x64 GEMM's weight images (nqk_pack_pg; used where it takes the case)
        # (int4 weights: the nibble image, paired with the big-tile GEMM's nibble pack: b_packed 2)
        self.bpg = {k: _pack_pg(b, self.bw, lay, nibbles=self.bp[k] is not None and self.bp[k][1] == 2)
                    for k, b, lay in (("qkv", self.bt_qkv, 0), ("o", self.bt_o, 1), ("1", self.bt_1, 0),
                                      ("2", self.bt_2, 1))}
        # max |column sum| of each weight: lets the GEMM epilogues prove f32 exactness
        self.cmax = {k: _absmax(c) for k, c in (("qkv", self.col_qkv), ("o", self.col_o), ("1", self.col_1),
                                                 ("2", self.col_2))}
        # max column L1 norm of each weight: a tighter |acc| bound for the same proof (FFN-down,
        # K = 3072, then dequantizes in f32 too)
        self.l1max = {k: _l1max(b) for k, b in (("qkv", self.bt_qkv), ("o", self.bt_o), ("1", self.bt_1),
                                                 ("2", self.bt_2))}
        # int32 zero-point column terms col * zp_a of each GEMM (the persistent GEMM's
        # per-column constant; None where they do not fit int32)
        self.ct = {k: _colterm(c, _zp(p)) for k, c, p in (("qkv", self.col_qkv, self.p_ln1), ("o", self.col_o, self.p_ctx),
                                                          ("1", self.col_1, self.p_ln2), ("2", self.col_2, self.p_h))}
        if self.D != m.heads * m.hdim or self.bt_o.shape != (self.D, self.D) or self.bt_2.shape != (self.D, self.F):
            raise NoMatch("layer dimensions")
        # the FFN-up epilogue's GELU chain + quantize as a table of its output bytes (built and
        # checked on all finite f32 inputs by nqk_gelu_lut_build; None: the filtered chain)
        self.glut = _gelu_lut(self.p_h, self.bw, m.gelu_div, m.gelu_add, m.gelu_mul)
        # the one-kernel attention covers head size 64, <= 224 tokens and zero points for
        # which every int32 intermediate is exact (nqk.h); otherwise three launches
        zs = [_zp(self.p_head["q"]), _zp(self.p_head["k"]), _zp(self.p_sm), _zp(self.p_head["v"])]
        self.attn_fused = (FUSED_ATTENTION and m.hdim == 64 and 1 <= m.tokens <= 224 and
                           abs(zs[0]) <= 4096 and abs(zs[1]) <= 4096 and abs(zs[2]) <= 1024 and abs(zs[3]) <= 1024)
        # round 6: at width 192 (ViT-Ti) a residual GEMM tile holds whole rows, so the LayerNorm that
        # reads its output (LN2 after the out-projection; the NEXT layer's LN1 after FFN-down, linked
        # by the Plan) runs inside its epilogue (nqk_epilogue.ln_out): 24 LayerNorm launches and their
        # f32 row reads fewer per forward.  NQK_NO_LNFUSE=1 keeps the separate launches.
        self.ln_fuse = self.D == 192 and not os.environ.get("NQK_NO_LNFUSE")
        self.next_ln = None        # the next fused layer, whose LN1 this layer's FFN-down computes
        self.ln1_by_prev = False   # this layer's LN1 is computed by the previous layer's FFN-down

    def _epi(self, **kw) -> Epilogue:
        e = Epilogue()
        e.bit_width = self.bw
        e.group_cols = kw.pop("group_cols", 1 << 30)
        e.tokens, e.heads, e.hdim = self.m.tokens, self.m.heads, self.m.hdim
        e.div, e.add1, e.mul2 = kw.pop("div", 1.0), kw.pop("add1", 0.0), kw.pop("mul2", 1.0)
        for k, v in kw.items():
            if k in ("s_acc", "s_out", "zp_out", "out"):
                arr = getattr(e, k)
                for i, x in enumerate(v):
                    arr[i] = x
            else:
                setattr(e, k, v)
        return e

    @staticmethod
    def _ln_into(e, g, b, eps, p, out):
        """Fuse the LayerNorm (gamma g, beta b, epsilon eps) of the residual epilogue's output rows,
        quantized with p, into e (nqk_epilogue.ln_*): out gets what nqk_ln_quant would write."""
        e.ln_gamma, e.ln_beta, e.ln_out = g.ptr, b.ptr, out.ptr
        e.ln_eps, e.ln_scale, e.ln_zp = eps, _f32(p.scale), _zp(p)

    def _b(self, e, key, bt):
        """The B operand of a projection GEMM: its packed image if there is one (and the
        nqk_pack_pg image in e.bt_pg)."""
        bp = self.bp[key]
        e.b_packed = 0 if bp is None else bp[1]
        pg = self.bpg[key]
        e.bt_pg = None if pg is None else pg.ptr
        return bt if bp is None else bp[0]

    def _attention_unfused(self, w, B, T, Tp, H, Dh, D):
        """Scores GEMM, softmax and PV GEMM as three launches (any T / head size)."""
        m, bw, call = self.m, self.bw, _lib.call
        pq, pk, pv_ = self.p_head["q"], self.p_head["k"], self.p_head["v"]
        # V -> V^T (the PV GEMM's Bt operand), zero padded to Tp tokens
        call("nqk_transpose_pad_i8", w["v"].vp, w["vt"].vp, None, B * H, T, Dh, Tp)
        # scores = dequant(Q K^T) / div
        e = self._epi(zp_flags=_lib.ZP_ROW | _lib.ZP_COL | _lib.ZP_KCONST, zpa=_zp(pq), zpb=_zp(pk), kdim=Dh,
                      s_acc=[_f32(np.float32(pq.scale) * np.float32(pk.scale))], out=[w["s"].ptr], div=m.div)
        _gemm(EPI_SCORES, w["q"], w["k"], B * H, T, T, Dh, Dh, Dh, None, T * Dh, T * Dh, e)
        # softmax + quantize
        call("nqk_softmax_quant", w["s"].vp, w["p"].vp, None, B * H * T, T, Tp,
             _f32(self.p_sm.scale), _zp(self.p_sm), bw)
        # context = dequant(P V) -> Transpose -> Reshape -> quantize
        e = self._epi(zp_flags=_lib.ZP_ROW | _lib.ZP_COL | _lib.ZP_KCONST, zpa=_zp(self.p_sm), zpb=_zp(pv_), kdim=T,
                      s_acc=[_f32(np.float32(self.p_sm.scale) * np.float32(pv_.scale))],
                      s_out=[_f32(self.p_ctx.scale)], zp_out=[_zp(self.p_ctx)], out=[w["ctx"].ptr], ld_out=D)
        _gemm(EPI_PV, w["p"], w["vt"], B * H, T, Dh, Tp, Tp, Tp, None, T * Tp, Dh * Tp, e)

    def run(self, ws: "Workspace", streams: Streams = _ONE_STREAM):
        """The layer on its input value.  With splitting on, the images in two halves,
        one per HIP stream, so each half's kernels fill the other's partial last dispatch
        rounds; every half touches only its own rows of every buffer."""
        m = self.m
        x = m.x_in.data
        if isinstance(x, QTensor):  # a quantized graph input: its LN and residual-Add
            streams.join()          # consumers both see the dequantized tensor (model.py:528-538),
            x = x.dequantize()      # computed whole-batch on stream 0
        if not isinstance(x, FTensor):
            raise ValueError("fused layer input must be a float or quantized tensor")
        B, T, D = x.dev.shape
        if T != m.tokens or D != self.D:
            raise ValueError(f"layer input {x.dev.shape} does not match the graph ({m.tokens}, {self.D})")
        H, Dh, F = m.heads, m.hdim, self.F
        Tp = (T + 15) // 16 * 16
        w = ws.get(B, T, Tp, H, Dh, D, F, unfused_attention=not self.attn_fused)
        # x1 is layer-private scratch shared by all layers (halves touch disjoint rows);
        # x2 is the layer's output value
        x2 = DeviceArray((B, T, D), np.float32)
        if not self.attn_fused:
            streams.join()  # the three-launch attention runs whole-batch on stream 0
            streams = _ONE_STREAM
        streams.halves(B, lambda s_idx, i0, nb: self._run_part(w, x.dev, w["x1"], x2, i0, nb, s_idx, streams.parts))
        m.x_out.data = FTensor(x2)

    def _run_part(self, w, xd, x1d, x2d, i0, nb, s_idx=0, parts=1):
        """Images [i0, i0 + nb) of the layer (row views of every buffer).  NQK_STREAM_LAG
        (ln1 / qkv / attn): part s > 0 starts the layer only after part s - 1 has finished that
        kernel of it, so the parts' kernels of different kinds run side by side (A/B switch)."""
        m, bw = self.m, self.bw
        lag = _stream_lag() if parts > 1 else None
        if lag and s_idx > 0:
            _lib.call("nqk_event_wait", _lag_event(s_idx - 1))

        def mark(point):
            if lag == point and s_idx + 1 < parts:
                _lib.call("nqk_event_record", _lag_event(s_idx))
        T, D = m.tokens, self.D
        H, Dh, F = m.heads, m.hdim, self.F
        Mrows = nb * T
        Tp = (T + 15) // 16 * 16
        r0 = i0 * T

        def rows(arr, ncol):
            return arr.offset_view(r0 * ncol, (Mrows, ncol))

        x, x1, x2 = (rows(t.reshape((t.size // D, D)), D) for t in (xd, x1d, x2d))
        lnq, ln2q, ctx, hh = rows(w["lnq"], D), rows(w["ln2q"], D), rows(w["ctx"], D), rows(w["h"], F)
        hq = i0 * H * T * Dh  # head-layout offset of the first image
        q, k, v = (w[r].offset_view(hq, (nb * H * T, Dh)) for r in "qkv")
        call = _lib.call
        # 1) LN1 + quantize (LN1 output feeds the Q/K/V MatMuls; already in lnq when the previous
        # layer's FFN-down epilogue computed it)
        if not self.ln1_by_prev:
            _ln_quant(x, self.g1, self.be1, lnq, Mrows, D, self.eps1, self.p_ln1, bw)
        mark("ln1")
        # 2) QKV projection: dequant + bias + head split + quantize with each head consumer's params
        s_a = np.float32(self.p_ln1.scale)
        e = self._epi(zp_flags=_lib.ZP_COL, zpa=_zp(self.p_ln1), group_cols=D, col=self.col_qkv.ptr,
                      col_absmax=self.cmax["qkv"], col_l1max=self.l1max["qkv"], colterm=_ptr(self.ct["qkv"]),
                      s_acc=[_f32(s_a * np.float32(self.s_w[r])) for r in "qkv"],
                      s_out=[_f32(self.p_head[r].scale) for r in "qkv"],
                      zp_out=[_zp(self.p_head[r]) for r in "qkv"],
                      out=[q.ptr, k.ptr, v.ptr], bias=self.bias_qkv.ptr)
        _gemm(EPI_QKV, lnq, self._b(e, "qkv", self.bt_qkv), 1, Mrows, 3 * D, D, D, D, None, 0, 0, e)
        mark("qkv")
        pq, pk, pv_ = self.p_head["q"], self.p_head["k"], self.p_head["v"]
        if self.attn_fused:
            # 3-6) one kernel per (image, head): scores, softmax, P V, context quantize
            a = _lib.Attention()
            a.heads, a.tokens, a.hdim, a.ld_out, a.bit_width = H, T, Dh, D, bw
            a.zq, a.zk = _zp(pq), _zp(pk)
            a.s_qk, a.div = _f32(np.float32(pq.scale) * np.float32(pk.scale)), m.div
            a.s_p, a.zp_p = _f32(self.p_sm.scale), _zp(self.p_sm)
            a.s_pv, a.zv = _f32(np.float32(self.p_sm.scale) * np.float32(pv_.scale)), _zp(pv_)
            a.s_ctx, a.zp_ctx = _f32(self.p_ctx.scale), _zp(self.p_ctx)
            t0 = KM.TIMER.begin() if KM.TIMER is not None else None
            call("nqk_attention_fused", q.vp, k.vp, v.vp, ctx.vp, nb * H, ctypes.byref(a))
            if t0 is not None:
                KM.TIMER.end("attention", t0, (2 * 2 * nb * H * T * T * Dh, 3 * nb * H * T * Dh + nb * T * D))
        else:
            self._attention_unfused(w, nb, T, Tp, H, Dh, D)  # whole batch only (i0 == 0)
        mark("attn")
        # 7) output projection + bias + residual
        e = self._epi(zp_flags=_lib.ZP_COL, zpa=_zp(self.p_ctx), col=self.col_o.ptr, col_absmax=self.cmax["o"], col_l1max=self.l1max["o"],
                      colterm=_ptr(self.ct["o"]),
                      s_acc=[_f32(np.float32(self.p_ctx.scale) * np.float32(self.s_wo))], bias=self.bias_o.ptr,
                      resid=x.ptr, out=[x1.ptr])
        if self.ln_fuse:  # 8) LN2 + quantize inside the epilogue
            self._ln_into(e, self.g2, self.be2, self.eps2, self.p_ln2, ln2q)
        _gemm(EPI_RESID, ctx, self._b(e, "o", self.bt_o), 1, Mrows, D, D, D, D, None, 0, 0, e)
        if not self.ln_fuse:  # 8) LN2 + quantize
            _ln_quant(x1, self.g2, self.be2, ln2q, Mrows, D, self.eps2, self.p_ln2, bw)
        # 9) FFN up + bias + GELU + quantize
        e = self._epi(zp_flags=_lib.ZP_COL, zpa=_zp(self.p_ln2), col=self.col_1.ptr, col_absmax=self.cmax["1"], col_l1max=self.l1max["1"],
                      colterm=_ptr(self.ct["1"]),
                      s_acc=[_f32(np.float32(self.p_ln2.scale) * np.float32(self.s_w1))], bias=self.bias_1.ptr,
                      s_out=[_f32(self.p_h.scale)], zp_out=[_zp(self.p_h)], out=[hh.ptr],
                      div=m.gelu_div, add1=m.gelu_add, mul2=m.gelu_mul)
        if self.glut is not None:
            e.gelu_lut, e.lut_n = self.glut[0].ptr, self.glut[2]
            for j, kv in enumerate(self.glut[1]):
                e.lut_k[j] = kv
        _gemm(EPI_GELU, ln2q, self._b(e, "1", self.bt_1), 1, Mrows, F, D, D, D, None, 0, 0, e)
        # 10) FFN down + bias + residual
        e = self._epi(zp_flags=_lib.ZP_COL, zpa=_zp(self.p_h), col=self.col_2.ptr, col_absmax=self.cmax["2"], col_l1max=self.l1max["2"],
                      colterm=_ptr(self.ct["2"]),
                      s_acc=[_f32(np.float32(self.p_h.scale) * np.float32(self.s_w2))], bias=self.bias_2.ptr,
                      resid=x1.ptr, out=[x2.ptr])
        nl = self.next_ln
        if nl is not None:  # the next layer's LN1 + quantize inside the epilogue, into the shared lnq rows
            self._ln_into(e, nl.g1, nl.be1, nl.eps1, nl.p_ln1, lnq)
        _gemm(EPI_RESID, hh, self._b(e, "2", self.bt_2), 1, Mrows, D, F, F, F, None, 0, 0, e)


def _pack_b(bt, bit_width=8):
    """(image, kind) of a constant Bt [N][K] for the big-tile GEMM: kind 1 = nqk_pack_b
    (int8 tiles), kind 2 = nqk_pack_b4 (nibble-packed int4, bit widths <= 4, whose
    symmetric weights lie in [-8, 7]; NQK_NO_B4 disables); None where the big-tile GEMM
    does not take the shape, or NQK_NO_BPACK is set."""
    N, K = bt.shape
    if K % 192 or N % 4 or os.environ.get("NQK_NO_BPACK"):
        return None
    if bit_width <= 4 and not os.environ.get("NQK_NO_B4"):
        out = DeviceArray(((N + 255) // 256 * 256, K // 2), np.uint8)
        _lib.call("nqk_pack_b4", bt.vp, out.vp, N, K, K)
        return out, 2
    out = DeviceArray(((N + 255) // 256 * 256, K), np.int8)
    _lib.call("nqk_pack_b", bt.vp, out.vp, N, K, K)
    return out, 1


def _pack_pg(bt, bit_width=8, layout=0, nibbles=False):
    """The nqk_pack_pg image of a constant Bt [N][K] (int8 weights, K in {192, 768, 3072},
    N % 64 == 0, padded with zero columns to a multiple of 256; layout 0 for the int8-output
    epilogues QKV / GELU, 1 for the residual epilogues), or with `nibbles` (int4 weights, bit
    widths <= 4) the nqk_pack_pg4 nibble image, or None (NQK_NO_PG set, or a shape the
    persistent 16x16x64 GEMM does not take)."""
    N, K = bt.shape
    if bit_width > 8 or K not in (192, 768, 3072) or N % 64 or os.environ.get("NQK_NO_PG"):
        return None
    if nibbles:
        if bit_width > 4:
            raise ValueError("nibble-packed weights need bit width <= 4")
        out = DeviceArray(((N + 255) // 256 * 256, K // 2), np.uint8)
        _lib.call("nqk_pack_pg4", bt.vp, out.vp, N, K, K, layout)
        return out
    out = DeviceArray(((N + 255) // 256 * 256, K), np.int8)
    _lib.call("nqk_pack_pg", bt.vp, out.vp, N, K, K, layout)
    return out


def _gelu_lut(p, bit_width, div, add1, mul2):
    """(table, bucket coordinate, entries) of the GELU + quantize step function for the FFN-up
    epilogue (nqk_gelu_lut_build), or None where no exact table exists (then the epilogue runs
    the filtered chain) or NQK_NO_GLUT is set."""
    if os.environ.get("NQK_NO_GLUT") or p.zero_point is None or not hasattr(_lib.load(), "nqk_gelu_lut_build"):
        return None
    lut = DeviceArray((int(_lib.load().nqk_gelu_lut_capacity()),), np.uint8)  # the builder's own size
    k = (ctypes.c_float * 5)()
    n = ctypes.c_int32(0)
    _lib.call("nqk_gelu_lut_build", _f32(p.scale), int(p.zero_point), int(bit_width), _f32(div), _f32(add1),
              _f32(mul2), lut.vp, k, ctypes.byref(n))
    if n.value <= 0:
        return None
    return lut, tuple(float(x) for x in k), int(n.value)


def _colterm(col, zpa):
    """col * zpa as an int32 device array, or None when a term leaves int32."""
    c = col.to_host().astype(np.int64) * int(zpa)
    if c.size and (c.min() < -2 ** 31 or c.max() >= 2 ** 31):
        return None
    return DeviceArray.from_host(c.astype(np.int32))


def _l1max(bt) -> int:
    """max over rows n of sum_k |Bt[n][k]| (int32-clamped; >= 1: 0 would mean unknown)."""
    h = np.abs(bt.to_host().astype(np.int64))
    v = int(h.sum(axis=1).max()) if h.size else 1
    return max(1, min(v, 2 ** 31 - 1))


def _absmax(col) -> int:
    """max |column sum| (int32-clamped; 0 would mean unknown to the kernel, so >= 1)."""
    v = int(np.abs(col.to_host()).max()) if col.size else 1
    return max(1, min(v, 2 ** 31 - 1))


def _ln_quant(x, g, b, out, rows, cols, eps, p, bw):
    t0 = KM.TIMER.begin() if KM.TIMER is not None else None
    _lib.call("nqk_ln_quant", x.vp, g.vp, b.vp, out.vp, rows, cols, eps, _f32(p.scale), _zp(p), bw)
    if t0 is not None:
        KM.TIMER.end("ln_quant", t0, (0, rows * cols * 5 + 2 * cols * 4))


def _ptr(arr):
    return None if arr is None else arr.ptr


def _cat0(arrs):
    """Concatenate contiguous device arrays along axis 0."""
    shape = (sum(a.shape[0] for a in arrs),) + tuple(arrs[0].shape[1:])
    out = DeviceArray(shape, arrs[0].dtype)
    off = 0
    for a in arrs:
        _lib.call("nqk_memcpy_d2d", ctypes.c_void_p(out.ptr + off), a.vp, a.nbytes)
        off += a.nbytes
    return out


def _gemm(epi, a, bt, batch, M, N, K, lda, ldb, bmap, a_ms, b_ms, e):
    if K % 16 or lda % 16 or ldb % 16:
        raise ValueError("fused GEMM operands must be 16-byte padded")
    need_a = (batch - 1) * a_ms + (M - 1) * lda + K if batch > 1 else (M - 1) * lda + K
    need_b = (batch - 1) * b_ms + (N - 1) * ldb + K if batch > 1 else (N - 1) * ldb + K
    if e.b_packed:  # a tile-packed image: nqk_pack_b / nqk_pack_b4 sized it for (N, K)
        need_b = ((N + 255) // 256 * 256) * K // (2 if e.b_packed == 2 else 1)
    if need_a > a.size or need_b > bt.size * bt.dtype.itemsize:
        raise ValueError("fused GEMM operand smaller than its shape")
    t0 = KM.TIMER.begin() if KM.TIMER is not None else None
    _lib.call("nqk_qgemm_fused", epi, a.vp, bt.vp, batch, M, N, K, lda, ldb,
              _lib.i64arr(bmap) if bmap is not None else None, a_ms, b_ms, ctypes.byref(e))
    if t0 is not None:
        # algorithmic HBM bytes: A, the weights, the epilogue's outputs (int8; the residual
        # epilogues read and write f32 rows); residual GEMMs split into the attention output
        # projection (K = N) and FFN-down (K > N)
        name = _EPI_NAMES[epi]
        out_b = 8 * M * N if epi == EPI_RESID else (M * N if epi in (EPI_QKV, EPI_GELU) else 0)
        if epi == EPI_RESID:
            name = "down" if K > N else "out"
        KM.TIMER.end("qgemm_" + name, t0, (2 * batch * M * N * K, batch * (M * K + N * K + out_b)))


class Workspace:
    """Scratch buffers of a fused layer, shared by all layers of one plan."""

    def __init__(self):
        self.key = None
        self.bufs = {}

    def get(self, B, T, Tp, H, Dh, D, F, unfused_attention=True):
        key = (B, T, Tp, H, Dh, D, F)
        if key != self.key:
            M = B * T
            self.bufs = {
                "lnq": DeviceArray((M, D), np.int8), "ln2q": DeviceArray((M, D), np.int8),
                "q": DeviceArray((B * H * T, Dh), np.int8), "k": DeviceArray((B * H * T, Dh), np.int8),
                "v": DeviceArray((B * H * T, Dh), np.int8),
                "ctx": DeviceArray((M, D), np.int8), "h": DeviceArray((M, F), np.int8),
                "x1": DeviceArray((B, T, D), np.float32),
            }
            self.key = key
        if unfused_attention and "s" not in self.bufs:
            # scores / probabilities of the three-launch attention (not needed by the fused kernel)
            self.bufs.update({"vt": DeviceArray((B * H, Dh, Tp), np.int8),
                              "s": DeviceArray((B * H, T, T), np.float32),
                              "p": DeviceArray((B * H, T, Tp), np.int8)})
        return self.bufs


class FusedAwayError(RuntimeError):
    """Reading a FusedAway value."""


class FusedAway:
    """The `.data` of a value computed inside a fused step during the last run (it never
    left the step's kernels).  Reading it raises: run with `keep_values = True` to get every
    intermediate (the reference's node loop fills them all, model.py:497-550)."""

    def __init__(self, name):
        self.name = name

    def _error(self):
        return FusedAwayError(f"value {self.name!r} was computed inside a fused plan step and not kept; "
                              "set QModel.keep_values = True to read intermediates")

    def __getattr__(self, attr):
        if attr.startswith("__") and attr.endswith("__"):
            # protocol probes (copy, pickle, NumPy's __array_interface__ / __array_struct__) see a
            # missing attribute; NumPy then calls __array__, which raises
            raise AttributeError(attr)
        raise self._error()

    def __array__(self, *args, **kwargs):
        raise self._error()

    def __repr__(self):
        return f"FusedAway({self.name!r})"


class Plan:
    """Ordered steps: eager nodes and fused layers."""

    def __init__(self, qmodel):
        self.steps = []
        self.ws = Workspace()
        # fused layers as two half batches on two streams (NQK_SPLIT=0: one stream)
        self.split = SPLIT_STREAMS and os.environ.get("NQK_SPLIT", "1") != "0"
        self.fused = 0
        claimed = {}
        self.embeds = 0
        for node in qmodel.nodes:
            if node.op != "Conv" or not FUSED_EMBED:
                continue
            try:
                em = EmbedMatch(qmodel, node)
                fe = FusedEmbed(qmodel, em)
            except NoMatch:
                continue
            for n in em.nodes:
                claimed[n] = fe
            self.embeds += 1
        self.pushdowns = 0
        for node in qmodel.nodes:
            if node.op != "LayerNormalization" or not LN_GATHER:
                continue
            try:
                lg = LnGather(qmodel, node)
            except NoMatch:
                continue
            claimed[lg.ln] = claimed[lg.g] = lg
            self.pushdowns += 1
        if qmodel.bit_width <= 8 and qmodel.bit_width >= 2:
            for node in qmodel.nodes:
                if node.op != "LayerNormalization" or node in claimed:
                    continue
                try:
                    m = LayerMatch(qmodel, node)
                    layer = FusedLayer(qmodel, m)
                except NoMatch:
                    continue
                if any(n in claimed for n in m.nodes):
                    continue
                for n in m.nodes:
                    claimed[n] = layer
        placed = set()
        for node in qmodel.nodes:
            layer = claimed.get(node)
            if layer is None:
                self.steps.append(("node", node))
            elif isinstance(layer, LnGather):
                if node is layer.g:
                    self.steps.append(("ln_gather", layer))
            elif isinstance(layer, FusedEmbed):
                if node is layer.m.conv:
                    self.steps.append(("embed_pre", layer))
                elif node is layer.m.add:
                    self.steps.append(("embed", layer))
            elif id(layer) not in placed:
                placed.add(id(layer))
                self.steps.append(("layer", layer))
                self.fused += 1
        # consecutive fused layers of width 192: layer i's FFN-down epilogue computes layer i + 1's
        # LN1 (the same workspace rows its QKV GEMM reads: equal layer dimensions)
        for (k0, a), (k1, b) in zip(self.steps, self.steps[1:]):
            if (k0 == "layer" and k1 == "layer" and a.ln_fuse and b.ln_fuse and b.m.x_in is a.m.x_out and
                    (a.D, a.F, a.m.heads, a.m.hdim, a.m.tokens, a.attn_fused) ==
                    (b.D, b.F, b.m.heads, b.m.hdim, b.m.tokens, b.attn_fused)):
                a.next_ln, b.ln1_by_prev = b, True
        # every value a fused step computes; each run first marks them all FusedAway, so that
        # no tensor of an earlier run (eager, keep_values) can be read as if it were this
        # run's; the steps then set the values their consumers outside the step read
        self.internal = [v for node in qmodel.nodes if node in claimed for v in node.outputs]

    def run(self, qmodel, times=None, profile=False):
        streams = Streams(self.split, int(os.environ.get("NQK_STREAMS", "2")))
        for v in self.internal:
            v.data = FusedAway(v.name)
        try:
            for kind, obj in self.steps:
                if kind == "node":
                    streams.join()  # everything eager waits for both streams
                    qmodel._run_node(obj, times, profile)
                elif kind == "embed_pre":
                    obj.pre(qmodel)  # host only: a shape placeholder
                elif kind == "embed":
                    obj.run(qmodel, streams)
                elif kind == "ln_gather":
                    streams.join()
                    obj.run(qmodel, times, profile)
                else:
                    obj.run(self.ws, streams)
        finally:
            _lib.call("nqk_set_stream", 0)
            streams.join()


def compile_plan(qmodel) -> Plan:
    return Plan(qmodel)
