#!/usr/bin/env python
"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container, where /root/reference exists (read-only).  The
reference never travels: only the .npz/.json vectors this script writes are
committed.  Usage:  python tests/golden/make_golden.py [--vit] [--only l1,mlp,attn,layer,api,vit,vit4]

How the reference is imported:
  * numpy_quant.numpy_quantization / .tensor / .numpy_helper are pure NumPy and
    are imported as they are;
  * numpy_quant.model does `import onnx` at module level (model.py:8-10) although
    only `Model.from_onnx` uses it.  `onnx` is not installed, so an EMPTY
    placeholder module is registered in sys.modules for the import statement to
    succeed (it defines nothing but the `ModelProto` name used in an annotation).
    `from_onnx` is never called: graphs are decoded by this repo's own reader and
    assembled with the reference's own IR constructors (Constant / Variable /
    Node / Model, model.py:17-54, 216-221), wired exactly as model.py:253-292 does.
    Everything the fixtures record (`Model.__call__`, `Model.quantize`,
    `QModel.__call__` and the L1 functions) is the reference's unmodified code.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True


def _import_reference():
    if "onnx" not in sys.modules:
        ph = types.ModuleType("onnx")
        ph.ModelProto = object  # annotation target only (model.py:250)
        for sub in ("mapping", "numpy_helper", "helper"):
            m = types.ModuleType("onnx." + sub)
            setattr(ph, sub, m)
            sys.modules["onnx." + sub] = m
        sys.modules["onnx"] = ph
    sys.path.insert(0, REF)
    import numpy_quant.numpy_quantization as rq
    import numpy_quant.tensor as rt
    import numpy_quant.numpy_helper as rh
    import numpy_quant.model as rm
    sys.path.pop(0)
    # the reference package must not shadow the product package of the same name
    mods = {k: sys.modules.pop(k) for k in list(sys.modules) if k == "numpy_quant" or k.startswith("numpy_quant.")}
    return rq, rt, rh, rm, mods


rq, rt, rh, rm, _refmods = _import_reference()
sys.path.insert(0, os.path.join(REPO, "numpy-quant_amd"))
from numpy_quant import onnx_proto  # noqa: E402  (this repo's decoder, not the reference)


def reference_model(proto):
    """Reference IR from a decoded graph, wired as model.py:253-292."""
    g = proto.graph
    vd = {}
    for t in g.initializer:
        vd[t.name] = rm.Constant(t.name, outputs=[], data=rt.FTensor(np.array(t.to_array())))
    inputs = []
    for vi in g.input:
        vd[vi.name] = rm.Variable(vi.name, inputs=[], outputs=[])
        inputs.append(vd[vi.name])
    nodes = {}
    for n in g.node:
        node = rm.Node(name=n.name, op=n.op_type,
                       attrs={a.name: onnx_proto.attribute_value(a) for a in n.attribute},
                       inputs=[vd[i] for i in n.input], outputs=[])
        for i in n.input:
            vd[i].outputs.append(node)
        for o in n.output:
            if o not in vd:
                vd[o] = rm.Variable(name=o, inputs=[node], outputs=[])
            else:
                vd[o].inputs.append(node)
        node.outputs = [vd[o] for o in n.output]
        nodes[n.name] = node
    outputs = [vd[vi.name] for vi in g.output]
    return rm.Model(list(nodes.values()), list(vd.values()), inputs, outputs)


def _h(arr: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest()


def tensor_record(t):
    """Canonical (kind, array) of a reference tensor: ITensor/FTensor data, QTensor int64 data."""
    if isinstance(t, rt.QTensor):
        return "Q", np.asarray(t.data, dtype=np.int64)
    if isinstance(t, rt.FTensor):
        return "F", np.asarray(t.data, dtype=np.float32)
    return "I", np.asarray(t.data)


def qparams_json(qp) -> dict:
    out = {}
    for k, p in qp.items():
        zp = p.zero_point
        out[k] = {"scale_bits": int(np.asarray(p.scale, np.float32).view(np.uint32)),
                  "zp": None if zp is None else int(zp),
                  "zp_is_scalar_zero": bool(zp is not None and not isinstance(zp, np.ndarray))}
    return out


# ----------------------------------------------------------------------------- L1 vectors
def gen_l1(path):
    rng = np.random.default_rng(20260101)
    rec = {}
    # quant_parameters: (min, max, bw, asym) grid incl. out-of-range zero points and zp -> 0
    qp_cases = []
    for bw in (1, 2, 3, 4, 5, 8, 12, 16):
        for mn, mx in [(-1.5, 2.0), (0.0, 2.0), (-2.0, 0.0), (-3.25, -0.5), (0.25, 7.0),
                       (-0.01, 5.0), (-127.0, 128.0), (-1e-3, 1e-3), (-0.3, 11.7), (-6.0, 6.0 * 127 / 128)]:
            for asym in (True, False):
                s, z = rq.quant_parameters(np.float32(mn), np.float32(mx), bw, asym)
                qp_cases.append([mn, mx, bw, int(asym), float(s),
                                 0 if z is None else int(z), int(z is None),
                                 int(z is not None and not isinstance(z, np.ndarray))])
    rec["qp_cases"] = np.array(qp_cases, dtype=np.float64)

    # quantize: normal data, exact .5 ties, clipping, zp variants, several bit widths
    xs = []
    base = rng.standard_normal(4096).astype(np.float32) * np.float32(3.0)
    ties = (np.arange(-300, 300, dtype=np.float32) + np.float32(0.5))
    xs = np.concatenate([base, ties, np.array([0.0, -0.0, 1e-30, -1e-30, 1e30, -1e30], np.float32)])
    rec["q_x"] = xs
    q_cases = []
    outs = []
    for bw in (1, 2, 4, 8, 12, 16, 32):
        for s, zp in [(1.0, None), (1.0, 0), (1.0, -138), (0.0213, 17), (0.0213, None), (0.5, 3),
                      (0.05, -140), (3.0, 0)]:
            sc = np.array(s, dtype=np.float32)
            zpa = None if zp is None else (np.int64(0) if zp == 0 else np.array(zp, dtype=np.int64))
            outs.append(rq.quantize(xs, bw, sc, zpa))
            q_cases.append([bw, s, -1 if zp is None else 0, 0 if zp is None else zp])
    rec["q_cases"] = np.array(q_cases, dtype=np.float64)
    rec["q_out"] = np.stack(outs)

    # dequantize with scalar / row / full zero points
    qi = rng.integers(-2 ** 20, 2 ** 20, size=(6, 7), dtype=np.int64)
    rec["dq_in"] = qi
    rec["dq_s"] = np.array(0.0173, np.float32)
    zrow = rng.integers(-500, 500, size=(1, 7), dtype=np.int64)
    zfull = rng.integers(-5000, 5000, size=(6, 7), dtype=np.int64)
    rec["dq_zrow"] = zrow
    rec["dq_zfull"] = zfull
    rec["dq_none"] = rq.dequantize(qi, rec["dq_s"], None)
    rec["dq_scalar"] = rq.dequantize(qi, rec["dq_s"], np.array(-37, np.int64))
    rec["dq_row"] = rq.dequantize(qi, rec["dq_s"], zrow)
    rec["dq_full"] = rq.dequantize(qi, rec["dq_s"], zfull)
    big = np.array([2 ** 24 + 1, 2 ** 30 + 3, -(2 ** 33) - 7, 123456789012], np.int64)
    rec["dq_big"] = big
    rec["dq_big_out"] = rq.dequantize(big, np.array(0.1, np.float32), None)

    # q_matmul: the 4 zp cases on test_quantization.py shapes (2,1,4,3)x(1,2,3,4) and a 2-D case
    a = rng.integers(-128, 128, size=(2, 1, 4, 3), dtype=np.int64)
    b = rng.integers(-128, 128, size=(1, 2, 3, 4), dtype=np.int64)
    a2 = rng.integers(-128, 128, size=(37, 70), dtype=np.int64)
    b2 = rng.integers(-128, 128, size=(70, 45), dtype=np.int64)
    rec["mm_a"], rec["mm_b"], rec["mm_a2"], rec["mm_b2"] = a, b, a2, b2
    sa, sb = np.array(0.031, np.float32), np.array(0.0047, np.float32)
    for tag, za, zb in [("nn", None, None), ("an", np.array(-9, np.int64), None),
                        ("na", None, np.array(5, np.int64)), ("aa", np.array(-138, np.int64), np.array(11, np.int64))]:
        for sfx, (A, B) in (("", (a, b)), ("2", (a2, b2))):
            acc, s, z = rq.q_matmul(A, sa, za, B, sb, zb)
            rec[f"mm{sfx}_{tag}_acc"] = acc
            rec[f"mm{sfx}_{tag}_s"] = np.float32(s)
            rec[f"mm{sfx}_{tag}_zp"] = np.zeros(0, np.int64) if z is None else np.asarray(z)
            for rz in (None, np.array(-3, np.int64)):
                for bw in (8, 4):
                    key = f"rq{sfx}_{tag}_{'n' if rz is None else 'a'}_{bw}"
                    rec[key] = rq.requantize(acc, s, z, np.array(0.37, np.float32), rz, bw)

    # erf over a dense range and special points
    ex = np.concatenate([np.linspace(-6, 6, 20001, dtype=np.float32),
                         np.array([0.0, -0.0, 1e-8, -1e-8, 9.0, -9.0, 30.0], np.float32)])
    rec["erf_x"] = ex
    rec["erf_y"] = rh.erf(ex)

    # conv2d: test_conv2d.py:20-27 geometry (float32) and a patch-embed-like case
    x = rng.standard_normal((2, 3, 9, 10)).astype(np.float32)
    w = rng.standard_normal((2, 3, 3, 2)).astype(np.float32)
    bb = rng.standard_normal(2).astype(np.float32)
    rec["cv_x"], rec["cv_w"], rec["cv_b"] = x, w, bb
    rec["cv_y"] = rt.fconv2d(rt.FTensor(x), rt.FTensor(w), rt.FTensor(bb), (0, 2, 2, 1), (2, 1)).data
    x2 = rng.standard_normal((2, 3, 64, 48)).astype(np.float32)
    w2 = (rng.standard_normal((96, 3, 16, 16)) * 0.05).astype(np.float32)
    b2 = rng.standard_normal(96).astype(np.float32)
    rec["cv2_x"], rec["cv2_w"], rec["cv2_b"] = x2, w2, b2
    rec["cv2_y"] = rt.fconv2d(rt.FTensor(x2), rt.FTensor(w2), rt.FTensor(b2), (0, 0, 0, 0), (16, 16)).data

    # float ops used by the ViT graph, through the reference's FTensor methods
    lx = (rng.standard_normal((3, 5, 768)) * 2 + 0.3).astype(np.float32)
    lg = (1 + 0.02 * rng.standard_normal(768)).astype(np.float32)
    lb = (0.02 * rng.standard_normal(768)).astype(np.float32)
    rec["ln_x"], rec["ln_g"], rec["ln_b"] = lx, lg, lb
    rec["ln_y"] = rm.onnx_operator_implementation(
        "LayerNormalization", [rt.FTensor(lx), rt.FTensor(lg), rt.FTensor(lb)],
        {"axis": -1, "epsilon": 9.999999960041972e-13})[0].data
    sx = (rng.standard_normal((2, 3, 197, 197)) * 4).astype(np.float32)
    rec["sm_x"] = sx
    rec["sm_y"] = rm.onnx_operator_implementation("Softmax", [rt.FTensor(sx)], {"axis": -1})[0].data
    gx = (rng.standard_normal(50000) * 3).astype(np.float32)
    rec["sg_x"] = gx
    rec["sg_y"] = rm.onnx_operator_implementation("Sigmoid", [rt.FTensor(gx)], {})[0].data
    rec["relu_y"] = rm.onnx_operator_implementation("Relu", [rt.FTensor(gx)], {})[0].data
    np.savez_compressed(path, **rec)
    print("wrote", path, os.path.getsize(path), "bytes")


# ----------------------------------------------------------------------------- model-level vectors
def run_model(proto, calib, test_inputs, bit_width):
    model = reference_model(proto)
    qmodel = model.quantize(calib, bit_width=bit_width)
    t0 = time.time()
    outs, prof = qmodel(test_inputs, profile=True)
    dt = time.time() - t0
    vals = {}
    for v in qmodel.values:
        if v.data is None:
            continue
        kind, arr = tensor_record(v.data)
        vals[v.name] = (kind, arr)
    return model, qmodel, outs, vals, prof, dt


def gen_mlp(out_dir):
    from sklearn.datasets import make_circles
    X, Y = make_circles(n_samples=100, noise=0.03, random_state=0)
    X = X.astype(np.float32)
    proto = onnx_proto.load(os.path.join(REF, "models", "mlp.onnx"))
    meta = {}
    arrays = {"X": X, "Y": Y.astype(np.int64)}
    for bw in range(1, 17):
        model, qmodel, outs, vals, prof, dt = run_model(proto, [X], [X], bw)
        arrays[f"bw{bw}_out"] = outs[0]
        meta[f"bw{bw}"] = {"qparams": qparams_json(qmodel.quant_params)}
        if bw in (8, 4):
            for name, (kind, arr) in vals.items():
                arrays[f"bw{bw}|{kind}|{name}"] = arr
        # float model values (after quantize() ran the float forward on X)
    fvals = {v.name: tensor_record(v.data) for v in model.values if v.data is not None}
    for name, (kind, arr) in fvals.items():
        arrays[f"float|{kind}|{name}"] = arr
    np.savez_compressed(os.path.join(out_dir, "mlp.npz"), **arrays)
    with open(os.path.join(out_dir, "mlp_qparams.json"), "w") as fh:
        json.dump(meta, fh, indent=0, sort_keys=True)
    print("wrote mlp fixtures")


def gen_vit_part(out_dir, fname, tag, batch, bit_widths=(8, 4), seed=0, keep_small=True):
    proto = onnx_proto.load(os.path.join(REF, "models", "vit", fname), synthetic_weights=True, seed=seed)
    if batch != 1:
        onnx_proto.rebatch(proto, batch)
    shape = [batch] + [d for d in proto.graph.input[0].shape[1:]]
    rng = np.random.default_rng(1000 + batch)
    x_cal = rng.standard_normal(shape).astype(np.float32)
    x_run = rng.standard_normal(shape).astype(np.float32)
    arrays = {"x_cal": x_cal, "x_run": x_run}
    meta = {"file": fname, "batch": batch, "seed": seed}
    for bw in bit_widths:
        model, qmodel, outs, vals, prof, dt = run_model(proto, [x_cal], [x_run], bw)
        arrays[f"bw{bw}_out"] = outs[0]
        hashes = {}
        for name, (kind, arr) in vals.items():
            hashes[name] = [kind, list(arr.shape), _h(arr)]
            if keep_small and arr.size <= 40_000 and kind != "I":
                arrays[f"bw{bw}|{kind}|{name}"] = arr
        meta[f"bw{bw}"] = {"qparams": qparams_json(qmodel.quant_params), "hashes": hashes,
                           "ref_seconds": dt, "profile": prof}
        if bw == bit_widths[0]:
            fh_ = {v.name: [tensor_record(v.data)[0], list(np.shape(v.data.data)), _h(tensor_record(v.data)[1])]
                   for v in model.values if v.data is not None}
            meta["float_hashes"] = fh_
        print(f"  {tag} bw{bw}: reference QModel {dt:.2f}s")
    np.savez_compressed(os.path.join(out_dir, f"{tag}.npz"), **arrays)
    with open(os.path.join(out_dir, f"{tag}.json"), "w") as fh:
        json.dump(meta, fh, indent=0, sort_keys=True)
    print("wrote", tag)


def gen_api(out_dir):
    """Reference API surfaces outside the node loops (VERDICT r2 missing #4 / next #8):
    QTensor.sigmoid (tensor.py:217-221), QTensor.relu on narrow storage (tensor.py:212-215),
    tensor_min_max / quantize_tensor_min_max (tensor.py:232-242); Model.quantize of the MLP
    on ONE calibration sample (one-row float products: model.py:328-442) and of the full
    ViT-Base graph on the bench's 8 calibration images (quantization parameters only)."""
    rng = np.random.default_rng(20261017)
    arrays, meta = {}, {}
    # QTensor.sigmoid: int8 storage, several scales / zero points (incl. None)
    sig = []
    for i, (bw, s, zp) in enumerate([(8, 0.05, 3), (8, 0.0123, -20), (4, 0.3, 2), (8, 0.031, None), (6, 0.11, 0)]):
        lo, hi = (-(1 << (bw - 1)), (1 << (bw - 1)) - 1)
        q = rng.integers(lo, hi + 1, size=(7, 33), dtype=np.int64)
        zpa = None if zp is None else (np.int64(0) if zp == 0 else np.array(zp, np.int64))
        t = rt.QTensor(q, bw, np.array(s, np.float32), zpa)
        y = t.sigmoid()
        arrays[f"sig{i}_q"] = q
        arrays[f"sig{i}_y"] = np.asarray(y.data, np.int64)
        sig.append({"bw": bw, "scale": s, "zp": zp})
    meta["sigmoid"] = sig
    # QTensor.relu (int64 data, as the reference requires) with zero points inside / outside the storage range
    rel = []
    for i, zp in enumerate([5, -3, 140, -300]):
        q = rng.integers(-128, 128, size=(9, 17), dtype=np.int64)
        y = rt.QTensor(q, 8, np.array(0.02, np.float32), np.array(zp, np.int64)).relu()
        arrays[f"relu{i}_q"] = q
        arrays[f"relu{i}_y"] = np.asarray(y.data)
        rel.append({"zp": zp, "dtype": str(np.asarray(y.data).dtype)})
    meta["relu"] = rel
    # tensor_min_max / quantize_tensor_min_max on FTensors of mixed / one-signed data
    mm = []
    for i, (shift, scale) in enumerate([(0.0, 1.0), (3.0, 0.5), (-4.0, 0.25), (0.0, 1e-3), (0.7, 2.0)]):
        x = (rng.standard_normal((5, 41)) * scale + shift).astype(np.float32)
        mn, mx = rt.tensor_min_max(rt.FTensor(x))
        arrays[f"mm{i}_x"] = x
        rec = {"min_bits": int(np.asarray(mn, np.float32).view(np.uint32)),
               "max_bits": int(np.asarray(mx, np.float32).view(np.uint32)),
               "min_dtype": str(np.asarray(mn).dtype), "max_dtype": str(np.asarray(mx).dtype), "q": {}}
        for bw in (8, 4):
            for asym in (True, False):
                qt = rt.quantize_tensor_min_max(rt.FTensor(x), bw, asym)
                key = f"{bw}_{int(asym)}"
                arrays[f"mm{i}_q{key}"] = np.asarray(qt.data, np.int64)
                rec["q"][key] = {"scale_bits": int(np.asarray(qt.scale, np.float32).view(np.uint32)),
                                 "zp": None if qt.zero_point is None else int(qt.zero_point)}
        mm.append(rec)
    meta["minmax"] = mm
    # the MLP calibrated on one sample (X[0:1]), run on the whole set, bit widths 8 and 4
    from sklearn.datasets import make_circles
    X, _ = make_circles(n_samples=100, noise=0.03, random_state=0)
    X = X.astype(np.float32)
    proto = onnx_proto.load(os.path.join(REF, "models", "mlp.onnx"))
    one = {}
    for i in (0, 7):
        for bw in (8, 4):
            model = reference_model(proto)
            qmodel = model.quantize([X[i:i + 1]], bit_width=bw)
            out = qmodel([X])[0]
            arrays[f"mlp1_{i}_bw{bw}_out"] = out
            one[f"{i}_bw{bw}"] = qparams_json(qmodel.quant_params)
    meta["mlp_one_sample"] = one
    # ViT-Base calibrated on the bench's 8 images (bench.py build_vit: seed 12345)
    vproto = onnx_proto.load(os.path.join(REF, "models", "vit", "vit_image_classifier_no_weights.onnx"),
                             synthetic_weights=True)
    onnx_proto.rebatch(vproto, 8)
    x_cal = np.random.default_rng(12345).standard_normal((8, 3, 224, 224)).astype(np.float32)
    t0 = time.time()
    vmodel = reference_model(vproto)
    vq = vmodel.quantize([x_cal], bit_width=8)
    meta["vit_b8_calibration"] = {"qparams": qparams_json(vq.quant_params), "seconds": time.time() - t0,
                                  "seed": 12345}
    np.savez_compressed(os.path.join(out_dir, "api.npz"), **arrays)
    with open(os.path.join(out_dir, "api.json"), "w") as fh:
        json.dump(meta, fh, indent=0, sort_keys=True)
    print("wrote api fixtures")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vit", action="store_true", help="also run the full ViT-Base graph (B=1, ~3 min)")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    if not os.path.isdir(REF):
        sys.exit("reference not present: fixtures are generated in the build container only")
    only = set(args.only.split(",")) if args.only else None
    if not only or "l1" in only:
        gen_l1(os.path.join(HERE, "l1.npz"))
    if not only or "mlp" in only:
        gen_mlp(HERE)
    if not only or "attn" in only:
        gen_vit_part(HERE, "vit_image_classifier_self_attention_no_weights.onnx", "attn_b1", 1)
        gen_vit_part(HERE, "vit_image_classifier_self_attention_no_weights.onnx", "attn_b2", 2, bit_widths=(8,))
    if not only or "layer" in only:
        gen_vit_part(HERE, "vit_image_classifier_encoder_layer_no_weights.onnx", "layer_b1", 1, keep_small=False)
    if not only or "api" in only:
        gen_api(HERE)
    if args.vit or (only and "vit" in only):
        gen_vit_part(HERE, "vit_image_classifier_no_weights.onnx", "vit_b1", 1, bit_widths=(8,), keep_small=False)
    if only and "vit4" in only:
        # configs[4] pinned at the full-classifier level (VERDICT r5 missing #3): the reference's own
        # Model.quantize(bit_width=4) + QModel.__call__ on the same seeded graph and images as vit_b1
        gen_vit_part(HERE, "vit_image_classifier_no_weights.onnx", "vit_b1_bw4", 1, bit_widths=(4,), keep_small=False)


if __name__ == "__main__":
    main()
