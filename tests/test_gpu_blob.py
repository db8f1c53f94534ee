"""GPU: the packed quantized-model blob (blob.py) and QTensor.relu on device.

QModel.save -> Model.load_quantized must give back the same model: the same
quantization parameters (values and Python types) and bit-identical outputs, without
a calibration forward or any re-quantization (reference state: model.py:441-442
quant_params + the quantized Constants of model.py:357-415)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
MODELS = os.path.join(ROOT, "numpy-quant_amd", "models")


@pytest.mark.parametrize("bw", [8, 4, 12])
def test_mlp_blob_round_trip(tmp_path, bw):
    from numpy_quant.model import Model
    X = np.load(os.path.join(GOLDEN, "mlp.npz"))["X"]
    x = np.random.default_rng(bw).uniform(-1.2, 1.2, size=(333, 2)).astype(np.float32)
    model = Model.from_onnx(os.path.join(MODELS, "mlp.onnx"))
    qmodel = model.quantize([X], bit_width=bw)
    want = qmodel([x])[0]
    path = tmp_path / "mlp.nqk"
    size = qmodel.save(path)
    assert size == os.path.getsize(path)
    fresh = Model.from_onnx(os.path.join(MODELS, "mlp.onnx"))
    q2 = fresh.load_quantized(path)
    assert q2.bit_width == bw
    assert set(q2.quant_params) == set(qmodel.quant_params)
    for k, p in qmodel.quant_params.items():
        p2 = q2.quant_params[k]
        assert type(p2.scale) is type(p.scale) and np.asarray(p2.scale).tobytes() == np.asarray(p.scale).tobytes(), k
        assert type(p2.zero_point) is type(p.zero_point), k
        assert (p.zero_point is None) or int(p2.zero_point) == int(p.zero_point), k
    np.testing.assert_array_equal(q2([x])[0], want)


def test_vit_blob_round_trip(tmp_path):
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    path_onnx = os.path.join(MODELS, "vit_image_classifier_no_weights.onnx")
    x = np.random.default_rng(3).standard_normal((2, 3, 224, 224)).astype(np.float32)
    proto = onnx_proto.load(path_onnx, synthetic_weights=True)
    onnx_proto.rebatch(proto, 2)
    qmodel = Model.from_onnx(proto).quantize([x], bit_width=8)
    want = qmodel([x])[0]
    blob = tmp_path / "vit.nqk"
    qmodel.save(blob)
    # the graph with DIFFERENT synthetic weights: every constant must come from the blob
    proto2 = onnx_proto.load(path_onnx, synthetic_weights=True, seed=99)
    onnx_proto.rebatch(proto2, 2)
    q2 = Model.from_onnx(proto2).load_quantized(blob)
    np.testing.assert_array_equal(q2([x])[0], want)


def test_blob_of_another_graph_is_refused(tmp_path):
    """A blob attaches only to a graph with exactly its constants and shapes:
    the ViT-Ti blob (redimensioned graph, same initializer names) must not attach to the
    ViT-Base graph, and the MLP blob not to the ViT."""
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    path_onnx = os.path.join(MODELS, "vit_image_classifier_no_weights.onnx")
    tiny = onnx_proto.load(path_onnx, synthetic_weights=True)
    onnx_proto.redimension(tiny, 192, 3, 768)
    x = np.random.default_rng(5).standard_normal((1, 3, 224, 224)).astype(np.float32)
    qtiny = Model.from_onnx(tiny).quantize([x], bit_width=8)
    blob = tmp_path / "tiny.nqk"
    qtiny.save(blob)
    base = Model.from_onnx(onnx_proto.load(path_onnx, synthetic_weights=True))
    with pytest.raises(ValueError, match="shape"):
        base.load_quantized(blob)
    X = np.load(os.path.join(GOLDEN, "mlp.npz"))["X"]
    qmlp = Model.from_onnx(os.path.join(MODELS, "mlp.onnx")).quantize([X], bit_width=8)
    mblob = tmp_path / "mlp.nqk"
    qmlp.save(mblob)
    with pytest.raises(ValueError, match="differ"):
        Model.from_onnx(onnx_proto.load(path_onnx, synthetic_weights=True)).load_quantized(mblob)


def test_qtensor_relu_device():
    """tensor.py:212-215: values below the zero point become the zero point; a zero
    point outside the int8 storage range widens the storage."""
    from numpy_quant.tensor import QTensor
    rng = np.random.default_rng(0)
    q = rng.integers(-128, 128, size=(7, 33)).astype(np.int64)
    for zp in (-5, 0, 127, -128, 140, -300):
        t = QTensor(q, 8, np.float32(0.1), np.int64(zp))
        r = t.relu()
        want = q.copy()
        want[want < zp] = zp
        np.testing.assert_array_equal(r.data, want)
        assert r.bit_width == 8 and r.zero_point == zp and r.scale == np.float32(0.1)
    with pytest.raises(TypeError):
        QTensor(q, 8, np.float32(0.1), None).relu()
