"""The RCCL device path of the replicas on one GPU: a
1-rank communicator (ReplicaGroup(force_device_comm=True)) runs the same pack ->
ncclBroadcast -> blob.attach path that ranks 1..N-1 take, and the ncclGather of the logits
into rank 0's [world, B, 1000] buffer.  The attached model must give the source model's
outputs bit for bit (reference: model.py:486-565 QModel.__call__ on both)."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _vit(batch):
    from numpy_quant import onnx_proto
    from numpy_quant.model import Model
    proto = onnx_proto.load(os.path.join(ROOT, "numpy-quant_amd", "models", "vit_image_classifier_no_weights.onnx"),
                            synthetic_weights=True)
    if batch != 1:
        onnx_proto.rebatch(proto, batch)
    return Model.from_onnx(proto)


def test_rccl_one_rank_broadcast_attach_and_gather():
    from numpy_quant import _lib
    from numpy_quant.device import DeviceArray
    from numpy_quant.replicas import ReplicaGroup
    from numpy_quant.tensor import FTensor
    B = 2
    rng = np.random.default_rng(11)
    x = rng.standard_normal((B, 3, 224, 224)).astype(np.float32)
    src_model = _vit(B)
    qmodel = src_model.quantize([x], bit_width=8)
    ref = qmodel([x])[0]
    group = ReplicaGroup(rank=0, world=1, force_device_comm=True)
    try:
        attached, nbytes = group.broadcast_qmodel(_vit(B), qmodel)
        assert group.device_comm and nbytes > 80_000_000  # the whole int8 ViT-Base blob went through RCCL
        assert attached is not qmodel
        out = attached([x])[0]
        np.testing.assert_array_equal(out, ref)
        # gather of the device logits into a [world, B, 1000] destination
        dev = attached.outputs_device()[0].dev
        dst = DeviceArray((1, B, 1000), np.float32)
        group.gather(dev, dst)
        _lib.call("nqk_sync")
        np.testing.assert_array_equal(dst.to_host()[0], ref)
    finally:
        group.close()
