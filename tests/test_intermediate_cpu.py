"""Engine-neutral IR (S/utils/intermediate/*): BlasToIR flattening, IRToBlas rebuild, IRToDnn inference fusion
(BN folded into conv weights), Container.toGraph sharing layers."""
import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.models.inception import Inception_v1_NoAuxClassifier
from bigdl_amd.models.resnet import DatasetType, ResNet
from bigdl_amd.utils.intermediate import BlasToIR, ConversionUtils, IRToDnn


def _randomize_bn(m):
    for layer in m.flattened_layers():
        if hasattr(layer, "runningMean"):
            layer.runningMean.uniform_(-0.5, 0.5)
            layer.runningVar.uniform_(0.5, 1.5)


@pytest.mark.parametrize("which", ["resnet20", "inception_v1"])
def test_ir_roundtrip_and_bn_folding(which):
    torch.manual_seed(0)
    if which == "resnet20":
        m, x = ResNet(10, 20, dataSet=DatasetType.CIFAR10), torch.randn(2, 3, 32, 32)
    else:
        m, x = Inception_v1_NoAuxClassifier(10), torch.randn(2, 3, 224, 224)
    _randomize_bn(m)
    m.evaluate()
    ref = m.forward(x)
    ir = BlasToIR.convert(m)
    assert not any(n.element.general for n in ir.nodes())          # every layer has an IR op
    g = ConversionUtils.convert(m, "blas")
    assert torch.allclose(g.forward(x), ref, atol=1e-6)
    fused = IRToDnn.fuse(BlasToIR.convert(m))
    if which == "resnet20":
        assert len(fused.nodes()) < len(ir.nodes())                  # BN nodes folded away
    assert torch.allclose(fused.build("blas").forward(x), ref, atol=1e-4)


def test_container_to_graph_shares_layers():
    torch.manual_seed(0)
    seq = nn.Sequential().add(nn.Linear(4, 5)).add(nn.ReLU()).add(
        nn.ConcatTable().add(nn.Linear(5, 3)).add(nn.Linear(5, 3))).add(nn.CAddTable())
    g = seq.toGraph()
    x = torch.randn(6, 4)
    assert torch.allclose(g.forward(x), seq.forward(x))
    lin = seq.modules[0]
    assert any(n.element is lin for n in g.order)
    gy = torch.randn(6, 3)
    seq.zeroGradParameters()
    gi_seq = seq.backward(x, gy).clone()
    gw_seq = lin.gradWeight.clone()
    seq.zeroGradParameters()
    g.forward(x)
    gi_g = g.backward(x, gy)
    assert torch.allclose(gi_g, gi_seq, atol=1e-6) and torch.allclose(lin.gradWeight, gw_seq, atol=1e-6)


def test_graph_inference_fusion_plan_cpu():
    """Caffe-style BN + Scale pairs fold into the conv at the IR level; the graph fusion pass schedules a concat's
    non-conv inputs before its producer convs and the residual shortcut before the residual conv, and the fused
    graph computes the same function (on the CPU the run-time hooks leave every node unfused)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    from test_graph_fusion_gpu import _inception_residual_graph

    from bigdl_amd.nn.fusion import fuse_graph_for_inference
    from bigdl_amd.utils.intermediate import BlasToIR, IRToDnn

    g = _inception_residual_graph()
    x = torch.randn(2, 3, 16, 16)
    ref = g.forward(x).clone()
    cg = IRToDnn.fuse(BlasToIR.convert(g)).build("blas", train=False)
    names = [type(n.element).__name__ for n in cg.order]
    assert "Scale" not in names and "SpatialBatchNormalization" not in names
    fuse_graph_for_inference(cg)
    order = [type(n.element).__name__ for n in cg.order]
    pos = {n.id: i for i, n in enumerate(cg.order)}
    join = [n for n in cg.order if names and type(n.element).__name__ == "JoinTable"][0]
    pool = [p for p in join.prevs if type(p.element).__name__ == "SpatialMaxPooling"][0]
    convs = [n for n in cg.order if n.fuse_pre is not None and type(n.element).__name__ == "SpatialConvolution"]
    assert convs and all(pos[pool.id] < pos[c.id] for c in convs if c.id != cg.order[1].id), order
    assert torch.allclose(cg.forward(x), ref, atol=1e-5)
