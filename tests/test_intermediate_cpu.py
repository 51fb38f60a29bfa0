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


def test_graph_training_fusion_plans_on_single_consumer_edges():
    """nn.fusion._fuse_graph_training: producers fuse only into their ONLY consumer; a fanned-out conv output,
    a graph output and a DynamicGraph are left alone."""
    from bigdl_amd import nn
    from bigdl_amd.nn.fusion import fuse_for_training

    inp = nn.Input()
    c1 = nn.SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1)
    b1 = nn.SpatialBatchNormalization(8)
    r1 = nn.ReLU()
    c2 = nn.SpatialConvolution(8, 8, 3, 3, 1, 1, 1, 1)
    b2 = nn.SpatialBatchNormalization(8)
    c3 = nn.SpatialConvolution(8, 8, 1, 1)          # c2's output fans out to b2 and c3: no stats epilogue
    n1 = r1(b1(c1(inp)))
    n2 = c2(n1)
    out = nn.CAddTable()(b2(n2), c3(n2))
    g = nn.Graph(inp, out)
    fuse_for_training(g)
    assert c1.emit_stats and b1.fuse_relu and r1.passthrough
    assert c2._dgrad_bn_ok and not c2.emit_stats and not getattr(c3, "_dgrad_bn_ok", False)
    lin = nn.Linear(4, 4)
    rl = nn.ReLU()
    i2 = nn.Input()
    g2 = nn.Graph(i2, rl(lin(i2)))
    fuse_for_training(g2)
    assert lin.fuse_relu and rl.passthrough
    i3 = nn.Input()
    l3 = nn.Linear(4, 4)
    g3 = nn.Graph(i3, [l3(i3)])
    fuse_for_training(g3)
    assert not l3.fuse_relu


def test_graph_training_fusion_residual_plan_is_exact_on_cpu():
    """The Graph residual plan (BN adds the shortcut + ReLU, the CAddTable passes through, the shortcut gradient
    comes from the BN's masked output gradient, downsample BNs reordered after their shortcut) computes the same
    fp32 forward and gradients as the unfused graph; unfuse restores the order."""
    import copy

    import torch

    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNetGraph
    from bigdl_amd.nn.fusion import fuse_for_training, unfuse
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(3)
    base = ResNetGraph(10, 20, dataSet=DatasetType.CIFAR10)
    torch.manual_seed(0)
    x, y = torch.randn(4, 3, 32, 32), torch.randint(1, 11, (4,)).float()
    res = []
    for fused in (False, True):
        m = copy.deepcopy(base)
        if fused:
            order = list(m.order)
            fuse_for_training(m)
            assert sum(getattr(n, "pass_index", None) is not None for n in m.order) == 9
            assert m.order != order
        c = nn.CrossEntropyCriterion()
        o = m.forward(x)
        c.forward(o, y)
        gi = m.backward(x, c.backward(o, y))
        res.append((o.clone(), torch.cat([t.reshape(-1) for t in m.parameters()[1]]).clone()))
        if fused:
            unfuse(m)
            assert m.order == order and all(getattr(n, "pass_index", None) is None for n in m.order)
    assert torch.allclose(res[0][0], res[1][0], atol=1e-5)
    assert torch.allclose(res[0][1], res[1][1], atol=1e-5)
