"""Model zoo builders on the CPU engine: output shapes, parameter counts, graph == sequential equivalence
(reference T/models/*Spec: VggSpec, InceptionSpec, ResNetSpec graph-vs-module comparisons)."""
import pytest
import torch

from bigdl_amd import models as M
from bigdl_amd import nn
from bigdl_amd.utils.random_generator import RNG


def _nparams(m):
    return sum(w.numel() for w in m.parameters()[0])


@pytest.mark.parametrize("build,shape,out", [
    (lambda: M.VggForCifar10(10), (2, 3, 32, 32), (2, 10)),
    (lambda: M.Inception_v1_NoAuxClassifier(7), (1, 3, 224, 224), (1, 7)),
    (lambda: M.Inception_v1(7), (1, 3, 224, 224), (1, 21)),
    (lambda: M.Inception_v2_NoAuxClassifier(7), (2, 3, 224, 224), (2, 7)),
    (lambda: M.Inception_v2(7), (2, 3, 224, 224), (2, 21)),
    (lambda: M.Autoencoder(32), (2, 28, 28), (2, 784)),
    (lambda: M.SimpleRNN(4, 8, 5), (2, 3, 4), (2, 3, 5)),
    (lambda: M.LeNet5(10), (2, 28 * 28), (2, 10)),
], ids=["vgg_cifar", "inc_v1_noaux", "inc_v1", "inc_v2_noaux", "inc_v2", "autoenc", "simplernn", "lenet"])
def test_model_shapes(build, shape, out):
    m = build()
    assert tuple(m.forward(torch.randn(*shape)).shape) == out


def test_param_counts_match_reference_architectures():
    assert _nparams(M.Vgg_16(1000)) == 138357544
    assert _nparams(M.Vgg_19(1000)) == 143667240
    assert _nparams(M.Inception_v1_NoAuxClassifier(1000)) == 6998552


@pytest.mark.parametrize("seq_fn,graph_fn,shape", [
    (M.VggForCifar10, M.VggForCifar10Graph, (2, 3, 32, 32)),
    (M.Inception_v1_NoAuxClassifier, M.Inception_v1_NoAuxClassifierGraph, (1, 3, 224, 224)),
    (M.Autoencoder, M.AutoencoderGraph, (2, 28, 28)),
])
def test_graph_variant_equals_sequential(seq_fn, graph_fn, shape):
    RNG.setSeed(5)
    s = seq_fn(10) if seq_fn is not M.Autoencoder else seq_fn(16)
    g = graph_fn(10) if graph_fn is not M.AutoencoderGraph else graph_fn(16)
    ws, wg = s.getParameters()[0], g.getParameters()[0]
    assert ws.numel() == wg.numel()
    wg.copy_(ws)
    s.evaluate(), g.evaluate()
    x = torch.randn(*shape)
    assert torch.allclose(s.forward(x), g.forward(x), atol=1e-4)


def test_inception_v1_backward_runs():
    m = M.Inception_v1_NoAuxClassifier(5)
    x = torch.randn(2, 3, 224, 224)
    y = m.forward(x)
    crit = nn.ClassNLLCriterion()
    crit.forward(y, torch.tensor([1.0, 3.0]))
    g = m.backward(x, crit.backward(y, torch.tensor([1.0, 3.0])))
    assert g.shape == x.shape and torch.isfinite(g).all()


def test_fusion_plans_deferred_bn():
    """nn.fusion defers the apply pass of every BN + ReLU whose only reader is a 3x3 / stride-1 conv or the stem max
    pool (ResNet-50: BN1 of the 13 bottlenecks whose 3x3 has stride 1, and the stem BN); the others keep theirs."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.nn.fusion import fuse_for_training, unfuse

    from bigdl_amd.nn import fusion

    m = ResNet(1000, 50, dataSet=DatasetType.ImageNet)
    fuse_for_training(m)
    bns = [l for l in m.flattened_layers() if isinstance(l, nn.BatchNormalization)]
    assert len(bns) == 53 and sum(1 for l in bns if getattr(l, "_defer_ok", False)) == 1    # default: the stem BN
    saved = fusion.DEFER_LEVEL[0]
    fusion.DEFER_LEVEL[0] = 2
    try:
        fuse_for_training(m)
    finally:
        fusion.DEFER_LEVEL[0] = saved
    deferred = [l for l in bns if getattr(l, "_defer_ok", False)]
    assert len(deferred) == 14
    assert all(l.fuse_relu for l in deferred)
    unfuse(m)
    assert not any(getattr(l, "_defer_ok", False) for l in bns)


def test_graph_fusion_plans_deferred_bn():
    """The same deferral decided on a Graph's edges (ResNetGraph): 14 of the 53 BNs."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNetGraph
    from bigdl_amd.nn.fusion import fuse_for_training

    from bigdl_amd.nn import fusion

    g = ResNetGraph(1000, 50, dataSet=DatasetType.ImageNet)
    saved = fusion.DEFER_LEVEL[0]
    fusion.DEFER_LEVEL[0] = 2
    try:
        fuse_for_training(g)
    finally:
        fusion.DEFER_LEVEL[0] = saved
    bns = [l for l in g.flattened_layers() if isinstance(l, nn.BatchNormalization)]
    assert len(bns) == 53
    assert sum(1 for l in bns if getattr(l, "_defer_ok", False)) == 14
