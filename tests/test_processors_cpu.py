"""ParameterProcessor clipping (reference ParameterOperations.scala), EvaluateMethods, MklInt8Convertible API."""
import torch

import bigdl_amd.nn as nn
from bigdl_amd.optim import EvaluateMethods
from bigdl_amd.parallel.processors import ConstantClippingProcessor, L2NormClippingProcessor


def test_constant_clipping():
    g = torch.tensor([3.0, -4.0, 0.5])
    ConstantClippingProcessor(-1, 2)(g)
    assert g.tolist() == [2.0, -1.0, 0.5]


def test_l2norm_clipping_scales_only_above_threshold():
    g = torch.tensor([3.0, -4.0])
    L2NormClippingProcessor(1.0)(g)
    assert torch.allclose(g, torch.tensor([0.6, -0.8]), atol=1e-5)
    g = torch.tensor([0.3, 0.4])
    L2NormClippingProcessor(1.0)(g)
    assert torch.allclose(g, torch.tensor([0.3, 0.4]))


def test_evaluate_methods():
    o = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1]])
    t = torch.tensor([2.0, 3.0])
    assert EvaluateMethods.calcAccuracy(o, t) == (1, 2)
    assert EvaluateMethods.calcTop5Accuracy(o, t) == (2, 2)
    assert EvaluateMethods.calcAccuracy(o[0], torch.tensor([2.0])) == (1, 1)


def test_int8_convertible_scales():
    m = nn.SpatialConvolution(3, 4, 3, 3)
    assert isinstance(m, nn.MklInt8Convertible)
    assert m.getWeightDimMask() == 1 and m.getInputDimMask() == 0
    ws = m.getWeightScales()[0]
    assert len(ws) == 4 and abs(ws[0] - float(m.weight[0].abs().max())) < 1e-6
    m.setInputScales([[2.5]])
    assert m.getInputScales() == [[2.5]]
    seq = nn.Sequential().add(nn.SpatialConvolution(3, 4, 3, 3)).add(nn.ReLU())
    seq.calcScales(torch.randn(2, 3, 8, 8))
    assert seq.modules[0].getInputScales()[0][0] > 0
    assert callable(nn.NNPrimitive.im2col)


def test_reference_named_entry_points(tmp_path):
    import bigdl_amd.dataset as D
    import bigdl_amd.optim as O
    from bigdl_amd.interop.tensorflow import BigDLToTensorflow, TensorflowLoader, TensorflowSaver, TensorflowToBigDL
    from bigdl_amd.utils.serializer import ModuleLoader, ModulePersister

    assert issubclass(D.ArrayTensorMiniBatch, D.MiniBatch) and O.AbstractOptimizer is O.Optimizer
    assert TensorflowToBigDL is TensorflowLoader and BigDLToTensorflow is TensorflowSaver
    m = nn.Sequential().add(nn.Linear(3, 2))
    p = str(tmp_path / "m.bigdl")
    ModulePersister.saveToFile(p, None, m, True)
    x = torch.randn(2, 3)
    assert torch.allclose(ModuleLoader.loadFromFile(p).forward(x), m.forward(x))
