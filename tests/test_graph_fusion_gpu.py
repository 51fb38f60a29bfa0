"""Graph-form inference fusion on the GPU engine (nn.fusion.fuse_graph_for_inference, IRToDnn.fuse): Caffe-style
conv -> BatchNorm -> Scale -> ReLU chains fold into the conv, residual adds (+ReLU) run in the conv epilogue, and
channel concats are written in place by their producer convs. Numerics vs the fp32 CPU graph."""
import copy
import os
import tempfile

import pytest
import torch

from bigdl_amd import nn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _bn_scale(c, seed):
    g = torch.Generator().manual_seed(seed)
    bn = nn.SpatialBatchNormalization(c, 1e-5, affine=False)
    bn.runningMean.copy_(torch.randn(c, generator=g) * 0.1)
    bn.runningVar.copy_(torch.rand(c, generator=g) + 0.5)
    sc = nn.Scale([1, c, 1, 1])
    sc.weight.data.copy_((torch.rand(c, generator=g) + 0.5).view(1, c, 1, 1))
    sc.bias.data.copy_((torch.randn(c, generator=g) * 0.1).view(1, c, 1, 1))
    return bn, sc


def _inception_residual_graph():
    torch.manual_seed(0)
    inp = nn.Input()
    c1 = nn.SpatialConvolution(3, 32, 3, 3, 1, 1, 1, 1)(inp)
    b1, s1 = _bn_scale(32, 1)
    x = nn.ReLU()(s1(b1(c1)))
    a = nn.ReLU()(nn.SpatialConvolution(32, 32, 1, 1)(x))                  # concat producer through a ReLU
    cb = nn.SpatialConvolution(32, 16, 3, 3, 1, 1, 1, 1)(x)
    b2, s2 = _bn_scale(16, 2)
    b = s2(b2(cb))                                                           # producer after BN+Scale folding
    p = nn.SpatialMaxPooling(3, 3, 1, 1, 1, 1)(x)                           # non-conv input (copied)
    j = nn.JoinTable(2, 0)(a, b, p)                                          # 32 + 16 + 32 = 80 channels
    main = nn.SpatialConvolution(80, 64, 3, 3, 1, 1, 1, 1)(j)
    b3, s3 = _bn_scale(64, 3)
    main = s3(b3(main))
    short = nn.SpatialConvolution(80, 64, 1, 1)(j)
    y = nn.ReLU()(nn.CAddTable()(main, short))                               # residual + ReLU in the epilogue
    out = nn.SpatialAveragePooling(8, 8, 8, 8)(y)
    g = nn.Graph([inp], [out])
    g.evaluate()
    return g


def test_graph_fusion_matches_fp32_and_fires():
    from bigdl_amd.nn.table_ops import CAddTable, JoinTable
    from bigdl_amd.utils.intermediate import ConversionUtils

    g = _inception_residual_graph()
    x = torch.randn(4, 3, 16, 16)
    ref = g.forward(x).clone()
    dev = torch.device("cuda:0")
    fused = ConversionUtils.convert(g, "dnn", device=dev, train=False)
    # Scale / BN layers folded away (no Scale or BN module left in the lowered graph)
    names = [type(n.element).__name__ for n in fused.order]
    assert "Scale" not in names and "SpatialBatchNormalization" not in names, names
    y = fused.forward(x.to(dev))
    assert _rel(y, ref) < 3e-2
    add = [n.element for n in fused.order if isinstance(n.element, CAddTable)][0]
    assert add.passthrough, "residual add did not run in the conv epilogue"
    join_n = [n for n in fused.order if isinstance(n.element, JoinTable)][0]
    jo = fused._outs[join_n.id]
    # the concat's conv producers wrote into the JoinTable output buffer (same storage)
    prod = [p for p in join_n.prevs if type(p.element).__name__ in ("ReLU", "SpatialConvolution")]
    assert prod and all(fused._outs[p.id].data_ptr() != 0 and
                        fused._outs[p.id].untyped_storage().data_ptr() == jo.untyped_storage().data_ptr() for p in prod)
    y2 = fused.forward(x.to(dev))         # second call: fresh buffers, same result
    assert _rel(y2, y) < 1e-6


def test_caffe_roundtrip_resnet_block_fuses(tmp_path):
    """A Caffe-exported residual model (BatchNorm + Scale layers) reloads as a Graph that fuses like the native
    model: same output as the fp32 CPU model."""
    from bigdl_amd.nn.module import Module
    from bigdl_amd.utils.intermediate import ConversionUtils

    g = _inception_residual_graph()
    x = torch.randn(2, 3, 16, 16)
    ref = g.forward(x).clone()
    proto, weights = str(tmp_path / "m.prototxt"), str(tmp_path / "m.caffemodel")
    g.saveCaffe(proto, weights, overwrite=True)
    m = Module.loadCaffeModel(proto, weights)
    m.evaluate()
    fused = ConversionUtils.convert(m, "dnn", device=torch.device("cuda:0"), train=False)
    names = [type(n.element).__name__ for n in fused.order]
    assert "Scale" not in names, names
    y = fused.forward(x.cuda())
    assert _rel(y, ref) < 3e-2


def test_resnet_graph_training_fusion_matches_unfused(monkeypatch):
    """Training fusion of a Graph-form model (nn.fusion._fuse_graph_training on ResNet.graph): conv -> BN statistics
    epilogue, BN -> ReLU, BN -> ReLU -> conv dgrad-epilogue BN reduction, the residual add + ReLU inside the last BN
    and the fan-out gradient sum in the next conv's dgrad epilogue fire on the graph's edges and stay as close to
    the fp32 CPU graph as the unfused graph with the same bf16 kernels."""
    from bigdl_amd.models.resnet import DatasetType, ResNetGraph
    from bigdl_amd.nn.fusion import fuse_for_training
    from bigdl_amd.ops import native
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(5)
    cpu = ResNetGraph(10, 20, dataSet=DatasetType.CIFAR10)
    torch.manual_seed(0)
    x = torch.randn(16, 3, 32, 32).to(torch.bfloat16).float()
    y = torch.randint(1, 11, (16,)).float()
    C_ = native.get()
    real = C_.bn_bwd_reduce
    calls = []

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)

    monkeypatch.setattr(C_, "bn_bwd_reduce", counting)
    res = {}
    for fused in (False, True):
        m = copy.deepcopy(cpu).to("cuda")
        if fused:
            fuse_for_training(m)
            L = m.flattened_layers()
            assert sum(getattr(q, "emit_stats", False) for q in L) == 21
            assert sum(getattr(q, "_dgrad_bn_ok", False) for q in L) == 9
            assert sum(getattr(n, "pass_index", None) is not None for n in m.order) == 9
            assert sum(getattr(n, "fold_fanout", False) for n in m.order) == 9
        calls.clear()
        crit = nn.CrossEntropyCriterion()
        out = m.forward(x.cuda())
        crit.forward(out, y.cuda())
        m.backward(x.cuda(), crit.backward(out, y.cuda()))
        torch.cuda.synchronize()
        grads = torch.cat([t.float().cpu().reshape(-1) for t in m.parameters()[1]])
        res[fused] = (out.float().cpu(), grads, len(calls))
    # 21 BNs; 9 reduce in the dgrad epilogue of the conv after BN->ReLU, 9 (stem + residual BNs) in the epilogue of
    # the next block's first conv, which also sums the shortcut gradient (fan-out fold); the 2 shortcut BNs remain
    assert res[False][2] == 21 and res[True][2] == 3, (res[False][2], res[True][2])
    assert _rel(res[True][0], res[False][0]) < 2e-2
    crit = nn.CrossEntropyCriterion()
    oc = cpu.forward(x)
    crit.forward(oc, y)
    cpu.backward(x, crit.backward(oc, y))
    gc = torch.cat([t.reshape(-1) for t in cpu.parameters()[1]])
    # bf16 through 20 batch-16 BN layers drifts ~0.27 from fp32 with or without fusion (tools/diag_graph_fusion.py:
    # Sequential and Graph, fused and unfused, all 0.27-0.28); fusion only moves rounding points, so it must not
    # be further from fp32 than the unfused graph
    e_f, e_u = _rel(res[True][1], gc), _rel(res[False][1], gc)
    assert e_f < 1.15 * e_u + 1e-2, (e_f, e_u)
    cos = float(torch.nn.functional.cosine_similarity(res[True][1], gc, dim=0))
    assert cos > 0.9, cos
