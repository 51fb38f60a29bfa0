"""CPU-engine layer tests: finite-difference gradient checks (reference T/nn/** + GradientChecker), containers,
graphs, 1-based dimension semantics, criterions."""
import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.utils.gradient_checker import GradientChecker
from bigdl_amd.utils.table import T, Table

torch.manual_seed(0)


def r(*s):
    return torch.randn(*s)


LAYERS = [
    ("Linear", lambda: nn.Linear(7, 5), lambda: r(3, 7)),
    ("SpatialConvolution", lambda: nn.SpatialConvolution(3, 4, 3, 3, 1, 1, 1, 1), lambda: r(2, 3, 6, 6)),
    ("SpatialConvolution-s2", lambda: nn.SpatialConvolution(3, 4, 3, 2, 2, 1, 0, 1), lambda: r(2, 3, 7, 6)),
    ("SpatialConvolution-g2", lambda: nn.SpatialConvolution(4, 6, 3, 3, 1, 1, 1, 1, nGroup=2), lambda: r(2, 4, 5, 5)),
    ("SpatialDilatedConvolution", lambda: nn.SpatialDilatedConvolution(2, 3, 3, 3, 1, 1, 2, 2, 2, 2), lambda: r(1, 2, 7, 7)),
    ("SpatialFullConvolution", lambda: nn.SpatialFullConvolution(3, 2, 3, 3, 2, 2, 1, 1), lambda: r(2, 3, 4, 4)),
    ("SpatialSeparableConvolution", lambda: nn.SpatialSeparableConvolution(2, 4, 2, 3, 3), lambda: r(1, 2, 5, 5)),
    ("VolumetricConvolution", lambda: nn.VolumetricConvolution(2, 3, 2, 2, 2), lambda: r(1, 2, 4, 4, 4)),
    ("TemporalConvolution", lambda: nn.TemporalConvolution(4, 3, 2), lambda: r(2, 5, 4)),
    ("LocallyConnected2D", lambda: nn.LocallyConnected2D(2, 5, 5, 3, 3, 3), lambda: r(2, 2, 5, 5)),
    ("SpatialMaxPooling", lambda: nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1), lambda: r(2, 3, 7, 7)),
    ("SpatialAveragePooling", lambda: nn.SpatialAveragePooling(3, 3, 2, 2, 1, 1), lambda: r(2, 3, 7, 7)),
    ("SpatialBatchNormalization", lambda: nn.SpatialBatchNormalization(3), lambda: r(4, 3, 3, 3)),
    ("BatchNormalization", lambda: nn.BatchNormalization(5), lambda: r(6, 5)),
    ("LayerNormalization", lambda: nn.LayerNormalization(6), lambda: r(3, 6)),
    ("SpatialCrossMapLRN", lambda: nn.SpatialCrossMapLRN(3, 1e-2, 0.75, 1.0), lambda: r(2, 5, 3, 3)),
    ("ReLU", lambda: nn.ReLU(), lambda: r(4, 5)),
    ("Tanh", lambda: nn.Tanh(), lambda: r(4, 5)),
    ("Sigmoid", lambda: nn.Sigmoid(), lambda: r(4, 5)),
    ("ELU", lambda: nn.ELU(), lambda: r(4, 5)),
    ("LeakyReLU", lambda: nn.LeakyReLU(0.1), lambda: r(4, 5)),
    ("PReLU", lambda: nn.PReLU(3), lambda: r(2, 3, 4)),
    ("SoftPlus", lambda: nn.SoftPlus(), lambda: r(4, 5)),
    ("SoftSign", lambda: nn.SoftSign(), lambda: r(4, 5)),
    ("LogSoftMax", lambda: nn.LogSoftMax(), lambda: r(4, 5)),
    ("SoftMax", lambda: nn.SoftMax(), lambda: r(4, 5)),
    ("HardTanh", lambda: nn.HardTanh(), lambda: r(4, 5) * 0.5),
    ("Power", lambda: nn.Power(2.0, 0.5, 2.0), lambda: r(4, 5)),
    ("CMul", lambda: nn.CMul([1, 5]), lambda: r(4, 5)),
    ("CAdd", lambda: nn.CAdd([1, 5]), lambda: r(4, 5)),
    ("Scale", lambda: nn.Scale([5]), lambda: r(4, 5)),
    ("Mul", lambda: nn.Mul(), lambda: r(4, 5)),
    ("Bilinear", lambda: nn.Bilinear(3, 4, 2), lambda: T(r(5, 3), r(5, 4))),
    ("Cosine", lambda: nn.Cosine(4, 3), lambda: r(5, 4)),
    ("Euclidean", lambda: nn.Euclidean(4, 3), lambda: r(5, 4)),
    ("Maxout", lambda: nn.Maxout(4, 3, 2), lambda: r(5, 4)),
    ("Highway", lambda: nn.Highway(4), lambda: r(5, 4)),
    ("Normalize", lambda: nn.Normalize(2.0), lambda: r(3, 4)),
    ("View", lambda: nn.View(12).setNumInputDims(2), lambda: r(2, 3, 4)),
    ("Reshape", lambda: nn.Reshape([12]), lambda: r(2, 3, 4)),
    ("Transpose", lambda: nn.Transpose([(2, 3)]), lambda: r(2, 3, 4)),
    ("Narrow", lambda: nn.Narrow(2, 2, 2), lambda: r(3, 5)),
    ("Select", lambda: nn.Select(2, 3), lambda: r(3, 5)),
    ("Squeeze", lambda: nn.Squeeze(2), lambda: r(3, 1, 4)),
    ("Unsqueeze", lambda: nn.Unsqueeze(2), lambda: r(3, 4)),
    ("Replicate", lambda: nn.Replicate(3), lambda: r(4)),
    ("Padding", lambda: nn.Padding(1, 2, 2), lambda: r(3, 4)),
    ("SpatialZeroPadding", lambda: nn.SpatialZeroPadding(1, 2, 0, 1), lambda: r(1, 2, 3, 3)),
    ("Sum", lambda: nn.Sum(2), lambda: r(3, 4)),
    ("Mean", lambda: nn.Mean(2), lambda: r(3, 4)),
    ("Max", lambda: nn.Max(2), lambda: r(3, 4)),
    ("UpSampling2D", lambda: nn.UpSampling2D([2, 2]), lambda: r(1, 2, 3, 3)),
    ("ResizeBilinear", lambda: nn.ResizeBilinear(5, 6), lambda: r(1, 2, 3, 3)),
    ("CAddTable", lambda: nn.CAddTable(), lambda: T(r(3, 4), r(3, 4))),
    ("CMulTable", lambda: nn.CMulTable(), lambda: T(r(3, 4), r(3, 4))),
    ("CSubTable", lambda: nn.CSubTable(), lambda: T(r(3, 4), r(3, 4))),
    ("CMaxTable", lambda: nn.CMaxTable(), lambda: T(r(3, 4), r(3, 4))),
    ("JoinTable", lambda: nn.JoinTable(2, 2), lambda: T(r(3, 4), r(3, 2))),
    ("MM", lambda: nn.MM(), lambda: T(r(2, 3, 4), r(2, 4, 5))),
    ("DotProduct", lambda: nn.DotProduct(), lambda: T(r(3, 4), r(3, 4))),
    ("PairwiseDistance", lambda: nn.PairwiseDistance(2), lambda: T(r(3, 4), r(3, 4))),
]


@pytest.mark.parametrize("name,mk,inp", LAYERS, ids=[l[0] for l in LAYERS])
def test_layer_gradients(name, mk, inp):
    from bigdl_amd.utils.random_generator import RNG

    torch.manual_seed(1)
    RNG.setSeed(1)
    m = mk()
    x = inp()
    gc = GradientChecker(1e-2, 3e-2)
    ok, worst = gc.checkLayer(m, x)
    assert ok, f"{name}: input-gradient error {worst}"
    if m.parameters() is not None and name not in ("SpatialBatchNormalization", "BatchNormalization"):
        ok, worst = gc.checkWeight(m, x)
        assert ok, f"{name}: weight-gradient error {worst}"


def test_linear_matches_formula():
    m = nn.Linear(4, 3)
    x = r(2, 4)
    y = m.forward(x)
    assert torch.allclose(y, x @ m.weight.t() + m.bias, atol=1e-6)


def test_sequential_and_concat_and_table_containers():
    seq = nn.Sequential().add(nn.Linear(4, 6)).add(nn.ReLU()).add(nn.Linear(6, 2))
    ct = nn.ConcatTable().add(nn.Identity()).add(nn.MulConstant(2.0))
    model = nn.Sequential().add(seq).add(ct).add(nn.CAddTable())
    x = r(3, 4)
    y = model.forward(x)
    assert torch.allclose(y, 3 * seq.output, atol=1e-6)
    g = model.backward(x, torch.ones(3, 2))
    assert g.shape == x.shape
    c = nn.Concat(2).add(nn.Linear(4, 2)).add(nn.Linear(4, 3))
    assert c.forward(x).shape == (3, 5)
    pt = nn.ParallelTable().add(nn.Linear(4, 2)).add(nn.Linear(3, 2))
    out = pt.forward(T(r(2, 4), r(2, 3)))
    assert out[1].shape == (2, 2) and out[2].shape == (2, 2)
    mt = nn.MapTable(nn.Linear(3, 2))
    o = mt.forward(T(r(2, 3), r(2, 3), r(2, 3)))
    assert o.length() == 3
    mt.backward(T(r(2, 3), r(2, 3), r(2, 3)), T(torch.ones(2, 2), torch.ones(2, 2), torch.ones(2, 2)))


def test_graph_matches_sequential():
    from bigdl_amd.models.lenet import LeNet5, LeNet5Graph

    torch.manual_seed(0)
    a = LeNet5(10)
    b = LeNet5Graph(10)
    pa, pb = a.parameters(), b.parameters()
    for wa, wb in zip(pa[0], pb[0]):
        wb.data.copy_(wa)
    x = r(4, 28 * 28)
    ya, yb = a.forward(x), b.forward(x)
    assert torch.allclose(ya, yb, atol=1e-5)
    ga = a.backward(x, torch.ones_like(ya))
    gb = b.backward(x, torch.ones_like(yb))
    assert torch.allclose(ga, gb, atol=1e-5)
    for g1, g2 in zip(pa[1], pb[1]):
        assert torch.allclose(g1, g2, atol=1e-5)


def test_graph_multi_input_output_and_stop_gradient():
    i1, i2 = nn.Input(), nn.Input()
    a = nn.Linear(3, 4).setName("a").inputs(i1)
    b = nn.Linear(2, 4).setName("b").inputs(i2)
    s = nn.CAddTable().inputs(a, b)
    o1 = nn.ReLU().inputs(s)
    o2 = nn.Tanh().inputs(s)
    g = nn.Graph([i1, i2], [o1, o2])
    out = g.forward(T(r(5, 3), r(5, 2)))
    assert out[1].shape == (5, 4) and out[2].shape == (5, 4)
    gi = g.backward(T(r(5, 3), r(5, 2)), T(torch.ones(5, 4), torch.ones(5, 4)))
    assert gi[1].shape == (5, 3) and gi[2].shape == (5, 2)
    g.stopGradient(["b"])


def test_one_based_dims():
    x = torch.arange(24.0).view(2, 3, 4)
    assert torch.equal(nn.Narrow(2, 2, 1).forward(x), x[:, 1:2, :])
    assert torch.equal(nn.Select(3, 1).forward(x), x[:, :, 0])
    assert torch.equal(nn.JoinTable(1).forward(T(x, x)), torch.cat([x, x], 0))
    st = nn.SplitTable(2).forward(x)
    assert st.length() == 3 and torch.equal(st[2], x[:, 1])


def test_table_semantics():
    t = T(1, 2, 3)
    assert t.length() == 3 and t[1] == 1
    t.insert(2, 9)
    assert t.toSeq() == [1, 9, 2, 3]
    assert t.remove(1) == 1 and t.length() == 3


CRITERIONS = [
    ("ClassNLL", nn.ClassNLLCriterion(), lambda: torch.log_softmax(r(4, 5), 1), lambda: torch.tensor([1., 3., 5., 2.])),
    ("CrossEntropy", nn.CrossEntropyCriterion(), lambda: r(4, 5), lambda: torch.tensor([1., 3., 5., 2.])),
    ("MSE", nn.MSECriterion(), lambda: r(4, 5), lambda: r(4, 5)),
    ("Abs", nn.AbsCriterion(), lambda: r(4, 5), lambda: r(4, 5)),
    ("SmoothL1", nn.SmoothL1Criterion(), lambda: r(4, 5), lambda: r(4, 5)),
    ("BCE", nn.BCECriterion(), lambda: torch.sigmoid(r(4, 5)), lambda: (r(4, 5) > 0).float()),
    ("Margin", nn.MarginCriterion(), lambda: r(4, 5), lambda: torch.sign(r(4, 5))),
    ("SoftMargin", nn.SoftMarginCriterion(), lambda: r(4, 5), lambda: torch.sign(r(4, 5))),
    ("MultiMargin", nn.MultiMarginCriterion(), lambda: r(4, 5), lambda: torch.tensor([1., 3., 5., 2.])),
    ("KLDiv", nn.DistKLDivCriterion(), lambda: torch.log_softmax(r(4, 5), 1), lambda: torch.softmax(r(4, 5), 1)),
    ("CosineEmbedding", nn.CosineEmbeddingCriterion(0.1), lambda: T(r(4, 5), r(4, 5)), lambda: torch.sign(r(4))),
]


@pytest.mark.parametrize("name,crit,inp,tgt", CRITERIONS, ids=[c[0] for c in CRITERIONS])
def test_criterion_gradient_is_numerical(name, crit, inp, tgt):
    torch.manual_seed(2)
    x, t = inp(), tgt()
    crit.forward(x, t)
    g = crit.backward(x, t)
    xs = [x] if isinstance(x, torch.Tensor) else x.toSeq()
    gs = [g] if isinstance(g, torch.Tensor) else g.toSeq()
    for xi, gi in zip(xs, gs):
        flat = xi.view(-1)
        for j in range(min(6, flat.numel())):
            o = flat[j].item()
            flat[j] = o + 1e-3
            lp = float(crit.forward(x, t))
            flat[j] = o - 1e-3
            lm = float(crit.forward(x, t))
            flat[j] = o
            num = (lp - lm) / 2e-3
            assert abs(num - gi.reshape(-1)[j].item()) < 2e-2 * max(1.0, abs(num)), (name, j)


def test_cross_entropy_equals_logsoftmax_nll():
    x = r(6, 7)
    t = torch.tensor([1., 2., 3., 7., 5., 6.])
    ce = nn.CrossEntropyCriterion().forward(x, t)
    nll = nn.ClassNLLCriterion().forward(torch.log_softmax(x, 1), t)
    assert abs(float(ce) - float(nll)) < 1e-5


def test_module_api_misc():
    m = nn.Sequential().add(nn.Linear(3, 4).setName("fc")).add(nn.ReLU())
    assert m["fc"] is m.modules[0]
    w, g = m.getParameters()
    assert w.numel() == 16 and g.numel() == 16
    m.modules[0].weight.data.fill_(0.5)
    assert torch.all(w[:12] == 0.5)  # parameters are views of the flat buffer
    m.freeze()
    x = torch.ones(2, 3)      # 0.5 * 3 + |bias| < 1 keeps every ReLU open
    m.forward(x)
    m.zeroGradParameters()
    m.backward(x, torch.ones(2, 4))
    assert float(g.abs().sum()) == 0.0
    m.unFreeze()
    m.backward(x, torch.ones(2, 4))
    assert float(g.abs().sum()) > 0
    times = m.getTimes()
    assert len(times) == 3
    c = m.cloneModule()
    assert torch.equal(c.modules[0].weight, m.modules[0].weight)
    m.evaluate()
    assert not m.modules[0].isTraining()


def test_regularizer_adds_decay():
    from bigdl_amd.optim.regularizer import L2Regularizer

    m = nn.Linear(3, 2, wRegularizer=L2Regularizer(0.1))
    x = r(4, 3)
    m.forward(x)
    m.zeroGradParameters()
    m.backward(x, torch.zeros(4, 2))
    assert torch.allclose(m.gradWeight, 0.1 * m.weight)


def test_time_distributed_criterion_flat_equals_per_step_loop():
    """The batched (B*T rows) fast path must equal the reference per-time-step loop (TimeDistributedCriterion.scala)."""
    torch.manual_seed(0)
    for inner in [nn.CrossEntropyCriterion(), nn.ClassNLLCriterion(), nn.MSECriterion(),
                  nn.CrossEntropyCriterion(sizeAverage=False)]:
        for sa in (True, False):
            x = torch.randn(3, 5, 7)
            y = torch.randn(3, 5, 7) if isinstance(inner, nn.MSECriterion) else torch.randint(1, 8, (3, 5)).float()
            if isinstance(inner, nn.ClassNLLCriterion):
                x = torch.log_softmax(x, -1)
            c = nn.TimeDistributedCriterion(inner, sa)
            loss, g = c.forward(x, y), c.backward(x, y)
            ref_l, ref_g = 0.0, []
            for t in range(5):
                ref_l = ref_l + inner.forward(x[:, t], y[:, t])
                ref_g.append(inner.backward(x[:, t], y[:, t]))
            ref_g = torch.stack(ref_g, 1)
            if sa:
                ref_l, ref_g = ref_l / 5, ref_g / 5
            assert abs(float(loss - ref_l)) < 1e-5 and torch.allclose(g, ref_g, atol=1e-6)


def test_class_simplex_criterion_embedding():
    from bigdl_amd.nn.criterion import ClassSimplexCriterion

    c = ClassSimplexCriterion(5)
    emb = c.simplex
    assert torch.allclose(emb.norm(dim=1), torch.ones(5, dtype=torch.float64))
    gram = emb @ emb.t()
    assert torch.allclose(gram[~torch.eye(5, dtype=torch.bool)], torch.full((20,), -0.25, dtype=torch.float64))
    x, y = torch.randn(3, 5), torch.tensor([1.0, 3.0, 5.0])
    loss = c.forward(x, y)
    assert abs(float(loss) - float(((x.double() - emb[y.long() - 1]) ** 2).mean())) < 1e-6
    assert c.backward(x, y).shape == x.shape


def test_nn_primitive_im2col_vol2col_match_conv():
    from bigdl_amd.nn import primitive as P

    torch.manual_seed(0)
    x, w = torch.randn(3, 7, 8), torch.randn(4, 3, 3, 3)
    cols = P.im2col(x, 3, 3, 2, 1, 1, 1)
    y = (w.reshape(4, -1) @ cols).reshape(4, P.out_size(7, 3, 1, 1), P.out_size(8, 3, 2, 1))
    assert torch.allclose(y, torch.nn.functional.conv2d(x[None], w, stride=(1, 2), padding=1)[0], atol=1e-5)
    r = torch.randn_like(cols)
    assert torch.allclose((cols * r).sum(), (x * P.col2im(r, 3, 7, 8, 3, 3, 2, 1, 1, 1)).sum(), atol=1e-4)
    v, wv = torch.randn(2, 4, 5, 6), torch.randn(5, 2, 2, 3, 3)
    cv = P.vol2col(v, 2, 3, 3, 1, 1, 1, 0, 1, 1)
    ref = torch.nn.functional.conv3d(v[None], wv, padding=(0, 1, 1))[0]
    assert torch.allclose((wv.reshape(5, -1) @ cv).reshape(ref.shape), ref, atol=1e-4)


def test_calc_scales_then_quantize_uses_static_ranges():
    m = nn.Sequential().add(nn.SpatialConvolution(3, 8, 3, 3)).add(nn.ReLU()).add(nn.View(8 * 6 * 6)) \
        .add(nn.Linear(288, 4))
    x = torch.randn(2, 3, 8, 8)
    m.calcScales(x)
    q = m.quantize()
    assert all(getattr(l, "inputAmax", None) is not None for l in q.flattened_layers()
               if "Quantized" in type(l).__name__)


def test_gemm_layer_matches_reference_formula():
    """nn.Gemm (ONNX Gemm, reference S/nn/onnx/Gemm.scala): alpha * op(A) op(B) + beta * C, constants or Table."""
    import torch as _t

    from bigdl_amd import nn as _nn
    from bigdl_amd.utils.table import T as _T

    g = _t.Generator().manual_seed(0)
    a, b, c = _t.randn(4, 3, generator=g), _t.randn(5, 3, generator=g), _t.randn(4, 5, generator=g)
    m = _nn.Gemm(0.5, 2.0, False, True, matrixB=b, matrixC=c)
    assert _t.allclose(m.forward(a), 0.5 * a @ b.t() + 2.0 * c, atol=1e-5)
    m2 = _nn.Gemm(1.0, 1.0, True, False)
    y = m2.forward(_T(a.t().contiguous(), b.t().contiguous(), c))
    assert _t.allclose(y, a @ b.t() + c, atol=1e-5)
    gi = m2.backward(_T(a.t().contiguous(), b.t().contiguous(), c), _t.ones(4, 5))
    assert gi[3].shape == c.shape


def test_compat_gemm_wrapper():
    from bigdl_amd.compat.nn.layer import Gemm

    assert Gemm(1.0, 1.0, False, False) is not None
