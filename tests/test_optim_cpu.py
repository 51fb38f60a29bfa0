"""Optim methods, schedules, triggers, validation methods and the training runtimes on the CPU engine,
including the distributed (gloo, 2 ranks) equivalence with the local optimizer (reference
T/optim/DistriOptimizerSpec.scala:378 "be same compare to ref optimizer")."""
import math

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd import optim as O
from bigdl_amd.dataset.core import DataSet, MiniBatch, Sample
from bigdl_amd.utils.table import T


def quad_feval(x):
    # f = 0.5 * ||x - 1||^2
    return float(0.5 * ((x - 1) ** 2).sum()), (x - 1).clone()


def test_sgd_matches_reference_rule():
    x = torch.tensor([2.0, -1.0])
    sgd = O.SGD(learningRate=0.1, momentum=0.9, weightDecay=0.01)   # dampening defaults to momentum
    xr = x.clone()
    buf = None
    for it in range(4):
        sgd.optimize(quad_feval, x)
        d = (xr - 1) + 0.01 * xr
        buf = d.clone() if buf is None else 0.9 * buf + (1 - 0.9) * d
        xr = xr - 0.1 * buf
    assert torch.allclose(x, xr, atol=1e-6)


def test_sgd_nesterov_and_lr_decay():
    x = torch.tensor([3.0])
    sgd = O.SGD(learningRate=0.5, learningRateDecay=0.1, momentum=0.5, dampening=0.0, nesterov=True)
    xr, buf = x.clone(), None
    for n in range(3):
        sgd.optimize(quad_feval, x)
        clr = 0.5 / (1 + n * 0.1)
        d = xr - 1
        buf = d.clone() if buf is None else 0.5 * buf + d
        xr = xr - clr * (d + 0.5 * buf)
    assert torch.allclose(x, xr, atol=1e-6)


@pytest.mark.parametrize("sched,expect", [
    (O.Step(2, 0.5), [1, 1, 0.5, 0.5, 0.25]),
    (O.MultiStep([1, 3], 0.1), [1, 0.1, 0.1, 0.01, 0.01]),
    (O.Poly(1.0, 4), [1, 0.75, 0.5, 0.25, 0.0]),
    (O.Exponential(2, 0.5, True), [1, 1, 0.5, 0.5, 0.25]),
    (O.Warmup(0.5), [1, 1.5, 2.0, 2.5, 3.0]),
    (O.NaturalExp(1, 1.0), [1, math.exp(-1), math.exp(-2), math.exp(-3), math.exp(-4)]),
])
def test_lr_schedules(sched, expect):
    sgd = O.SGD(learningRate=1.0, learningRateSchedule=sched)
    got = []
    for _ in range(5):
        sgd.updateHyperParameter()
        got.append(-sgd.getLearningRate())
    assert all(abs(a - b) < 1e-9 for a, b in zip(got, expect)), got


def test_sequential_schedule_and_epoch_schedules():
    seq = O.SequentialSchedule(10).add(O.Warmup(0.1), 3).add(O.Poly(1.0, 10), 20)
    sgd = O.SGD(learningRate=1.0, learningRateSchedule=seq)
    lrs = []
    for _ in range(6):
        sgd.updateHyperParameter()
        lrs.append(-sgd.getLearningRate())
    assert lrs[:4] == pytest.approx([1.0, 1.1, 1.2, 1.3])
    sgd2 = O.SGD(learningRate=1.0, learningRateSchedule=O.EpochStep(1, 0.5))
    sgd2.state["epoch"] = 3
    sgd2.updateHyperParameter()
    assert -sgd2.getLearningRate() == pytest.approx(0.125)   # reference: gamma ^ (epoch / stepSize)


@pytest.mark.parametrize("method", [O.Adam(0.1), O.ParallelAdam(0.1), O.Adagrad(0.5), O.Adadelta(0.9, 1e-2),
                                    O.Adamax(0.1), O.RMSprop(0.05), O.Ftrl(0.5), O.LarsSGD(None, 1.0, 0.1)],
                         ids=lambda m: type(m).__name__)
def test_methods_minimize_quadratic(method):
    x = torch.tensor([3.0, -2.0, 0.5])
    f0 = quad_feval(x)[0]
    for _ in range(200):
        method.optimize(quad_feval, x)
    assert quad_feval(x)[0] < f0 * 0.2


def test_adam_matches_formula():
    x = torch.tensor([1.0, 2.0])
    a = O.Adam(0.01, beta1=0.9, beta2=0.99, Epsilon=1e-8)
    xr, m, v = x.clone(), torch.zeros(2), torch.zeros(2)
    for t in range(1, 4):
        a.optimize(quad_feval, x)
        g = xr - 1
        m = 0.9 * m + 0.1 * g
        v = 0.99 * v + 0.01 * g * g
        xr = xr - 0.01 * math.sqrt(1 - 0.99 ** t) / (1 - 0.9 ** t) * m / (v.sqrt() + 1e-8)
    assert torch.allclose(x, xr, atol=1e-6)


def test_lbfgs_solves_quadratic():
    x = torch.tensor([3.0, -2.0])
    O.LBFGS(maxIter=50).optimize(quad_feval, x)
    assert torch.allclose(x, torch.ones(2), atol=1e-3)


def test_triggers():
    st = {"epoch": 1, "neval": 1}
    assert not O.Trigger.maxEpoch(1)(st)
    st["epoch"] = 2
    assert O.Trigger.maxEpoch(1)(st)
    assert O.Trigger.maxIteration(5)({"neval": 6})
    assert O.Trigger.severalIteration(2)({"neval": 3})
    assert not O.Trigger.severalIteration(2)({"neval": 4})
    assert O.Trigger.minLoss(0.1)({"Loss": 0.05})
    assert O.Trigger.or_(O.Trigger.maxEpoch(10), O.Trigger.minLoss(0.1))({"epoch": 1, "Loss": 0.01})
    e = O.Trigger.everyEpoch()
    assert not e({"epoch": 1}) and not e({"epoch": 1}) and e({"epoch": 2})


def test_validation_methods():
    out = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1], [0.2, 0.3, 0.5]])
    tgt = torch.tensor([2.0, 1.0, 1.0])
    r = O.Top1Accuracy()(out, tgt)
    assert r.result() == (pytest.approx(2 / 3), 3)
    r2 = r + O.Top1Accuracy()(out, tgt)
    assert r2.result()[1] == 6
    assert O.Top5Accuracy()(out, tgt).result()[0] == 1.0
    assert O.MAE()(torch.ones(4), torch.zeros(4)).result()[0] == pytest.approx(1.0)
    l = O.Loss(nn.ClassNLLCriterion())(torch.log(out + 1e-6), tgt)
    assert l.result()[1] == 3
    auc = O.PrecisionRecallAUC()(torch.tensor([0.9, 0.8, 0.3, 0.1]), torch.tensor([1.0, 1.0, 0.0, 0.0]))
    assert auc.result()[0] == pytest.approx(1.0)


def _regression_data(n=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, 4, generator=g)
    W = torch.tensor([[1.0, -2.0, 0.5, 3.0]])
    Y = X @ W.t() + 0.3
    return [Sample(X[i], Y[i]) for i in range(n)]


def _mlp(seed=0):
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(seed)
    return nn.Sequential().add(nn.Linear(4, 8)).add(nn.Tanh()).add(nn.Linear(8, 1))


def test_local_optimizer_converges_and_validates(tmp_path):
    data = _regression_data()
    model = _mlp()
    opt = O.Optimizer(model, DataSet.array(data), nn.MSECriterion(), batchSize=16,
                      optimMethod=O.SGD(0.05, momentum=0.9, dampening=0.0),
                      endTrigger=O.Trigger.maxEpoch(30))
    assert isinstance(opt, O.LocalOptimizer)
    opt.setValidation(O.Trigger.everyEpoch(), DataSet.array(data, shuffle=False), [O.MAE()], 16)
    opt.setCheckpoint(str(tmp_path), O.Trigger.everyEpoch())
    opt.optimize()
    res = model.evaluate(DataSet.array(data, shuffle=False), [O.MAE()], 16)
    assert res[0][0].result()[0] < 0.5
    assert any(p.name.startswith("model") for p in tmp_path.iterdir())


def _distri_job(rank, world, data, seed, iters):
    import torch as _t
    from bigdl_amd import nn as _nn
    from bigdl_amd import optim as _O
    from bigdl_amd.dataset.core import DataSet as _DS
    from bigdl_amd.utils.engine import Engine

    Engine.setProperty("bigdl.compress", "fp32")     # exact equivalence needs the uncompressed exchange
    model = _mlp(seed)
    opt = _O.Optimizer(model, _DS.rdd(data, shuffle=False), _nn.MSECriterion(), batchSize=16,
                       optimMethod=_O.SGD(0.05, momentum=0.9, dampening=0.0),
                       endTrigger=_O.Trigger.maxIteration(iters))
    assert isinstance(opt, _O.DistriOptimizer)
    opt.optimize()
    w, _ = model.getParameters()
    return w[:model._flat_total].clone()


def test_distri_optimizer_equals_local_optimizer():
    from bigdl_amd.utils.testing import run_distributed

    data = _regression_data(64)
    res = run_distributed(_distri_job, 2, (data, 3, 6))
    assert torch.allclose(res[0], res[1])
    model = _mlp(3)
    opt = O.LocalOptimizer(model, DataSet.array(data, shuffle=False), nn.MSECriterion(), 16,
                           O.SGD(0.05, momentum=0.9, dampening=0.0), O.Trigger.maxIteration(6))
    opt.optimize()
    w, _ = model.getParameters()
    assert torch.allclose(res[0], w[:model._flat_total], atol=1e-5)


def test_gradient_clipping_and_predictor():
    data = _regression_data(32)
    model = _mlp()
    opt = O.LocalOptimizer(model, DataSet.array(data), nn.MSECriterion(), 8, O.SGD(0.01),
                           O.Trigger.maxIteration(3))
    opt.setGradientClippingByl2Norm(0.5)
    opt.setConstantGradientClipping(-0.1, 0.1)
    opt.optimize()
    x = torch.stack([s.feature() for s in data])
    p = O.Predictor(model, 8).predict(x)
    assert p.shape == (32, 1)
    cls = nn.Sequential().add(nn.Linear(4, 3)).add(nn.LogSoftMax())
    pc = O.Predictor(cls, 8).predictClass(x)
    assert pc.min() >= 1 and pc.max() <= 3


def test_prediction_service_bytes_roundtrip():
    from bigdl_amd.optim.predictor import deserialize_activity, serialize_activity

    model = _mlp()
    svc = O.PredictionService(model)
    x = torch.randn(3, 4)
    out = deserialize_activity(svc.predict(serialize_activity(x)))
    assert torch.allclose(out, model.forward(x), atol=1e-6)
    t = deserialize_activity(serialize_activity(T(torch.ones(2), torch.arange(3))))
    assert torch.equal(t[2], torch.arange(3))


def _pb_varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _pb_field(num, wire, payload):
    import struct

    if wire == 0:
        return _pb_varint(num << 3) + _pb_varint(payload)
    if wire == 2:
        return _pb_varint(num << 3 | 2) + _pb_varint(len(payload)) + payload
    raise ValueError(wire)


def _pb_packed_ints(num, vals):
    return _pb_field(num, 2, b"".join(_pb_varint(v) for v in vals))


def test_prediction_service_decodes_hand_built_attrvalue():
    """The bytes protocol is bigdl.proto's AttrValue (S/optim/PredictionService.scala:184-280): a message assembled
    here field by field (proto3 packed repeated fields, as the JVM writes them) decodes to the tensor / table, the
    service answers in the same encoding, and a malformed request gets the reference's STRING error Activity."""
    import struct

    from bigdl_amd.optim.predictor import deserialize_activity, serialize_activity

    vals = [0.5, -1.0, 2.0, 3.25, 4.0, -6.5]
    storage = (_pb_field(1, 0, 2) + _pb_field(2, 2, struct.pack("<6f", *vals)) + _pb_field(9, 0, 7))   # FLOAT
    tensor = (_pb_field(1, 0, 2) + _pb_packed_ints(2, [2, 3]) + _pb_packed_ints(3, [3, 1]) + _pb_field(4, 0, 1)
              + _pb_field(5, 0, 2) + _pb_field(6, 0, 6) + _pb_field(8, 2, storage) + _pb_field(9, 0, 6))
    attr = _pb_field(1, 0, 10) + _pb_field(10, 2, tensor)                 # dataType TENSOR, tensorValue
    t = deserialize_activity(attr)
    assert t.dtype == torch.float32 and torch.equal(t, torch.tensor(vals).view(2, 3))

    def scalar(dt, field, payload):                                      # a scalar key tensor of one element
        st = _pb_field(1, 0, dt) + payload
        return _pb_field(1, 0, dt) + _pb_field(5, 0, 0) + _pb_field(6, 0, 1) + _pb_field(7, 0, 1) + \
            _pb_field(4, 0, 1) + _pb_field(8, 2, st)
    is_prim = scalar(5, 4, _pb_field(4, 0, 1))                            # BOOL true (bool_data)
    key1 = scalar(0, 6, _pb_field(6, 0, 1))                               # INT32 1 (int_data)
    key2 = scalar(0, 6, _pb_field(6, 0, 2))
    arr = _pb_field(1, 0, 5) + _pb_field(2, 0, 10) + b"".join(_pb_field(10, 2, x) for x in (is_prim, key1, key2,
                                                                                           tensor, tensor))
    tab = deserialize_activity(_pb_field(1, 0, 15) + _pb_field(15, 2, arr))   # ARRAY_VALUE
    assert sorted(tab.keys()) == [1, 2] and torch.equal(tab[2], torch.tensor(vals).view(2, 3))
    # our encoding decodes back (tensor keys too) and the service speaks it
    model = _mlp()
    svc = O.PredictionService(model)
    x = torch.randn(3, 4)
    out = deserialize_activity(svc.predict(serialize_activity(x)))
    assert torch.allclose(out, model.forward(x), atol=1e-6)
    err = deserialize_activity(svc.predict(b"\x0a\xff\xff"))
    assert isinstance(err, str) and "DeSerialize Input" in err
    bad = deserialize_activity(svc.predict(serialize_activity(torch.randn(3, 7))))   # wrong width: forward fails
    assert isinstance(bad, str) and "running forward" in bad


def test_prediction_service_replica_pool_concurrent():
    from concurrent.futures import ThreadPoolExecutor

    model = _mlp()
    svc = O.PredictionService(model, numThreads=3)
    assert svc._pool.qsize() == 3
    replicas = [svc._pool.get() for _ in range(3)]
    for r in replicas:
        svc._pool.put(r)
    def first_weight(m):
        return [q for q in m.flattened_layers() if getattr(q, "weight", None) is not None][0].weight

    # replicas share the weight tensors, not copies
    assert all(first_weight(r[0]) is first_weight(model) for r in replicas)
    xs = [torch.randn(5, 4) for _ in range(12)]
    with ThreadPoolExecutor(4) as ex:
        outs = list(ex.map(svc.predict, xs))
    for x, o in zip(xs, outs):
        assert torch.allclose(o, model.forward(x), atol=1e-6)


def test_optim_method_save_load(tmp_path):
    sgd = O.SGD(0.1, momentum=0.9)
    x = torch.tensor([1.0, 2.0])
    sgd.optimize(quad_feval, x)
    p = str(tmp_path / "om")
    sgd.save(p)
    s2 = O.OptimMethod.load(p)
    assert isinstance(s2, O.SGD) and s2.learningRate == 0.1
    assert torch.equal(s2.state["dfdx"], sgd.state["dfdx"])
