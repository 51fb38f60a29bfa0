"""Optimizer.optimize() on the GPU: pinned double-buffered host->device feed + the iteration captured in HIP graphs
after two eager iterations must train exactly like the eager loop (reference DistriOptimizer iteration,
S/optim/DistriOptimizer.scala:185-418)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graph, iters=6, hook=None):
    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.dataset.core import DataSet, Sample
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.utils.engine import Engine
    from bigdl_amd.utils.random_generator import RNG

    Engine.setProperty("bigdl.optim.graph", "true" if graph else "false")
    RNG.setSeed(42)
    model = ResNet(10, 20, dataSet=DatasetType.CIFAR10)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(96, 3, 32, 32, generator=g)
    Y = torch.randint(1, 11, (96,), generator=g).float()
    ds = DataSet.array([Sample(X[i], Y[i]) for i in range(96)])
    opt = O.Optimizer(model, ds, nn.CrossEntropyCriterion(), batchSize=16,
                      optimMethod=O.SGD(0.05, momentum=0.9, dampening=0.0, learningRateDecay=0.01),
                      endTrigger=O.Trigger.maxIteration(iters))
    opt.device = torch.device("cuda:0")
    graphed = []
    def _hook(n):
        graphed.append(opt._graph is not None)
        if hook is not None:
            hook(opt)

    opt._iteration_hook = _hook
    # the dataset reshuffles from a random offset: pin it
    RNG.setSeed(7)
    m = opt.optimize()
    Engine.setProperty("bigdl.optim.graph", "true")
    w = m.getParameters()[0][:opt._step.total].detach().float().cpu().clone()
    meth = next(iter(opt.optimMethods.values()))
    return w, graphed, float(opt.state["Loss"]), (meth.state.get("evalCounter"), meth.learningRateSchedule.currentRate)


def _train_state(opt):
    """Every tensor an iteration reads and writes: fp32 master weights, their bf16 shadow, optimizer state buffers."""
    st = opt._step
    out = [st.w] + ([st.w16] if st.w16 is not None else [])
    for m in opt.optimMethods.values():
        for k in sorted(m.state.keys(), key=str):
            v = m.state[k]
            if torch.is_tensor(v) and v.is_floating_point() and v.numel() > 1:
                out.append(v)
    return out


def test_graphed_optimizer_matches_eager():
    """Lock-step: the eager run records the training state after every iteration; the graph run (2 eager warm-up
    iterations, then captured replays) is compared with it after every iteration and then reset to it, so each
    comparison covers exactly one iteration from identical state. (End-to-end trajectories of ANY two runs, eager or
    graph, separate by 5e-4..7e-3 after 6 iterations: fp32-atomic ordering in the parameter gradients flips the
    rare ReLU mask element within ~1e-8 of zero, profiles/r4_determinism.txt; one iteration from identical state
    differs by ~1e-9.)"""
    snaps = []
    w_e, g_e, l_e, s_e = _run(False, hook=lambda opt: snaps.append([t.detach().clone() for t in _train_state(opt)]))
    rels = []

    def lockstep(opt):
        cur = _train_state(opt)
        ref = snaps[len(rels)]
        assert len(cur) == len(ref)
        rels.append(max(((c.float() - r.float()).norm() / r.float().norm().clamp_min(1e-30)).item()
                        for c, r in zip(cur, ref)))
        for c, r in zip(cur, ref):
            c.copy_(r)

    w_g, g_g, l_g, s_g = _run(True, hook=lockstep)
    assert not any(g_e)
    assert g_g[:2] == [False, False] and all(g_g[2:]), g_g     # eager warm-up, then captured replays
    assert s_g == s_e, (s_g, s_e)                                 # same schedule position and rate
    print("per-iteration graph vs eager", rels)
    assert len(rels) == len(snaps) == 6
    assert max(rels) < 1e-5, rels
    assert abs(l_g - l_e) < 2e-2 * max(1.0, abs(l_e))


def test_failed_capture_rolls_back_schedule(monkeypatch):
    """A capture that raises leaves the Optimizer on eager iterations with the schedule exactly where an eager run
    has it: GraphedTrainStep undoes its prologue's schedule step and drops the device rate scalar (an SGD holding one
    skips its own schedule update)."""
    from bigdl_amd.parallel import graph_segments

    def boom(self, fn):
        raise RuntimeError("injected capture failure")

    snaps = []
    w_e, _, _, s_e = _run(False, hook=lambda opt: snaps.append([t.detach().clone() for t in _train_state(opt)]))
    monkeypatch.setattr(graph_segments.SegmentedGraph, "record", boom)
    rels = []

    def lockstep(opt):      # one iteration from identical state per comparison (see the test above)
        cur, ref = _train_state(opt), snaps[len(rels)]
        rels.append(max(((c.float() - r.float()).norm() / r.float().norm().clamp_min(1e-30)).item()
                        for c, r in zip(cur, ref)))
        for c, r in zip(cur, ref):
            c.copy_(r)

    w_f, g_f, _, s_f = _run(True, hook=lockstep)
    assert not any(g_f)
    assert s_f == s_e, (s_f, s_e)
    assert len(rels) == 6 and max(rels) < 1e-5, rels
