"""A training step captured once into HIP graphs and replayed (runtime counterpart of the reference's
per-iteration task launch, S/optim/DistriOptimizer.scala:204-396).

On one rank the whole iteration is ONE ``hipGraphLaunch``. With collectives the step is recorded as a chain of
single-stream graphs cut at every RCCL launch / wait (parallel/graph_segments.py): the collectives are re-issued
between the graph launches, so the bucketed reduce-scatter still overlaps backward and the deferred weight
all-gather still overlaps the next forward, while no captured graph ever forks onto RCCL's stream.

Capture rules this wrapper enforces:
  * warm-up steps run eagerly first (kernel plans, workspaces, momentum buffers and RCCL communicators are
    created outside the capture; the SGD "first step" branch is never captured);
  * the input batch lives in static device buffers: ``replay(x, y)`` copies the new batch into them;
  * the learning-rate schedule keeps advancing: every captured SGD reads its rate from a device scalar that
    ``replay`` refreshes on the host side of the graph (``SGD.graph_prologue``) — methods whose update
    depends on host values that change per step (Adam bias correction, LARS) are refused;
  * nothing in the step synchronises with the host (TrainStep guarantees it), so capture succeeds with the
    collectives inside.
"""
import warnings

import torch

from ..ops import side_stream as _side
from ..parallel.graph_segments import SegmentedGraph
from .sgd import SGD


def graphable(step):
    """Whether ``step`` can be captured: every update is a plain SGD (its only per-step host value, the rate, is
    published to a device scalar by ``graph_prologue``) and no parameter processor reads host values."""
    from ..parallel.processors import LarsProcessor

    return (all(type(p.method) is SGD for p in step.plan)
            and not any(isinstance(q, LarsProcessor) for q in step.processors))


class GraphedTrainStep:
    """``prewarmed=True``: the caller has already run eager iterations of ``step`` on batches of this shape
    (kernel plans, workspaces, momentum buffers and communicators exist), so nothing extra is executed: the
    constructor only captures, and the first ``replay`` runs the captured iteration (the Optimizer loop uses this
    so capturing changes no training step). Otherwise ``warmup`` eager steps on (x, y) and one more on the
    capture stream run first (bench)."""

    def __init__(self, step, x, y, warmup=2, prewarmed=False):
        self.step = step
        for p in step.plan:
            if type(p.method) is not SGD:
                raise TypeError(f"GraphedTrainStep: {type(p.method).__name__} updates depend on per-step host "
                                "values; use the eager TrainStep")
        self.x = x.clone()
        self.y = y.clone()
        if not prewarmed:
            for _ in range(max(warmup, 1)):
                step.step(self.x, self.y)
        torch.cuda.synchronize()
        methods, seen = [], set()
        for p in step.plan:
            if id(p.method) not in seen:
                seen.add(id(p.method))
                methods.append(p.method)
        self.methods = methods
        # what a failed capture must undo: the schedule position the prologue advanced, and the device rate scalar
        # (an SGD holding ``_lr_dev`` skips its own schedule update, so a stale one would freeze the rate)
        snap = [(m, {k: v for k, v in list(m.state.items()) if not torch.is_tensor(v)},
                 dict(vars(m.learningRateSchedule)) if hasattr(m, "learningRateSchedule") else None,
                 getattr(m, "_lr_dev", None)) for m in methods]
        try:
            for m in methods:
                if getattr(m, "_lr_dev", None) is None:
                    m._lr_dev = torch.zeros(1, device=step.device)
            self._prologue()
            if not prewarmed:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):          # one more eager step on the capture stream (allocator warm-up)
                    step.step(self.x, self.y)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                self._prologue()
            self.graph = SegmentedGraph()
            # single-stream capture: the weight-gradient side stream (ops/side_stream.py) is off while recording, so
            # no captured graph has parallel branches. HIP's multi-queue graph executor was measured to break the
            # captured edges of such graphs (module docstring of parallel/graph_segments.py).
            was = _side.enabled()
            _side.set_enabled(False)
            try:
                with warnings.catch_warnings():
                    warnings.filterwarnings("ignore", message=".*CUDA Graph is empty.*")
                    self.loss = self.graph.record(lambda: step.step(self.x, self.y))
            finally:
                _side.set_enabled(was)
        except BaseException:
            for m, st, sched, lr in snap:
                for k in [k for k, v in list(m.state.items()) if k not in st and not torch.is_tensor(v)]:
                    del m.state[k]             # counters the prologue created
                for k, v in st.items():
                    m.state[k] = v
                if sched is not None:
                    vars(m.learningRateSchedule).update(sched)
                m._lr_dev = lr
            _side.reset()
            raise
        self._fresh = True                  # capture did not execute: the first replay uses this prologue

    def _prologue(self):
        for m in self.methods:
            m.graph_prologue()

    def replay(self, x=None, y=None):
        if x is not None:
            self.x.copy_(x, non_blocking=True)
        if y is not None:
            self.y.copy_(y, non_blocking=True)
        if not self._fresh:
            self._prologue()
        self._fresh = False
        self.graph.replay()
        return self.loss

    def matches(self, x, y):
        return (tuple(x.shape) == tuple(self.x.shape) and x.dtype == self.x.dtype
                and tuple(y.shape) == tuple(self.y.shape) and y.dtype == self.y.dtype)

    def eager(self, x, y):
        """One eager iteration while the captured methods read their rate from the device scalar (a batch whose
        shape differs from the captured one)."""
        if not self._fresh:
            self._prologue()
        self._fresh = False
        return self.step.step(x, y)

    def release(self):
        for m in self.methods:
            m._lr_dev = None
        self.graph = None
        self.x = self.y = self.loss = None     # static buffers live in the graph pool
