"""Segmented HIP-graph capture: a training step recorded as a chain of single-stream HIP graphs cut at every
collective launch / wait, with the RCCL calls themselves re-issued eagerly between the graph launches.

Why not one graph with the collectives inside: a capture that forks onto RCCL's stream (async reduce-scatter in
flight while the next layers' backward kernels are captured on the compute stream) replays with wrong results on
this ROCm 7.0 / PyTorch 2.10 stack. Localised by ``tools/diag_fork_graph.py`` (1 rank, the training step as ONE
graph, the reduce-scatter replaced by a side-stream branch; weights after 3 replays vs 6 eager steps):
  * pure PyTorch chains with a forked branch, joined at the end or in the middle of the chain: exact;
  * the training step with a branch that launches NO kernel (fork + join only): exact (fp32-atomic noise, 7e-9);
  * the same branch forked only after the last backward kernel (no backward kernel beside it): exact;
  * a branch with ANY kernel (even ``mul_`` on a tensor the step never touches) beside the backward kernels:
    max |dw| 1.5e-3 on 99.9 % of the weights, the same value on every run (deterministic, not a timing race);
    the same with every memset node replaced by a kernel, and with record_stream on the branch's tensors;
  * eager execution with the same overlapping side-stream kernel: exact (tools/diag_overlap.py eager_ov_fake).
So the fault needs a graph with parallel branches whose kernel nodes are this step's kernels (large-kernarg
implicit-GEMM / BN kernels from our code object) — it is not a data race in those kernels (eager overlap is
exact) nor allocator reuse (the branch touches a pre-capture tensor); we could not reduce it to pure PyTorch.
Round 3 (profiles/r3_fork_graph_diag.txt): with the weight gradients on their own side stream (ops/side_stream.py,
the default) every variant above is exact in ONE graph (tests/test_distributed_gpu.py::
test_one_graph_step_with_forked_branches_matches_eager); with BIGDL_WGRAD_STREAM=0 it still diverges, and the
divergence changes from run to run (1.5e-3, nan), so it is a race rather than a deterministic miscompute. A self-join
of the compute stream just before the fork, forking through a kernel-less hop stream, or the weight-gradient kernel
without its split-K workspace do not remove it. The segmented form stays the multi-rank capture path (it needs no
assumption about which configuration is safe).
Cutting the step at the collectives keeps every captured graph a single stream; overlap still happens because a
collective issued between two graph launches runs on RCCL's stream while the next graph runs on the compute
stream.

Replay cost is one ``hipGraphLaunch`` per segment plus the eager collective calls (a few µs each, all async): for
ResNet-50 with 8M-element buckets that is ~15 launches per step instead of ~1,400 kernel launches.

Usage (optim/graphed.py): ``rec = SegmentedGraph(); rec.record(lambda: step.step(x, y))``; code on the step's
path announces collective boundaries with ``boundary(fn)`` / ``issue(fn)`` (no-ops outside a recording).
"""
import torch

from ..ops import side_stream as _side

_ACTIVE = None


def active():
    """The recorder currently capturing, or None."""
    return _ACTIVE


def boundary(fn):
    """Run ``fn`` (a host-issued collective launch or stream wait). Inside a recording the current graph segment
    is closed first, ``fn`` runs eagerly and is kept for replay, and a new segment is opened."""
    rec = _ACTIVE
    if rec is None:
        return fn()
    return rec.boundary(fn)


class _Cell:
    """Handle of a collective issued through ``issue`` during a recording: replays re-issue the collective and
    store the fresh work object here, so a recorded ``wait`` always waits for the current step's collective."""

    def __init__(self):
        self.h = None

    def wait(self):
        boundary(lambda: _raw_wait(self.h))
        return True

    def is_completed(self):
        return False


def _raw_wait(h):
    if h is not None:
        h.wait()


def issue(fn):
    """Launch a collective: ``fn()`` returns a work handle (or None). Inside a recording the launch becomes a
    replayed boundary and a ``_Cell`` proxy is returned."""
    rec = _ACTIVE
    if rec is None:
        return fn()
    cell = _Cell()

    def run():
        cell.h = fn()

    rec.boundary(run)
    return cell


class SegmentedGraph:
    def __init__(self):
        self.items = []          # ("g", CUDAGraph) | ("f", callable)
        self.pool = None
        self._g = None
        self.n_graphs = 0
        self.n_calls = 0

    # ------------------------------------------------------------------ recording
    def _begin(self):
        self._g = torch.cuda.CUDAGraph()
        self._g.capture_begin(pool=self.pool)

    def _end(self):
        g = self._g
        self._g = None
        g.capture_end()
        self.items.append(("g", g))
        self.n_graphs += 1

    def boundary(self, fn):
        _side.join()        # a segment ends with every side-stream fork joined (ops/side_stream.py)
        self._end()
        try:
            out = fn()
        finally:
            self.items.append(("f", fn))
            self.n_calls += 1
            self._begin()
        return out

    def record(self, fn):
        """Record ``fn()`` (one training step) on a private capture stream; returns its result (tensors in the
        graphs' pool, refreshed by every replay)."""
        global _ACTIVE
        if _ACTIVE is not None:
            raise RuntimeError("nested segmented capture")
        torch.cuda.synchronize()
        self.pool = torch.cuda.graph_pool_handle()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            _ACTIVE = self
            try:
                self._begin()
                out = fn()
                self._end()
            except BaseException:
                if self._g is not None:
                    try:
                        self._g.capture_end()
                    except Exception:  # noqa: BLE001 - the original error is the one to report
                        pass
                    self._g = None
                raise
            finally:
                _ACTIVE = None
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        return out

    # ------------------------------------------------------------------ replay
    def replay(self):
        for kind, x in self.items:
            if kind == "g":
                x.replay()
            else:
                x()

    def __len__(self):
        return len(self.items)
