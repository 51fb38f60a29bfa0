"""Segmented HIP-graph capture: a training step recorded as a chain of single-stream HIP graphs cut at every
collective launch / wait, with the RCCL calls themselves re-issued eagerly between the graph launches.

Why not one graph with the collectives inside: RCCL's stream would become a parallel branch of the captured graph,
and graphs with parallel branches replay wrong on this ROCm 7 stack when HIP spreads them over several hardware
queues. Localised in round 4 (profiles/r4_graph_queue_probe.txt, tests/graph_fork_cases.py): the training step as
ONE graph with a side-stream branch that runs any kernel beside the backward kernels diverges (1.5e-3 at the default
queue count, 5.2 with 4 queues, NaN with 2) although the captured topology is right — the hipGraphDebugDotPrint dump
orders every update kernel after the last backward kernel and marks every cross-queue source as signalling — and is
exact with DEBUG_HIP_FORCE_GRAPH_QUEUES=1 or serialised kernels. Hence (a) bigdl_amd sets that variable before the
HIP runtime starts (bigdl_amd/__init__.py), and (b) captures are single-stream: GraphedTrainStep records with the
weight-gradient side stream off, and collectives cut the graph here.
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
_DOT_DIR = __import__("os").environ.get("BIGDL_GRAPH_DOT", "")


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
        if _DOT_DIR:
            self._g.enable_debug_mode()
        # thread-local capture: collectives launched eagerly between segments stay in the process group's watchdog
        # list, and that thread's event queries are illegal under a process-wide ("global") capture — RCCL's watchdog
        # then aborts the job (hipErrorStreamCaptureUnsupported). Only this thread's calls are restricted.
        self._g.capture_begin(pool=self.pool, capture_error_mode="thread_local")

    def _end(self):
        g = self._g
        self._g = None
        g.capture_end()
        if _DOT_DIR:       # BIGDL_GRAPH_DOT=dir: the captured topology (hipGraphDebugDotPrint), one file per segment
            import os

            os.makedirs(_DOT_DIR, exist_ok=True)
            g.debug_dump(os.path.join(_DOT_DIR, f"segment_{id(self) & 0xffff:04x}_{self.n_graphs}.dot"))
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
