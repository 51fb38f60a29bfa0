"""Device-timed phases of a training iteration (HIP events on the compute stream).

Reference: DistriOptimizer's per-iteration metrics (S/optim/DistriOptimizer.scala:188-196 — "computing time average",
"aggregate gradient time", "get weights average", "put gradient", "send weights average"; S/optim/Metrics.scala).
There they are host wall-clock times of Spark tasks; here every phase is GPU work, so it is measured with events the
compute stream executes:

  computing time (device)   forward + criterion + backward on the compute stream, all-gather waits excluded
  aggregate gradient time   the compute stream blocked on reduce-scatters (the exposed part of the gradient exchange)
  get weights time          the compute stream blocked on weight all-gathers (exposed weight distribution)
  update time (device)      the sharded optimizer update (and processors) after backward, waits excluded
  step time (device)        first forward kernel to last update kernel

A wait is timed with an event just before and just after ``work.wait()``: nothing else runs on the compute stream in
between, so the difference is exactly the time the stream stalled for the collective (0 when it had already landed:
fully hidden behind backward). Steps are resolved once their last event has completed (TrainStep.throttle), so timing
adds no host synchronisation; inside a HIP-graph capture nothing is recorded.
"""
import collections
import contextlib

import torch


class PhaseTimer:
    KEEP = 64

    def __init__(self, enabled=True):
        self.enabled = enabled
        self._cur = None
        self._pending = collections.deque()
        self.history = collections.deque(maxlen=self.KEEP)

    def _active(self):
        return (self.enabled and torch.cuda.is_available() and torch.cuda.is_initialized()
                and not torch.cuda.is_current_stream_capturing())

    @staticmethod
    def _event():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def begin_step(self):
        self._cur = {"t0": self._event(), "spans": []} if self._active() else None

    def mark(self, name):
        if self._cur is not None and self._active():
            self._cur[name] = self._event()

    @contextlib.contextmanager
    def span(self, name, on=True):
        """Time the enclosed launches / waits on the compute stream (a collective wait: its exposed stall)."""
        if not on or self._cur is None or not self._active():
            yield
            return
        a = self._event()
        try:
            yield
        finally:
            self._cur["spans"].append((name, a, self._event()))

    def end_step(self):
        if self._cur is None or not self._active():
            self._cur = None
            return
        self._cur["end"] = self._event()
        self._pending.append(self._cur)
        self._cur = None

    def collect(self, block=False):
        """Resolve finished steps (all of them with ``block``); returns their phase dicts (ms)."""
        out = []
        while self._pending:
            st = self._pending[0]
            if not block and not st["end"].query():
                break
            self._pending.popleft()
            st["end"].synchronize()
            t0 = st["t0"]
            tot = t0.elapsed_time(st["end"])
            waits = collections.defaultdict(float)
            for name, a, b in st["spans"]:
                waits[name] += a.elapsed_time(b)
            bwd = st.get("bwd")
            fb = t0.elapsed_time(bwd) if bwd is not None else tot
            ag_fwd = sum(a.elapsed_time(b) for name, a, b in st["spans"]
                         if name == "ag" and (bwd is None or t0.elapsed_time(a) <= fb))
            d = {"step_ms": tot, "compute_ms": max(0.0, fb - ag_fwd), "rs_wait_ms": waits.get("rs", 0.0),
                 "ag_wait_ms": waits.get("ag", 0.0)}
            d["update_ms"] = max(0.0, tot - fb - d["rs_wait_ms"] - (d["ag_wait_ms"] - ag_fwd))
            d["comm_exposed_ms"] = d["rs_wait_ms"] + d["ag_wait_ms"]
            self.history.append(d)
            out.append(d)
        return out

    def summary(self, last=None):
        """Mean of every phase over the resolved steps (the last ``last`` of them), or None."""
        self.collect(block=True)
        hist = list(self.history)[-last:] if last else list(self.history)
        if not hist:
            return None
        keys = hist[0].keys()
        return {k: round(sum(h[k] for h in hist) / len(hist), 4) for k in keys} | {"steps": len(hist)}


METRIC_NAMES = {"compute_ms": "computing time (device)", "rs_wait_ms": "aggregate gradient time",
                "ag_wait_ms": "get weights time", "update_ms": "update time (device)", "step_ms": "step time (device)"}
