"""Which part of a failed HIP-graph capture changes the Optimizer's training (tests/test_optimizer_graph_gpu.py
test_failed_capture_rolls_back_schedule)? Variants of a GraphedTrainStep construction that raises:
  raise0  raise immediately (only the Optimizer's fallback runs: side_stream.reset())
  full    the real constructor with SegmentedGraph.record raising
  reset   only side_stream.reset(), then raise
  prolog  prologue + rollback (no stream changes), then raise"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_optimizer_graph_gpu import _run  # noqa: E402

from bigdl_amd.ops import side_stream  # noqa: E402
from bigdl_amd.optim import graphed  # noqa: E402
from bigdl_amd.parallel import graph_segments  # noqa: E402

orig_init, orig_record = graphed.GraphedTrainStep.__init__, graph_segments.SegmentedGraph.record
w_e, _, _, s_e = _run(False)
w_e2, _, _, _ = _run(False)
print("eager vs eager", float((w_e2 - w_e).norm() / w_e.norm()), flush=True)


def boom(*a, **k):
    raise RuntimeError("injected")


for v in sys.argv[1:] or ["raise0", "full", "reset", "prolog"]:
    if v == "raise0":
        graphed.GraphedTrainStep.__init__ = lambda self, *a, **k: boom()
    elif v == "full":
        graph_segments.SegmentedGraph.record = boom
    elif v == "reset":
        def init(self, *a, **k):
            side_stream.reset()
            boom()
        graphed.GraphedTrainStep.__init__ = init
    elif v == "prolog":
        def rec(self, fn):
            side_stream.set_enabled(True)
            boom()
        graph_segments.SegmentedGraph.record = rec
    w, g, _, s = _run(True)
    graphed.GraphedTrainStep.__init__, graph_segments.SegmentedGraph.record = orig_init, orig_record
    print(v, "captured", g, "sched", s, s_e, "rel", float((w - w_e).norm() / w_e.norm()), flush=True)
