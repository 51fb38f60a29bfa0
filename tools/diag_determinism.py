"""Run-to-run determinism of the Optimizer loop on the GPU (tests/test_optimizer_graph_gpu.py _run, eager): N eager
runs in one process, relative weight difference of each against the first. Run under different env settings
(BIGDL_WGRAD_STREAM=0, BIGDL_MAX_INFLIGHT=1, AMD_SERIALIZE_KERNEL=3, ...) to localise a nondeterministic path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_optimizer_graph_gpu import _run  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ws = [_run(False)[0] for _ in range(n)]
print(os.environ.get("DIAG_TAG", ""), "rel vs run 0:", [f"{float((w - ws[0]).norm() / ws[0].norm()):.2e}" for w in ws[1:]],
      "vs run 1:", [f"{float((w - ws[1]).norm() / ws[1].norm()):.2e}" for w in ws[2:]], flush=True)
