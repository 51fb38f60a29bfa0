"""bigdl_amd — an MI355X-native distributed deep-learning framework with BigDL's capabilities.

Numeric backend: hand-written gfx950 HIP kernels (bigdl_amd/_C, sources in csrc/). Distribution:
one process per GPU with torch.distributed over RCCL/xGMI. API: BigDL-style nn modules
(forward/backward/updateOutput/updateGradInput/accGradParameters), criterions, optim methods,
Optimizer/DistriOptimizer, DataSet/Transformer pipeline, model persistence and Caffe/Torch loaders.
"""
import os as _os

__version__ = "0.1.0"

# HIP graphs with parallel branches replay wrong on this ROCm 7 stack when the runtime spreads them over several
# hardware queues: tools/diag_fork_graph.py variant B (a correctly captured topology — checked node by node in the
# hipGraphDebugDotPrint dump with tools/graph_dot_check.py) diverges by 1.5e-3 at the default queue count, 5.2 with 4
# queues and NaN with 2, and is exact with one queue or serialised kernels (profiles/r4_graph_queue_probe.txt).
# One queue executes every graph in topological order. Set before the HIP runtime initialises (first GPU call);
# an explicit setting in the environment wins.
import sys as _sys

_GQ_PRESET = _os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES")
_torch_mod = _sys.modules.get("torch")
# the HIP runtime reads the variable when it initialises: if torch already started it, setting it now has no effect
_HIP_STARTED = bool(_torch_mod is not None and getattr(getattr(_torch_mod, "cuda", None), "is_initialized",
                                                        lambda: False)())
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")
# True when graph replays are known to run on one hardware queue in captured order: either the variable was "1"
# before the process started HIP, or bigdl_amd set it before HIP initialised. When False, forked (multi-stream)
# captures are disabled (ops/side_stream.py: no side-stream fork inside a capture).
GRAPH_ONE_QUEUE = (_GQ_PRESET == "1") or (_GQ_PRESET is None and not _HIP_STARTED)
if not GRAPH_ONE_QUEUE:
    import warnings as _warnings

    _warnings.warn("bigdl_amd: DEBUG_HIP_FORCE_GRAPH_QUEUES=1 did not take effect (HIP was initialised before "
                   "`import bigdl_amd`, or the variable is set to another value): HIP-graph captures stay "
                   "single-stream (no side-stream forks inside a capture)", RuntimeWarning, stacklevel=2)


def graph_one_queue():
    """Whether forked HIP-graph captures are safe in this process (see GRAPH_ONE_QUEUE)."""
    return GRAPH_ONE_QUEUE
