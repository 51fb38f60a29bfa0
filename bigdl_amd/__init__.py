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
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")
