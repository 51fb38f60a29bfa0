"""bigdl_amd — an MI355X-native distributed deep-learning framework with BigDL's capabilities.

Numeric backend: hand-written gfx950 HIP kernels (bigdl_amd/_C, sources in csrc/). Distribution:
one process per GPU with torch.distributed over RCCL/xGMI. API: BigDL-style nn modules
(forward/backward/updateOutput/updateGradInput/accGradParameters), criterions, optim methods,
Optimizer/DistriOptimizer, DataSet/Transformer pipeline, model persistence and Caffe/Torch loaders.
"""
__version__ = "0.1.0"
