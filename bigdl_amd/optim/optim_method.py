"""OptimMethod base (reference S/optim/OptimMethod.scala:28-180).

``optimize(feval, x)`` takes a closure returning (loss, dfdx) and updates the flat parameter tensor ``x``
in place. On the GPU engine ``x`` / ``dfdx`` are the flat fp32 master buffers produced by
``AbstractModule.getParameters()`` and the update runs as ONE fused HIP kernel over the whole buffer
(or over this rank's ZeRO-1 shard), optionally writing the bf16 compute copy of the weights in the same
pass (``attach_shadow``).
"""
import copy

import torch

from ..utils.table import Table


class OptimMethod:
    def __init__(self):
        self.state = Table()
        self.state["epoch"] = 1
        self.state["neval"] = 1
        self._shadow16 = None

    def optimize(self, feval, parameter):
        raise NotImplementedError

    def attach_shadow(self, w16):
        """bf16 copy of ``parameter`` to be rewritten by the fused update kernel (GPU engine)."""
        self._shadow16 = w16
        return self

    def clearHistory(self):
        keep = {k: self.state.get(k) for k in ("epoch", "neval", "evalCounter", "recordsProcessedThisEpoch")}
        self.state = Table()
        for k, v in keep.items():
            if v is not None:
                self.state[k] = v
        return self

    def updateHyperParameter(self):
        pass

    def getHyperParameter(self):
        return ""

    def getLearningRate(self):
        return 0.0

    def loadFromTable(self, config):
        for k, v in config.items():
            if hasattr(self, k):
                setattr(self, k, v)
        return self

    def clone(self):
        c = copy.copy(self)
        c.state = self.state.clone()
        c._shadow16 = None
        return c

    def save(self, path, overWrite=False):
        """Persist this method (hyper-parameters, schedule, state table) as a safetensors file with a JSON
        structure header (utils/safe_state.py): nothing in the file is executed when it is loaded."""
        import os

        from ..utils import safe_state

        if os.path.exists(path) and not overWrite:
            raise FileExistsError(path)
        sh = self._shadow16
        self._shadow16 = None
        try:
            safe_state.save(self, path)
        finally:
            self._shadow16 = sh
        return self

    @staticmethod
    def load(path):
        """Load an OptimMethod saved by ``save``; only OptimMethod / schedule classes of this package are
        instantiated."""
        from ..utils import safe_state

        m = safe_state.load(path)
        if not isinstance(m, OptimMethod):
            raise ValueError(f"{path} does not hold an OptimMethod")
        m._shadow16 = None
        return m


def _cpu(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu()
    if isinstance(v, Table):
        t = Table()
        for k, x in v.items():
            t[k] = _cpu(x)
        return t
    return v


def native_ok(*ts):
    return all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
               for t in ts)
