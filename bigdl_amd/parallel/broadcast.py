"""Model broadcast (reference S/models/utils/ModelBroadcast.scala:51-349, ModelBroadcastFactory.scala).

The reference ships the model structure once per executor and the weights separately, caching executor-side
replicas by UUID. With one process per GPU every rank already builds the structure from the same code, so
broadcasting is only the weights: every parameter and buffer tensor of rank 0 is sent over RCCL, packed into one
flat buffer per dtype so the whole model costs one collective per dtype instead of one per tensor.
"""
import torch
import torch.distributed as dist


def _tensors(model):
    out = []
    for m in model.flattened_layers():
        for w, _ in getattr(m, "_params", ()):
            t = getattr(m, w, None)
            if torch.is_tensor(t):
                out.append(t)
        for b in getattr(m, "_buffers", ()):
            t = getattr(m, b, None)
            if torch.is_tensor(t):
                out.append(t)
    return out


def _refresh_bf16(model):
    """Rewrite the bf16 compute copies (GPU engine) from the broadcast fp32 weights, so kernels that read the
    shadow see the new values too."""
    for m in model.flattened_layers():
        if getattr(m, "_w16_managed", False):
            for name, t16 in m._w16.items():
                w = getattr(m, name, None)
                if torch.is_tensor(w):
                    t16.copy_(w)


class ModelBroadcast:
    def __init__(self, applyProtoBuffer=False, group=None, src=0):
        self.group, self.src = group, src
        self._model = None

    def broadcast(self, model):
        """Make every rank's weights equal to rank ``src``'s (no-op outside a multi-rank job)."""
        self._model = model
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(self.group) == 1:
            return self
        by_dtype = {}
        for t in _tensors(model):
            by_dtype.setdefault((t.dtype, t.device), []).append(t)
        for (_, _), ts in by_dtype.items():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            dist.broadcast(flat, self.src, group=self.group)
            off = 0
            for t in ts:
                n = t.numel()
                t.data.copy_(flat[off:off + n].view_as(t))
                off += n
        _refresh_bf16(model)
        return self

    def value(self, initGradient=False, shareWeight=True):
        """The broadcast model (shareWeight=False returns an independent copy, like the reference)."""
        if shareWeight:
            return self._model
        return self._model.cloneModule()


class ModelBroadcastFactory:
    @staticmethod
    def create(applyProtoBuffer=False):
        return ModelBroadcast(applyProtoBuffer)


__all__ = ["ModelBroadcast", "ModelBroadcastFactory"]
