"""Reference ``bigdl.models.utils.model_broadcast`` (P/models/utils/model_broadcast.py).

The reference pickles a layer into a Spark broadcast by saving it in the BigDL model format and reloading it on
first access of ``value``. Same contract here without Spark: ``broadcast_model`` writes the model once
(``saveModel``), and every ``ModelBroadcast.value`` access on a fresh handle loads an independent copy, so
tasks never share parameter storage with the driver's layer. Across ranks use
``bigdl_amd.parallel.broadcast.ModelBroadcast``, which broadcasts the weights over the process group."""
import os
import tempfile

from ...nn.layer import Model


def broadcast_model(sc, layer):
    return ModelBroadcast(sc, layer)


class ModelBroadcast:
    def __init__(self, sc=None, layer=None, pickle_registry=None, path=None, bigdl_type="float"):
        self.bigdl_type = getattr(layer, "bigdl_type", bigdl_type) if layer is not None else bigdl_type
        self._path = path
        if layer is not None:
            fd, self._path = tempfile.mkstemp(suffix=".bigdl")
            os.close(fd)
            self.dump(layer, self._path)
            self._value = layer

    @staticmethod
    def dump(value, path):
        try:
            value.saveModel(path, over_write=True)
        except Exception as e:
            raise ValueError(f"Could not serialize broadcast: {e.__class__.__name__}") from e
        return path

    def _load(self, path):
        return Model.loadModel(path, bigdl_type=self.bigdl_type)

    @property
    def value(self):
        if not hasattr(self, "_value") and self._path is not None:
            self._value = self._load(self._path)
        return self._value

    def __reduce__(self):
        # a handle pickled to a task carries only the path; the task loads its own copy
        return ModelBroadcast, (None, None, None, self._path, self.bigdl_type)

    def unpersist(self):
        if self._path and os.path.exists(self._path):
            os.remove(self._path)
        self._path = None


__all__ = ["broadcast_model", "ModelBroadcast"]
