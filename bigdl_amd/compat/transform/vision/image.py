"""Reference ``bigdl.transform.vision.image`` (P/transform/vision/image.py): snake_case transformer
constructors (``Resize(resize_h, resize_w)``, ``ChannelNormalize(mean_r, ...)``, ``MatToTensor(to_rgb=...)``)
and the ImageFrame accessors (``get_image`` / ``get_label`` / ``get_predict`` / ``get_sample``, ``is_local``)
over ``bigdl_amd.transform.vision.image``."""
import inspect

import numpy as np
import torch

from ....transform.vision import image as _im
from ..._convert import convert_kwargs, to_numpy

_WRAPPERS = {}


class FeatureTransformer:
    """Handle on an engine FeatureTransformer; ``transform`` applies it to an ImageFrame or an ImageFeature."""

    _impl = None

    def __init__(self, *args, **kwargs):
        self.value = kwargs.pop("jvalue", None) or self._impl(*args, **convert_kwargs(self._impl, kwargs))
        self.bigdl_type = "float"

    def transform(self, image_frame, bigdl_type="float"):
        return image_frame.transform(self)

    def __call__(self, image_frame, bigdl_type="float"):
        return self.transform(image_frame)


def _make(name, impl):
    cls = type(name, (FeatureTransformer,), {"_impl": impl, "__doc__": f"Reference ``{name}`` over the engine's "
                                                                       f"``transform.vision.image.{name}``."})
    cls.__module__ = __name__
    return cls


for _name, _obj in inspect.getmembers(_im, inspect.isclass):
    if issubclass(_obj, _im.FeatureTransformer) and not _name.startswith("_") and _name != "FeatureTransformer":
        _WRAPPERS[_name] = _make(_name, _obj)
        globals()[_name] = _WRAPPERS[_name]


class ImageFrame:
    def __init__(self, jvalue=None, bigdl_type="float"):
        self.value = jvalue
        self.bigdl_type = bigdl_type

    @classmethod
    def read(cls, path, sc=None, min_partitions=1, bigdl_type="float"):
        frame = _im.ImageFrame.read(path, min_partitions)
        return (LocalImageFrame if frame.isLocal() else DistributedImageFrame)(jvalue=frame)

    def transform(self, transformer, bigdl_type="float"):
        t = transformer.value if isinstance(transformer, FeatureTransformer) else transformer
        return type(self)(jvalue=self.value.transform(t))

    def is_local(self):
        return self.value.isLocal()

    def is_distributed(self):
        return self.value.isDistributed()

    def _features(self):
        return list(self.value.toLocal().array) if hasattr(self.value, "toLocal") else list(self.value.array)

    def get_image(self, float_key="floats", to_chw=True):
        out = []
        for f in self._features():
            t = f.get(_im.ImageFeature.imageTensor)
            if t is None:
                t = torch.as_tensor(f.get(float_key) if f.get(float_key) is not None else f.opencvMat()).float()
                t = t.permute(2, 0, 1) if to_chw and t.dim() == 3 else t
            elif not to_chw and t.dim() == 3:
                t = t.permute(1, 2, 0)
            out.append(to_numpy(t))
        return out

    def get_label(self):
        return [None if f.getLabel() is None else to_numpy(torch.as_tensor(f.getLabel())) for f in self._features()]

    def get_predict(self, key="predict"):
        return [(f.getUri(), None if f.get(key) is None else to_numpy(f.get(key))) for f in self._features()]

    def get_sample(self, key="sample"):
        return [f.get(key) for f in self._features()]


class LocalImageFrame(ImageFrame):
    def __init__(self, image_list=None, label_list=None, jvalue=None, bigdl_type="float"):
        if jvalue is None:
            feats = []
            for i, img in enumerate(image_list or []):
                f = _im.ImageFeature(label=None if label_list is None else torch.as_tensor(label_list[i]))
                f[_im.ImageFeature.mat] = torch.as_tensor(np.asarray(img, dtype=np.float32))
                f[_im.ImageFeature.originalSize] = tuple(np.asarray(img).shape)
                feats.append(f)
            jvalue = _im.LocalImageFrame(feats)
        super().__init__(jvalue, bigdl_type)


class DistributedImageFrame(ImageFrame):
    pass


__all__ = ["FeatureTransformer", "ImageFrame", "LocalImageFrame", "DistributedImageFrame"] + sorted(_WRAPPERS)
