"""Reference ``bigdl.dlframes.dl_image_transformer`` (P/dlframes/dl_image_transformer.py): takes a facade
FeatureTransformer (``bigdl.transform.vision.image``) or an engine transformer."""
from ... import dlframes as _d


class DLImageTransformer(_d.DLImageTransformer):
    def __init__(self, transformer, jvalue=None, bigdl_type="float"):
        super().__init__(getattr(transformer, "value", transformer))


__all__ = ["DLImageTransformer"]
