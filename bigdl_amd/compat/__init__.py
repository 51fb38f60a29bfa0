"""Reference-compatible Python API (``bigdl.*`` module layout of P/ = pyspark/bigdl) over the bigdl_amd engine.

    from bigdl_amd.compat.nn.layer import *          # Sequential, Linear, SpatialConvolution, Model, ...
    from bigdl_amd.compat.nn.criterion import *      # ClassNLLCriterion, ...
    from bigdl_amd.compat.optim.optimizer import *   # Optimizer, SGD, MaxEpoch, Top1Accuracy, ...
    from bigdl_amd.compat.util.common import *       # Sample, init_engine, SparkContext, ...

or, for unmodified reference scripts, ``bigdl_amd.compat.install()`` registers these modules under the
``bigdl.*`` names so ``from bigdl.nn.layer import *`` resolves to them.
"""
import importlib
import sys

_MODULES = {
    "bigdl": "bigdl_amd.compat",
    "bigdl.util": "bigdl_amd.compat.util",
    "bigdl.util.common": "bigdl_amd.compat.util.common",
    "bigdl.nn": "bigdl_amd.compat.nn",
    "bigdl.nn.layer": "bigdl_amd.compat.nn.layer",
    "bigdl.nn.criterion": "bigdl_amd.compat.nn.criterion",
    "bigdl.optim": "bigdl_amd.compat.optim",
    "bigdl.optim.optimizer": "bigdl_amd.compat.optim.optimizer",
    "bigdl.dataset": "bigdl_amd.compat.dataset",
    "bigdl.dataset.transformer": "bigdl_amd.compat.dataset.transformer",
    "bigdl.dataset.mnist": "bigdl_amd.compat.dataset.mnist",
    "bigdl.dataset.base": "bigdl_amd.compat.dataset.base",
    "bigdl.dataset.news20": "bigdl_amd.compat.dataset.news20",
    "bigdl.dataset.movielens": "bigdl_amd.compat.dataset.movielens",
    "bigdl.dataset.sentence": "bigdl_amd.compat.dataset.sentence",
    "bigdl.dlframes": "bigdl_amd.compat.dlframes",
    "bigdl.dlframes.dl_classifier": "bigdl_amd.compat.dlframes.dl_classifier",
    "bigdl.dlframes.dl_image_reader": "bigdl_amd.compat.dlframes.dl_image_reader",
    "bigdl.dlframes.dl_image_transformer": "bigdl_amd.compat.dlframes.dl_image_transformer",
    "bigdl.transform": "bigdl_amd.compat.transform",
    "bigdl.transform.vision": "bigdl_amd.compat.transform.vision",
    "bigdl.transform.vision.image": "bigdl_amd.compat.transform.vision.image",
    "bigdl.nn.keras": "bigdl_amd.compat.nn.keras",
    "bigdl.nn.keras.layer": "bigdl_amd.compat.nn.keras.layer",
    "bigdl.nn.keras.topology": "bigdl_amd.compat.nn.keras.topology",
    "bigdl.nn.onnx": "bigdl_amd.compat.nn.onnx",
    "bigdl.nn.onnx.layer": "bigdl_amd.compat.nn.onnx.layer",
    "bigdl.nn.initialization_method": "bigdl_amd.compat.nn.initialization_method",
    "bigdl.util.tf_utils": "bigdl_amd.compat.util.tf_utils",
    "bigdl.util.engine": "bigdl_amd.compat.util.engine",
    "bigdl.version": "bigdl_amd.compat.version",
    "bigdl.contrib": "bigdl_amd.compat.contrib",
    "bigdl.contrib.onnx": "bigdl_amd.compat.contrib.onnx",
    "bigdl.models": "bigdl_amd.compat.models",
    "bigdl.models.utils": "bigdl_amd.compat.models.utils",
    "bigdl.models.utils.model_broadcast": "bigdl_amd.compat.models.utils.model_broadcast",
}


def install():
    """Alias the facade as the reference's ``bigdl`` package (only if no real ``bigdl`` is imported)."""
    for name, target in _MODULES.items():
        if name in sys.modules and not sys.modules[name].__name__.startswith("bigdl_amd"):
            raise RuntimeError(f"a different {name!r} is already imported")
        sys.modules[name] = importlib.import_module(target)
    return sys.modules["bigdl"]
