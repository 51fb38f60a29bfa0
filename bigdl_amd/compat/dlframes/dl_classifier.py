"""Reference ``bigdl.dlframes.dl_classifier`` (P/dlframes/dl_classifier.py): DataFrame estimators taking the
facade's Layer / Criterion handles (or engine modules) with the reference argument order."""
from ... import dlframes as _d
from ...dlframes import HasBatchSize, HasFeatureSize, HasLearningRate, HasMaxEpoch  # noqa: F401


def _v(x):
    return getattr(x, "value", x)


class DLEstimator(_d.DLEstimator):
    def __init__(self, model, criterion, feature_size, label_size=(1,), jvalue=None, bigdl_type="float"):
        super().__init__(_v(model), _v(criterion), feature_size, label_size)


class DLModel(_d.DLModel):
    def __init__(self, model, featureSize, jvalue=None, bigdl_type="float"):
        super().__init__(_v(model), featureSize)


class DLClassifier(_d.DLClassifier):
    def __init__(self, model, criterion, feature_size, bigdl_type="float"):
        super().__init__(_v(model), _v(criterion), feature_size)


class DLClassifierModel(_d.DLClassifierModel):
    def __init__(self, model, featureSize, jvalue=None, bigdl_type="float"):
        super().__init__(_v(model), featureSize)


__all__ = ["HasBatchSize", "HasMaxEpoch", "HasFeatureSize", "HasLearningRate", "DLEstimator", "DLModel",
           "DLClassifier", "DLClassifierModel"]
