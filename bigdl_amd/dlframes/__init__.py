"""ML-pipeline integration: estimators / transformers over DataFrames.

Reference: S/dlframes/DLEstimator.scala:35-440 (DLEstimator.fit -> DLModel; DLModel.transform appends a
prediction column), DLClassifier.scala:37-88 (DLClassifier / DLClassifierModel: argmax class, 1-based),
DLImageReader.scala (readImages -> DataFrame of image rows), DLImageTransformer.scala (vision transformer over
an image column), SharedParamsAdapter.scala. The reference binds to Spark ML; Spark is not part of an MI355X
node's software stack, so the same estimator / model / params API is provided over pandas DataFrames (one per
rank for distributed jobs: the Optimizer underneath does the RCCL data parallelism).

    est = DLClassifier(model, ClassNLLCriterion(), featureSize=[784]).setBatchSize(128).setMaxEpoch(5)
    dlmodel = est.fit(df)                     # df: "features" (array-like) + "label" columns
    out = dlmodel.transform(test_df)          # adds "prediction"
"""
import copy
import os

import numpy as np
import torch

from ..dataset.core import LocalArrayDataSet, Sample


def _pd():
    import pandas as pd
    return pd


class _Params:
    """Spark-ML style fluent params (SharedParamsAdapter)."""

    def __init__(self, **defaults):
        self._params = dict(defaults)

    def set(self, k, v):
        self._params[k] = v
        return self

    def get(self, k):
        return self._params.get(k)

    def getOrDefault(self, k):
        return self._params[k]

    def explainParams(self):
        return "\n".join(f"{k}: {v!r}" for k, v in sorted(self._params.items()))


class HasBatchSize(_Params):
    """Param mixin (reference P/dlframes/dl_classifier.py HasBatchSize)."""

    def setBatchSize(self, v):
        return self.set("batchSize", int(v))

    def getBatchSize(self):
        return self.get("batchSize")


class HasMaxEpoch(_Params):
    def setMaxEpoch(self, v):
        return self.set("maxEpoch", int(v))

    def getMaxEpoch(self):
        return self.get("maxEpoch")


class HasLearningRate(_Params):
    def setLearningRate(self, v):
        return self.set("learningRate", float(v))

    def getLearningRate(self):
        return self.get("learningRate")


class HasFeatureSize(_Params):
    def setFeatureSize(self, v):
        self.featureSize = list(v)
        return self

    def getFeatureSize(self):
        return self.featureSize


def _row_tensor(v, size):
    t = torch.as_tensor(np.asarray(v, dtype=np.float32))
    return t.reshape(size) if size else t


class DLEstimator(HasBatchSize, HasMaxEpoch, HasLearningRate, HasFeatureSize):
    def __init__(self, model, criterion, featureSize, labelSize=(1,)):
        super().__init__(featuresCol="features", labelCol="label", predictionCol="prediction", batchSize=1,
                         maxEpoch=50, learningRate=1e-3, learningRateDecay=0.0, optimMethod=None, endWhen=None)
        self.model, self.criterion = model, criterion
        self.featureSize = list(featureSize)
        self.labelSize = list(labelSize)
        self.trainSummary = None
        self.validationSummary = None
        self.validation = None

    # fluent setters (DLEstimator.scala:171-243)
    def setFeaturesCol(self, v):
        return self.set("featuresCol", v)

    def setLabelCol(self, v):
        return self.set("labelCol", v)

    def setPredictionCol(self, v):
        return self.set("predictionCol", v)

    def setBatchSize(self, v):
        return self.set("batchSize", int(v))

    def setEndWhen(self, trigger):
        return self.set("endWhen", trigger)

    def setLearningRate(self, v):
        return self.set("learningRate", float(v))

    def setLearningRateDecay(self, v):
        return self.set("learningRateDecay", float(v))

    def setMaxEpoch(self, v):
        if int(v) <= 0:
            raise ValueError("maxEpoch must be > 0")
        return self.set("maxEpoch", int(v))

    def setOptimMethod(self, m):
        return self.set("optimMethod", m)

    def setTrainSummary(self, s):
        self.trainSummary = s
        return self

    def setValidationSummary(self, s):
        self.validationSummary = s
        return self

    def setValidation(self, trigger, validationDF, vMethods, batchSize):
        self.validation = (trigger, validationDF, vMethods, batchSize)
        return self

    def getBatchSize(self):
        return self.get("batchSize")

    def getMaxEpoch(self):
        return self.get("maxEpoch")

    def getLearningRate(self):
        return self.get("learningRate")

    def _label(self, v):
        return _row_tensor(v, self.labelSize)

    def _samples(self, df, with_label=True):
        fc, lc = self.get("featuresCol"), self.get("labelCol")
        out = []
        for _, row in df.iterrows():
            f = _row_tensor(row[fc], self.featureSize)
            out.append(Sample(f, self._label(row[lc])) if with_label else Sample(f))
        return out

    def _optim_method(self):
        m = self.get("optimMethod")
        if m is not None:
            return m
        from ..optim.sgd import SGD
        return SGD(learningRate=self.get("learningRate"), learningRateDecay=self.get("learningRateDecay"))

    def fit(self, df):
        from ..optim.optimizer import Optimizer
        from ..optim.trigger import Trigger

        ds = LocalArrayDataSet(self._samples(df), True)
        opt = Optimizer(self.model, ds, self.criterion, batchSize=self.get("batchSize"),
                        optimMethod=self._optim_method(),
                        endTrigger=self.get("endWhen") or Trigger.maxEpoch(self.get("maxEpoch")))
        if self.trainSummary is not None:
            opt.setTrainSummary(self.trainSummary)
        if self.validationSummary is not None:
            opt.setValidationSummary(self.validationSummary)
        if self.validation is not None:
            trig, vdf, methods, bs = self.validation
            opt.setValidation(trig, LocalArrayDataSet(self._samples(vdf), False), methods, bs)
        trained = opt.optimize()
        return self._wrap(trained)

    def _wrap(self, trained):
        return DLModel(trained, self.featureSize).setFeaturesCol(self.get("featuresCol")) \
            .setPredictionCol(self.get("predictionCol")).setBatchSize(self.get("batchSize"))


class DLModel(HasBatchSize, HasFeatureSize):
    def __init__(self, model, featureSize):
        super().__init__(featuresCol="features", predictionCol="prediction", batchSize=4)
        self.model = model
        self.featureSize = list(featureSize)

    def setFeaturesCol(self, v):
        return self.set("featuresCol", v)

    def setPredictionCol(self, v):
        return self.set("predictionCol", v)

    def setFeatureSize(self, v):
        self.featureSize = list(v)
        return self

    def setBatchSize(self, v):
        return self.set("batchSize", int(v))

    def getFeatureSize(self):
        return self.featureSize

    def _outputs(self, df):
        fc = self.get("featuresCol")
        feats = [_row_tensor(v, self.featureSize) for v in df[fc]]
        bs = max(int(self.get("batchSize")), 1)
        self.model.evaluate()
        dev = getattr(self.model, "_device", torch.device("cpu"))
        outs = []
        with torch.no_grad():
            for i in range(0, len(feats), bs):
                x = torch.stack(feats[i:i + bs]).to(dev)
                outs.append(self.model.forward(x).float().cpu())
        return torch.cat(outs) if outs else torch.empty(0)

    def _to_column(self, out):
        return [row.reshape(-1).tolist() for row in out]

    def transform(self, df):
        out = df.copy()
        out[self.get("predictionCol")] = self._to_column(self._outputs(df))
        return out


class DLClassifier(DLEstimator):
    """DLEstimator with a scalar 1-based class label and a DLClassifierModel result."""

    def __init__(self, model, criterion, featureSize):
        super().__init__(model, criterion, featureSize, [1])

    def _label(self, v):
        return torch.tensor(float(np.asarray(v).reshape(-1)[0]))

    def _wrap(self, trained):
        return DLClassifierModel(trained, self.featureSize).setFeaturesCol(self.get("featuresCol")) \
            .setPredictionCol(self.get("predictionCol")).setBatchSize(self.get("batchSize"))


class DLClassifierModel(DLModel):
    """Prediction = argmax class (1-based, like the reference's label convention)."""

    def _to_column(self, out):
        return (out.reshape(out.shape[0], -1).argmax(1) + 1).double().tolist()


# ---------------------------------------------------------------------------------------------- images
class DLImageReader:
    """readImages(path) -> DataFrame with one "image" row per file: origin, height, width, nChannels, mode
    (OpenCV type code 16 = CV_8UC3) and the BGR bytes (DLImageReader.scala schema)."""

    @staticmethod
    def readImages(path, minPartitions=1):
        from ..dataset.image import LocalImageFiles, read_image

        files = []
        if os.path.isdir(path):
            for root, _, fs in os.walk(path):
                for f in sorted(fs):
                    if f.endswith(LocalImageFiles.EXT):
                        files.append(os.path.join(root, f))
        else:
            files = [path]
        rows = []
        for f in sorted(files):
            img = read_image(f)
            rows.append({"image": {"origin": f, "height": int(img.shape[0]), "width": int(img.shape[1]),
                                   "nChannels": 3, "mode": 16, "data": bytes(img.numpy().tobytes())}})
        return _pd().DataFrame(rows)


def image_row_to_tensor(row):
    return torch.frombuffer(bytearray(row["data"]), dtype=torch.uint8).reshape(row["height"], row["width"],
                                                                               row["nChannels"])


class DLImageTransformer(_Params):
    """Applies a vision FeatureTransformer (transform/vision) to the image column; the output column holds the
    transformed image as an fp32 CHW array (DLImageTransformer.scala)."""

    def __init__(self, transformer):
        super().__init__(inputCol="image", outputCol="output")
        self.transformer = transformer

    def setInputCol(self, v):
        return self.set("inputCol", v)

    def setOutputCol(self, v):
        return self.set("outputCol", v)

    def transform(self, df):
        from ..transform.vision.image import ImageFeature

        res = []
        for row in df[self.get("inputCol")]:
            mat = image_row_to_tensor(row).float()
            feat = ImageFeature(uri=row.get("origin"))
            feat[ImageFeature.mat] = mat
            feat[ImageFeature.originalSize] = tuple(mat.shape)
            out = self.transformer.transform(feat)
            t = out.get(ImageFeature.imageTensor)
            if t is None:
                t = out.opencvMat().permute(2, 0, 1)           # HWC -> CHW
            res.append(np.asarray(t, dtype=np.float32))
        out_df = df.copy()
        out_df[self.get("outputCol")] = res
        return out_df


__all__ = ["HasBatchSize", "HasMaxEpoch", "HasLearningRate", "HasFeatureSize", "DLEstimator", "DLModel", "DLClassifier", "DLClassifierModel", "DLImageReader", "DLImageTransformer",
           "image_row_to_tensor"]
