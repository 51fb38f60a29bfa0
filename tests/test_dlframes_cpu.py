"""DLEstimator / DLClassifier / DLImageReader / DLImageTransformer over pandas DataFrames
(reference S/dlframes/*, DLEstimatorSpec / DLClassifierSpec behaviour)."""
import numpy as np
import pandas as pd
import torch

from bigdl_amd import nn
from bigdl_amd.dlframes import DLClassifier, DLEstimator, DLImageReader, DLImageTransformer
from bigdl_amd.utils.random_generator import RNG


def _blobs(n=200, seed=0):
    rng = np.random.RandomState(seed)
    y = rng.randint(1, 3, n)
    x = rng.randn(n, 4) * 0.3 + (y[:, None] - 1.5) * 2.0
    return pd.DataFrame({"features": list(x), "label": y.astype(float)})


def test_dlclassifier_fit_transform_learns_separable_data():
    RNG.setSeed(1)
    model = nn.Sequential().add(nn.Linear(4, 8)).add(nn.ReLU()).add(nn.Linear(8, 2)).add(nn.LogSoftMax())
    est = DLClassifier(model, nn.ClassNLLCriterion(), [4]).setBatchSize(20).setMaxEpoch(10).setLearningRate(0.1)
    m = est.fit(_blobs())
    out = m.transform(_blobs(100, seed=1))
    acc = (out["prediction"] == out["label"]).mean()
    assert acc > 0.95, acc
    assert set(out["prediction"].unique()) <= {1.0, 2.0}


def test_dlestimator_regression_prediction_column():
    RNG.setSeed(2)
    rng = np.random.RandomState(0)
    x = rng.randn(256, 3).astype(np.float32)
    w = np.array([1.0, -2.0, 0.5], dtype=np.float32)
    df = pd.DataFrame({"f": list(x), "y": list((x @ w)[:, None])})
    est = DLEstimator(nn.Linear(3, 1), nn.MSECriterion(), [3], [1]).setFeaturesCol("f").setLabelCol("y") \
        .setBatchSize(32).setMaxEpoch(30).setLearningRate(0.1).setPredictionCol("p")
    out = est.fit(df).transform(df)
    pred = np.array([p[0] for p in out["p"]])
    assert np.abs(pred - x @ w).mean() < 0.05


def test_image_reader_and_transformer(tmp_path):
    from PIL import Image
    from bigdl_amd.transform.vision.image.augmentation import ChannelNormalize

    arr = (np.arange(4 * 5 * 3) % 200).astype(np.uint8).reshape(4, 5, 3)
    Image.fromarray(arr).save(tmp_path / "a.png")
    df = DLImageReader.readImages(str(tmp_path))
    row = df["image"][0]
    assert (row["height"], row["width"], row["nChannels"]) == (4, 5, 3)
    out = DLImageTransformer(ChannelNormalize(10.0, 20.0, 30.0)).transform(df)
    t = out["output"][0]
    assert t.shape == (3, 4, 5)
    bgr = arr[..., ::-1].astype(np.float32)
    assert np.allclose(t[0], bgr[..., 0] - 30.0) or np.allclose(t[0], bgr[..., 0] - 10.0)


def test_reference_dlframes_facade_takes_layer_handles():
    """bigdl.dlframes.dl_classifier (P/dlframes/dl_classifier.py) with the facade's Layer / Criterion handles."""
    from bigdl_amd import compat

    compat.install()
    from bigdl.dlframes.dl_classifier import DLClassifier as RefDLClassifier
    from bigdl.nn.criterion import ClassNLLCriterion
    from bigdl.nn.layer import Linear, LogSoftMax, ReLU, Sequential

    RNG.setSeed(1)
    model = Sequential().add(Linear(4, 8)).add(ReLU()).add(Linear(8, 2)).add(LogSoftMax())
    est = RefDLClassifier(model, ClassNLLCriterion(), [4]).setBatchSize(20).setMaxEpoch(10).setLearningRate(0.1)
    out = est.fit(_blobs()).transform(_blobs(100, seed=1))
    assert (out["prediction"] == out["label"]).mean() > 0.95
