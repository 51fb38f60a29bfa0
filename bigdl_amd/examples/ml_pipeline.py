"""DataFrame ML-pipeline examples: DLClassifier / DLEstimator fitted on a DataFrame, then used as a transformer.

Reference: S/example/MLPipeline/DLClassifierLeNet.scala (LeNet on an MNIST DataFrame), DLClassifierLogisticRegression
.scala (a 2-feature logistic regression classifier) and DLEstimatorMultiLabelLR.scala (multi-output linear regression
with an MSE criterion). pandas stands in for the Spark DataFrame (bigdl_amd.dlframes).

    python -m bigdl_amd.examples mlpipeline --task {lenet, logreg, multilabel}
"""
import argparse

import numpy as np
import pandas as pd
import torch


def _logreg(args):
    from .. import nn
    from ..dlframes import DLClassifier

    rng = np.random.RandomState(0)
    n = 200
    x = rng.randn(n, 2).astype(np.float32)
    y = (x[:, 0] + 0.5 * x[:, 1] > 0).astype(np.float32) + 1.0           # 1-based labels
    df = pd.DataFrame({"features": list(x), "label": list(y)})
    torch.manual_seed(0)
    model = nn.Sequential().add(nn.Linear(2, 2)).add(nn.LogSoftMax())
    est = DLClassifier(model, nn.ClassNLLCriterion(), [2]).setLabelCol("label").setFeaturesCol("features") \
        .setBatchSize(args.batchSize).setMaxEpoch(args.maxEpoch).setLearningRate(0.2)
    out = est.fit(df).transform(df)
    acc = float((np.asarray(out["prediction"], dtype=np.float32) == y).mean())
    return {"task": "logreg", "rows": n, "train_accuracy": acc}


def _multilabel(args):
    from .. import nn
    from ..dlframes import DLEstimator

    rng = np.random.RandomState(1)
    n = 160
    x = rng.randn(n, 2).astype(np.float32)
    w = np.array([[1.0, -2.0], [0.5, 3.0]], dtype=np.float32)
    y = x @ w.T
    df = pd.DataFrame({"features": list(x), "label": list(y)})
    torch.manual_seed(0)
    est = DLEstimator(nn.Linear(2, 2), nn.MSECriterion(), [2], [2]).setBatchSize(args.batchSize) \
        .setMaxEpoch(args.maxEpoch * 4).setLearningRate(0.2)
    out = est.fit(df).transform(df)
    pred = np.stack([np.asarray(p, dtype=np.float32) for p in out["prediction"]])
    return {"task": "multilabel", "rows": n, "mse": float(((pred - y) ** 2).mean())}


def _lenet(args):
    from .. import nn
    from ..dlframes import DLClassifier
    from ..models.lenet import LeNet5
    from .lenet_local import load, write_synthetic_mnist
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        write_synthetic_mnist(d, n_train=256, n_test=64)
        train, test = load(d, True), load(d, False)
    tr = pd.DataFrame({"features": [s.feature().reshape(-1).numpy() for s in train],
                       "label": [float(s.label()) for s in train]})
    te = pd.DataFrame({"features": [s.feature().reshape(-1).numpy() for s in test],
                       "label": [float(s.label()) for s in test]})
    torch.manual_seed(0)
    est = DLClassifier(LeNet5(10), nn.ClassNLLCriterion(), [1, 28, 28]).setBatchSize(args.batchSize) \
        .setMaxEpoch(args.maxEpoch).setLearningRate(0.05)
    out = est.fit(tr).transform(te)
    acc = float((np.asarray(out["prediction"], dtype=np.float32) == np.asarray(te["label"])).mean())
    return {"task": "lenet", "rows": len(tr), "test_accuracy": acc}


def run(args):
    return {"lenet": _lenet, "logreg": _logreg, "multilabel": _multilabel}[args.task](args)


def build_parser():
    p = argparse.ArgumentParser(prog="mlpipeline")
    p.add_argument("--task", choices=["lenet", "logreg", "multilabel"], default="logreg")
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--maxEpoch", type=int, default=10)
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
