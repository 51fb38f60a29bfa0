"""Transfer learning from a TensorFlow model: load a frozen GraphDef as a feature extractor, train a new head.

Reference: S/example/tensorflow/transferlearning/TransferLearning.scala (``Module.loadTF`` of a pre-trained
slim model cut at a bottleneck node, wrapped as a frozen feature extractor, a new Linear + LogSoftMax trained on
top with the Optimizer) and dump_model_example.py (exporting the TF graph). Without ``--pb`` the "pre-trained"
extractor is a small NHWC conv net saved with ``saveTF`` first.
"""
import argparse
import os
import tempfile

import torch

from ._common import device_of


def _extractor():
    from .. import nn

    torch.manual_seed(0)
    return (nn.Sequential().add(nn.SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1, format="NHWC")).add(nn.ReLU())
            .add(nn.SpatialMaxPooling(2, 2, 2, 2, format="NHWC"))
            .add(nn.SpatialConvolution(8, 16, 3, 3, 1, 1, 1, 1, format="NHWC")).add(nn.ReLU())
            .add(nn.SpatialMaxPooling(2, 2, 2, 2, format="NHWC")).add(nn.Reshape([4 * 4 * 16])))


def _data(n, g):
    """Two classes told apart by which image half is brighter: separable from generic conv features."""
    x = torch.randn(n, 16, 16, 3, generator=g) * 0.3
    y = torch.randint(0, 2, (n,), generator=g)
    x[y == 0, :8] += 1.0
    x[y == 1, 8:] += 1.0
    return x, (y + 1).float()


def run(args):
    from .. import nn
    from ..dataset.core import LocalArrayDataSet, Sample
    from ..nn.module import Module
    from ..optim.optimizer import Optimizer
    from ..optim.sgd import SGD
    from ..optim.trigger import Trigger
    from ..optim.validation import Top1Accuracy

    dev = device_of(args.device)
    with tempfile.TemporaryDirectory() as d:
        pb = args.pb
        out_node = args.outputNode
        if pb is None:
            pb = os.path.join(d, "extractor.pb")
            ext = _extractor()
            ext.evaluate()
            out_node = ext.saveTF([("input", [None, 16, 16, 3])], pb)
        features = Module.loadTF(pb, ["input"], [out_node])
    features.freeze()
    head = nn.Sequential().add(nn.Linear(4 * 4 * 16, 2)).add(nn.LogSoftMax())
    model = nn.Sequential().add(features).add(head)
    g = torch.Generator().manual_seed(2)
    xtr, ytr = _data(256, g)
    xte, yte = _data(64, g)
    frozen_before = [p.clone() for p in features.parameters()[0]]
    opt = Optimizer(model.to(dev), LocalArrayDataSet([Sample(a, b) for a, b in zip(xtr, ytr)], True),
                    nn.ClassNLLCriterion(), batchSize=args.batchSize,
                    optimMethod=SGD(learningRate=args.learningRate, momentum=0.9, dampening=0.0),
                    endTrigger=Trigger.maxEpoch(args.maxEpoch))
    trained = opt.optimize()
    (acc, _), = trained.evaluate(LocalArrayDataSet([Sample(a, b) for a, b in zip(xte, yte)], False),
                                 [Top1Accuracy()], args.batchSize)
    unchanged = all(torch.equal(a.cpu(), b.cpu()) for a, b in zip(frozen_before, features.parameters()[0]))
    return {"test_accuracy": float(acc.result()[0]), "extractor_frozen": unchanged}


def build_parser():
    p = argparse.ArgumentParser(prog="tftransferlearning")
    p.add_argument("--pb", default=None, help="frozen TF GraphDef with an 'input' placeholder")
    p.add_argument("--outputNode", default=None)
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--maxEpoch", type=int, default=5)
    p.add_argument("--learningRate", type=float, default=0.05)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
