"""LeNet-5 on MNIST without a cluster: train, test and predict on one process.

Reference: S/example/lenetLocal/{Train,Test,Predict}.scala (LocalOptimizer over MNIST idx files, Top-1 validation,
``predictClass`` on the first test images). Without ``--folder`` a small synthetic MNIST (idx format, digits drawn as
class-dependent bars) is written first, so the idx readers are exercised end to end.
"""
import argparse
import os
import tempfile

import torch

from ._common import device_of


def write_synthetic_mnist(folder, n_train=512, n_test=128, seed=0):
    """idx files whose images encode the class as a bright horizontal band: learnable, deterministic."""
    from ..dataset.mnist_cifar import write_mnist

    g = torch.Generator().manual_seed(seed)
    for pre, n in (("train", n_train), ("t10k", n_test)):
        labels = torch.randint(0, 10, (n,), generator=g)
        imgs = (torch.rand(n, 28, 28, generator=g) * 60).to(torch.uint8)
        for i, c in enumerate(labels.tolist()):
            imgs[i, 2 + 2 * c: 4 + 2 * c, 4:24] = 250
        write_mnist(os.path.join(folder, f"{pre}-images-idx3-ubyte"), os.path.join(folder, f"{pre}-labels-idx1-ubyte"),
                    imgs.numpy(), labels.numpy())


def load(folder, train):
    from ..dataset.core import Sample
    from ..dataset.image import BytesToGreyImg
    from ..dataset.mnist_cifar import load_mnist

    pre = "train" if train else "t10k"
    recs = load_mnist(os.path.join(folder, f"{pre}-images-idx3-ubyte"), os.path.join(folder, f"{pre}-labels-idx1-ubyte"))
    mean, std = 0.13066047740239506 * 255, 0.3081078 * 255
    return [Sample(((img.content * 255.0 - mean) / std).reshape(1, 28, 28), torch.tensor(img.label()))
            for img in BytesToGreyImg(28, 28).apply(iter(recs))]


def run(args):
    from .. import nn
    from ..dataset.core import LocalArrayDataSet
    from ..models.lenet import LeNet5
    from ..optim.optimizer import Optimizer
    from ..optim.sgd import SGD
    from ..optim.trigger import Trigger
    from ..optim.validation import Top1Accuracy

    tmp = None
    folder = args.folder
    if folder is None:
        tmp = tempfile.TemporaryDirectory()
        folder = tmp.name
        write_synthetic_mnist(folder)
    train, test = load(folder, True), load(folder, False)
    torch.manual_seed(0)
    model = LeNet5(10).to(device_of(args.device))
    opt = Optimizer(model, LocalArrayDataSet(train, True), nn.ClassNLLCriterion(), batchSize=args.batchSize,
                    optimMethod=SGD(learningRate=args.learningRate, momentum=0.9, dampening=0.0),
                    endTrigger=Trigger.maxEpoch(args.maxEpoch))
    trained = opt.optimize()
    (acc, _), = trained.evaluate(LocalArrayDataSet(test, False), [Top1Accuracy()], args.batchSize)
    first = torch.stack([s.feature() for s in test[:10]])
    pred = trained.predictClass(first.to(device_of(args.device)))
    out = {"train": len(train), "test": len(test), "top1": float(acc.result()[0]),
           "predicted": [int(p) for p in torch.as_tensor(pred).reshape(-1).tolist()],
           "labels": [int(s.label()) for s in test[:10]]}
    if tmp is not None:
        tmp.cleanup()
    return out


def build_parser():
    p = argparse.ArgumentParser(prog="lenetlocal")
    p.add_argument("--folder", default=None, help="MNIST idx files (train-*/t10k-*)")
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--maxEpoch", type=int, default=3)
    p.add_argument("--learningRate", type=float, default=0.05)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
