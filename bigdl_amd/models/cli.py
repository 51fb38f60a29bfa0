"""Model-zoo entry points: train / test / perf for every model family.

Reference mains: S/models/lenet/{Train,Test}.scala, S/models/resnet/{TrainCIFAR10,TrainImageNet,Test}.scala,
S/models/vgg/{Train,Test}.scala, S/models/inception/{Train,Test}.scala (ImageNet seq files, Options.scala),
S/models/rnn/{Train,Test}.scala (tiny-Shakespeare style LM), S/models/autoencoder/Train.scala,
S/models/utils/{LocalOptimizerPerf,DistriOptimizerPerf}.scala (synthetic-data throughput).

    python -m bigdl_amd.models.cli train --model lenet5 --data /path/mnist --maxEpoch 15
    python -m bigdl_amd.models.cli train --model resnet --depth 20 --data /path/cifar-10-batches-bin
    python -m bigdl_amd.models.cli train --model inception_v1 --data /path/imagenet_seq --classNum 1000
    python -m bigdl_amd.models.cli test  --model lenet5 --modelPath model.bigdl --data /path/mnist
    python -m bigdl_amd.models.cli perf  --model resnet_50 --batchSize 128 --iteration 20
Without --data the commands run on synthetic data of the model's input shape (--synthetic N samples).
Multi-GPU: launch with torch.distributed.run (one process per GPU); the Optimizer picks the distributed path.
"""
import argparse
import os
import sys
import time

import torch

from .. import nn
from ..dataset.core import LocalArrayDataSet, Sample

# family -> (builder(args), input shape (C, H, W) or None for sequences, default lr, criterion)
MEAN_STD = {"mnist": (0.13066047740239506 * 255, 0.3081078 * 255),
            "cifar": ((125.3, 123.0, 113.9), (63.0, 62.1, 66.7)),
            "imagenet": ((123.0, 117.0, 104.0), (58.4, 57.1, 57.4))}


def build_model(name, classNum, depth=20):
    from . import autoencoder, inception, lenet, resnet, rnn, vgg

    if name == "lenet5":
        return lenet.LeNet5(classNum), (1, 28, 28)
    if name == "resnet":
        return resnet.ResNet(classNum, depth, dataSet=resnet.DatasetType.CIFAR10), (3, 32, 32)
    if name == "resnet_50":
        return resnet.ResNet(classNum, 50, dataSet=resnet.DatasetType.ImageNet), (3, 224, 224)
    if name == "vgg":
        return vgg.VggForCifar10(classNum), (3, 32, 32)
    if name == "vgg16":
        return vgg.Vgg_16(classNum), (3, 224, 224)
    if name == "inception_v1":
        return inception.Inception_v1_NoAuxClassifier(classNum), (3, 224, 224)
    if name == "inception_v2":
        return inception.Inception_v2_NoAuxClassifier(classNum), (3, 224, 224)
    if name == "inception_v3":
        return inception.Inception_v3(classNum), (3, 299, 299)
    if name == "autoencoder":
        return autoencoder.Autoencoder(32), (1, 28, 28)
    if name == "rnn":
        return rnn.SimpleRNN(classNum, 40, classNum), None
    raise SystemExit(f"unknown model {name}")


def _criterion(name):
    if name == "autoencoder":
        return nn.MSECriterion()
    if name == "rnn":
        return nn.TimeDistributedCriterion(nn.CrossEntropyCriterion(), True)
    if name in ("lenet5", "inception_v3"):
        return nn.ClassNLLCriterion()
    return nn.CrossEntropyCriterion()


def synthetic(name, shape, classNum, n, seqLen=25):
    g = torch.Generator().manual_seed(0)
    out = []
    for _ in range(n):
        if shape is None:      # token sequences: one-hot inputs, next-token labels
            ids = torch.randint(1, classNum + 1, (seqLen + 1,), generator=g)
            x = torch.nn.functional.one_hot(ids[:-1] - 1, classNum).float()
            out.append(Sample(x, ids[1:].float()))
        else:
            x = torch.randn(shape, generator=g)
            y = x.reshape(-1) if name == "autoencoder" else torch.tensor(float(torch.randint(1, classNum + 1, (1,),
                                                                                               generator=g)))
            out.append(Sample(x, y))
    return out


def load_data(args, shape, train=True):
    """Samples for a model family from a local dataset directory (MNIST idx / CIFAR-10 binary / ImageNet seq
    files or an image folder)."""
    from ..dataset.image import BytesToBGRImg, BytesToGreyImg

    d = args.data
    if args.model in ("lenet5", "autoencoder"):
        from ..dataset.mnist_cifar import load_mnist

        pre = "train" if train else "t10k"
        recs = load_mnist(os.path.join(d, f"{pre}-images-idx3-ubyte"), os.path.join(d, f"{pre}-labels-idx1-ubyte"))
        mean, std = MEAN_STD["mnist"]
        out = []
        for img in BytesToGreyImg(28, 28).apply(iter(recs)):
            x = ((img.content * 255.0 - mean) / std).reshape(1, 28, 28)
            out.append(Sample(x, x.reshape(-1) if args.model == "autoencoder" else torch.tensor(img.label())))
        return out
    if args.model in ("resnet", "vgg"):
        from ..dataset.mnist_cifar import load_cifar_test, load_cifar_train

        recs = load_cifar_train(d) if train else load_cifar_test(d)
        mean, std = MEAN_STD["cifar"]
        m = torch.tensor(mean).view(3, 1, 1)
        s = torch.tensor(std).view(3, 1, 1)
        return [Sample((img.toTensor(True) * 255.0 - m) / s, torch.tensor(img.label()))
                for img in BytesToBGRImg().apply(iter(recs))]
    from ..dataset.seqfile import ImageFolder, NativeBGRImgToBatch, SeqFileFolder

    ds = SeqFileFolder.files(d, args.classNum) if SeqFileFolder.paths(d) else ImageFolder.images(d)
    mean, std = MEAN_STD["imagenet"]
    tf = NativeBGRImgToBatch(shape[2], shape[1], 256, mean, std, train=train)
    out = []
    for mb in tf.apply(iter(ds.data(False))):
        x, y = mb.getInput(), mb.getTarget()
        out.extend(Sample(x[i], y[i]) for i in range(x.shape[0]))
    return out


def cmd_train(args):
    from ..optim.optimizer import Optimizer
    from ..optim.sgd import SGD
    from ..optim.trigger import Trigger
    from ..optim.validation import Loss, Top1Accuracy

    model, shape = build_model(args.model, args.classNum, args.depth)
    train = load_data(args, shape, True) if args.data else synthetic(args.model, shape, args.classNum, args.synthetic)
    opt = Optimizer(model, LocalArrayDataSet(train, True), _criterion(args.model), batchSize=args.batchSize,
                    optimMethod=SGD(learningRate=args.learningRate, momentum=args.momentum,
                                    weightDecay=args.weightDecay, dampening=0.0),
                    endTrigger=Trigger.maxEpoch(args.maxEpoch))
    if args.data and args.model not in ("autoencoder", "rnn"):
        val = load_data(args, shape, False)
        opt.setValidation(Trigger.everyEpoch(), LocalArrayDataSet(val, False), [Top1Accuracy(), Loss()],
                          args.batchSize)
    if args.checkpoint:
        opt.setCheckpoint(args.checkpoint, Trigger.everyEpoch())
        if args.overWrite:
            opt.overWriteCheckpoint()
    trained = opt.optimize()
    if args.modelPath:
        trained.saveModule(args.modelPath, overWrite=True)
    return 0


def cmd_test(args):
    from ..nn.module import Module
    from ..optim.validation import Loss, Top1Accuracy, Top5Accuracy

    model = Module.loadModule(args.modelPath)
    _, shape = build_model(args.model, args.classNum, args.depth)
    data = load_data(args, shape, False) if args.data else synthetic(args.model, shape, args.classNum, args.synthetic)
    methods = [Top1Accuracy(), Top5Accuracy(), Loss()] if args.model not in ("autoencoder",) else [Loss()]
    results = model.evaluate(LocalArrayDataSet(data, False), methods, args.batchSize)
    for r, m in results:
        print(f"{m.format() if hasattr(m, 'format') else type(m).__name__} is {r}")
    return 0


def cmd_perf(args):
    """LocalOptimizerPerf / DistriOptimizerPerf: forward + backward + update on one fixed random batch."""
    from ..optim.sgd import SGD
    from ..optim.train_step import TrainStep

    model, shape = build_model(args.model, args.classNum, args.depth)
    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    step = TrainStep(model, _criterion(args.model), SGD(learningRate=0.01), device=dev)
    if shape is None:
        x = torch.randn(args.batchSize, 25, args.classNum, device=dev)
        y = torch.randint(1, args.classNum + 1, (args.batchSize, 25), device=dev).float()
    else:
        x = torch.randn((args.batchSize,) + tuple(shape), device=dev)
        if args.inputData == "constant":
            x.fill_(0.01)
        y = x.reshape(args.batchSize, -1) if args.model == "autoencoder" else \
            torch.randint(1, args.classNum + 1, (args.batchSize,), device=dev).float()
    for _ in range(2):
        step.step(x, y)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    for i in range(args.iteration):
        t0 = time.perf_counter()
        step.step(x, y)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"Iteration {i + 1}: {dt * 1e3:.1f} ms, throughput {args.batchSize / dt:.1f} records/second, "
              f"loss {float(step.loss):.4f}")
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="bigdl_amd.models.cli")
    ap.add_argument("command", choices=["train", "test", "perf"])
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--data", "-f", default=None, help="dataset folder (MNIST / CIFAR-10 / ImageNet seq files)")
    ap.add_argument("--synthetic", type=int, default=512, help="samples of synthetic data when --data is absent")
    ap.add_argument("--classNum", type=int, default=10)
    ap.add_argument("--depth", type=int, default=20)
    ap.add_argument("--batchSize", "-b", type=int, default=128)
    ap.add_argument("--maxEpoch", "-e", type=int, default=15)
    ap.add_argument("--learningRate", "-r", type=float, default=0.05)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weightDecay", type=float, default=1e-4)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--overWrite", action="store_true")
    ap.add_argument("--modelPath", default=None)
    ap.add_argument("--iteration", "-i", type=int, default=20)
    ap.add_argument("--inputData", default="random", choices=["random", "constant"])
    args = ap.parse_args(argv)
    from ..utils.engine import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    Engine.init(master=f"local[{world}]", dist=world > 1)
    try:
        return {"train": cmd_train, "test": cmd_test, "perf": cmd_perf}[args.command](args)
    finally:
        Engine.shutdown()


if __name__ == "__main__":
    sys.exit(main())
