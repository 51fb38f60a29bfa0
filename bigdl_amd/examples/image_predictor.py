"""Predict the class of every image in a folder with a DataFrame pipeline.

Reference: S/example/imageclassification/ImagePredictor.scala (DLImageReader.readImages -> DLImageTransformer
(resize / crop / normalise) -> DLClassifierModel.transform, showing the predicted label per file) and
S/example/dlframes/imageInference.

Without ``--folder`` a few synthetic images are written to a temporary directory first.
"""
import argparse
import os
import tempfile

import numpy as np
import torch

from ._common import device_of


def _write_synthetic(d, n=6, side=40):
    from PIL import Image

    rng = np.random.RandomState(0)
    for i in range(n):
        Image.fromarray(rng.randint(0, 255, (side, side, 3), dtype=np.uint8)).save(os.path.join(d, f"img{i}.png"))


def run(args):
    from ..dlframes import DLClassifierModel, DLImageReader, DLImageTransformer
    from ..models.lenet import LeNet5
    from ..transform.vision.image import ChannelNormalize, MatToTensor, Resize

    dev = device_of(args.device)
    tmp = None
    folder = args.folder
    if folder is None:
        tmp = tempfile.TemporaryDirectory()
        folder = tmp.name
        _write_synthetic(folder)
    side = args.imageSize
    df = DLImageReader.readImages(folder)
    chain = Resize(side, side) >> ChannelNormalize(123.0, 117.0, 104.0, 58.0, 57.0, 57.0) >> MatToTensor()
    tf = DLImageTransformer(chain).setInputCol("image").setOutputCol("features")
    feats = tf.transform(df)
    if args.modelPath:
        from ..nn.module import Module

        model = Module.loadModule(args.modelPath)
    else:
        torch.manual_seed(0)
        model = _small_cnn(side, args.classNum)
    model.evaluate()
    clf = DLClassifierModel(model.to(dev), [3, side, side]).setFeaturesCol("features").setBatchSize(args.batchSize)
    out = clf.transform(feats)
    preds = [(r["origin"], int(p)) for r, p in zip(out["image"], out["prediction"])]
    if tmp is not None:
        tmp.cleanup()
    return {"images": len(preds), "predictions": preds[:5]}


def _small_cnn(side, classes):
    from .. import nn

    return (nn.Sequential().add(nn.SpatialConvolution(3, 8, 3, 3, 2, 2, 1, 1)).add(nn.ReLU())
            .add(nn.SpatialAveragePooling(side // 2, side // 2, 1, 1)).add(nn.View(8).setNumInputDims(3))
            .add(nn.Linear(8, classes)).add(nn.LogSoftMax()))


def build_parser():
    p = argparse.ArgumentParser(prog="imagepredictor")
    p.add_argument("--folder", default=None)
    p.add_argument("--modelPath", default=None)
    p.add_argument("--imageSize", type=int, default=32)
    p.add_argument("--classNum", type=int, default=10)
    p.add_argument("--batchSize", type=int, default=4)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
