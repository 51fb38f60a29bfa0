"""DataFrame transfer learning on images: a pre-trained network embeds every image, a small classifier is fitted on
the embeddings.

Reference: S/example/dlframes/imageTransferLearning/ImageTransferLearning.scala (DLImageReader -> DLImageTransformer
(resize, centre crop, normalise, to tensor) -> DLModel(pre-trained Inception) producing an "embedding" column ->
DLClassifier(Linear + LogSoftMax) fitted on it -> accuracy on a held-out split). Without ``--folder`` a two-class
synthetic image folder (reddish vs bluish images) is written first; the embedding network is random-initialised
unless ``--modelPath`` names a saved model.
"""
import argparse
import os
import tempfile

import numpy as np
import torch


def _write_two_classes(d, n=16, side=24):
    from PIL import Image

    rng = np.random.RandomState(0)
    for i in range(n):
        img = rng.randint(0, 80, (side, side, 3)).astype(np.uint8)
        img[..., 0 if i % 2 == 0 else 2] += 150            # RGB: class 1 red, class 2 blue
        Image.fromarray(img).save(os.path.join(d, f"{'red' if i % 2 == 0 else 'blue'}_{i}.png"))


def _embedder(side):
    from .. import nn

    torch.manual_seed(0)
    return (nn.Sequential().add(nn.SpatialConvolution(3, 16, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
            .add(nn.SpatialAveragePooling(side, side, 1, 1)).add(nn.View(16).setNumInputDims(3)))


def run(args):
    import pandas as pd

    from .. import nn
    from ..dlframes import DLClassifier, DLImageReader, DLImageTransformer, DLModel
    from ..transform.vision.image import CenterCrop, ChannelNormalize, MatToTensor, Resize

    tmp = None
    folder = args.folder
    if folder is None:
        tmp = tempfile.TemporaryDirectory()
        folder = tmp.name
        _write_two_classes(folder)
    side = args.imageSize
    df = DLImageReader.readImages(folder)
    chain = Resize(side + 4, side + 4) >> CenterCrop(side, side) >> \
        ChannelNormalize(123.0, 117.0, 104.0, 58.0, 57.0, 57.0) >> MatToTensor()
    feats = DLImageTransformer(chain).setInputCol("image").setOutputCol("features").transform(df)
    if args.modelPath:
        from ..nn.module import Module

        net = Module.loadModule(args.modelPath)
    else:
        net = _embedder(side)
    net.evaluate()
    emb = DLModel(net, [3, side, side]).setFeaturesCol("features").setPredictionCol("embedding").transform(feats)
    names = [os.path.basename(r["origin"]) for r in emb["image"]]
    labels = [1.0 if n.startswith("red") else 2.0 for n in names]
    data = pd.DataFrame({"embedding": [np.asarray(e, dtype=np.float32) for e in emb["embedding"]], "label": labels})
    train, test = data.iloc[::2].reset_index(drop=True), data.iloc[1::2].reset_index(drop=True)
    dim = len(data["embedding"][0])
    torch.manual_seed(0)
    clf = DLClassifier(nn.Sequential().add(nn.Linear(dim, 2)).add(nn.LogSoftMax()), nn.ClassNLLCriterion(), [dim]) \
        .setFeaturesCol("embedding").setBatchSize(4).setMaxEpoch(args.maxEpoch).setLearningRate(0.1)
    out = clf.fit(train).transform(test)
    acc = float((np.asarray(out["prediction"], dtype=np.float32) == np.asarray(test["label"])).mean())
    if tmp is not None:
        tmp.cleanup()
    return {"images": len(names), "embedding_dim": dim, "test_accuracy": acc}


def build_parser():
    p = argparse.ArgumentParser(prog="imagetransferlearning")
    p.add_argument("--folder", default=None)
    p.add_argument("--modelPath", default=None)
    p.add_argument("--imageSize", type=int, default=24)
    p.add_argument("--maxEpoch", type=int, default=20)
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
