"""Save a model as a TensorFlow GraphDef, load it back as a BigDL graph, and check both agree.

Reference: S/example/tensorflow/loadandsave (Save.scala: ``model.saveTF(inputs, path)``; Load.scala:
``Module.loadTF(path, inputs, outputs)`` then forward) — the TensorFlow interop round trip.
"""
import argparse
import os
import tempfile

import torch

from .. import nn
from ..nn.module import Module


def build_model():
    """LeNet-style classifier in TensorFlow's NHWC layout (the reference example's LeNet)."""
    torch.manual_seed(0)
    return (nn.Sequential().add(nn.SpatialConvolution(1, 6, 5, 5, format="NHWC")).add(nn.Tanh())
            .add(nn.SpatialMaxPooling(2, 2, 2, 2, format="NHWC")).add(nn.Reshape([12 * 12 * 6]))
            .add(nn.Linear(12 * 12 * 6, 10)).add(nn.SoftMax()))


def run(args):
    from ..interop.tensorflow import parse_graph

    model = build_model()
    model.evaluate()
    with tempfile.TemporaryDirectory() as d:
        path = args.path or os.path.join(d, "model.pb")
        out = model.saveTF([("input", [None, 28, 28, 1])], path)
        nodes = len(parse_graph(path))
        loaded = Module.loadTF(path, ["input"], [out])
    x = torch.randn(args.batch, 28, 28, 1)
    a = model.forward(x)
    b = loaded.forward(x)
    return {"nodes": nodes, "output": out, "max_abs_diff": float((a - b).abs().max())}


def build_parser():
    p = argparse.ArgumentParser(prog="tfloadandsave")
    p.add_argument("--path", default=None)
    p.add_argument("--batch", type=int, default=4)
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
