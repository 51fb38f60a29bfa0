"""Load a pre-trained model from any supported format and validate it on an image folder.

Reference: S/example/loadmodel/ModelValidator.scala (``--modelType`` caffe / torch / bigdl, ``--caffeDefPath``,
``--modelPath``, ``--folder``, ``--batchSize``; ImageNet-style preprocessing per model family in DatasetUtil.scala;
Top1 / Top5 accuracy through the Validator) and the int8 path of S/example/mkldnn/int8 (calibrated quantization
of the loaded model).

``--engine``: ``blas`` runs the loaded module as is; ``dnn`` lowers it through the IR to the fused GPU graph
(BatchNorm / Scale folding, residual and concat fusion); ``int8`` quantizes it with calibrated static scales and
attaches the int8 execution plan. Without ``--folder`` the model is built from the zoo (``--model``), exported /
re-imported through ``--modelType``, and validated on synthetic images (accuracy is then chance; the run checks the
pipeline and reports throughput).
"""
import argparse
import os
import tempfile
import time

import torch

from ..dataset.core import DataSet, Sample
from ..nn.module import Module
from ..optim import Top1Accuracy, Top5Accuracy
from ..optim.evaluator import evaluate_dataset
from ._common import device_of

MEAN = {"inception": (0.5, 0.5, 0.5), "default": (0.485, 0.456, 0.406)}
STD = {"inception": (0.5, 0.5, 0.5), "default": (0.229, 0.224, 0.225)}


def zoo(name, classes):
    from ..models.inception import Inception_v1, Inception_v3
    from ..models.resnet import DatasetType, ResNet
    from ..models.vgg import Vgg_16

    if name == "resnet50":
        return ResNet(classes, 50, dataSet=DatasetType.ImageNet), 224
    if name == "inception_v1":
        return Inception_v1(classes), 224
    if name == "inception_v3":
        return Inception_v3(classes), 299
    if name == "vgg16":
        return Vgg_16(classes), 224
    raise ValueError(name)


def load(args, model=None):
    t = args.modelType
    if t == "bigdl":
        return Module.loadModule(args.modelPath)
    if t == "caffe":
        return Module.loadCaffeModel(args.caffeDefPath, args.modelPath)
    if t == "torch":
        return Module.loadTorch(args.modelPath)
    if t == "tf":
        return Module.loadTF(args.modelPath, args.tfInputs.split(","), args.tfOutputs.split(","))
    raise ValueError(t)


def export(model, args, d):
    """Write the zoo model in the requested format (to exercise the loader end to end)."""
    if args.modelType == "bigdl":
        args.modelPath = os.path.join(d, "model.bigdl")
        model.saveModule(args.modelPath, overWrite=True)
    elif args.modelType == "caffe":
        args.caffeDefPath, args.modelPath = os.path.join(d, "net.prototxt"), os.path.join(d, "net.caffemodel")
        model.saveCaffe(args.caffeDefPath, args.modelPath, overwrite=True)
    elif args.modelType == "torch":
        args.modelPath = os.path.join(d, "model.t7")
        model.saveTorch(args.modelPath, overWrite=True)
    else:
        raise ValueError(f"cannot export the zoo model as {args.modelType}")


def image_samples(folder, side, family, limit=None):
    from ..dataset.image import LocalImageFiles, read_image

    mean = torch.tensor(MEAN.get(family, MEAN["default"])).view(3, 1, 1)
    std = torch.tensor(STD.get(family, STD["default"])).view(3, 1, 1)
    out = []
    for p in LocalImageFiles.readPaths(folder)[:limit]:
        img = read_image(p.path, resizeW=side, resizeH=side).float() / 255.0      # HWC BGR
        x = img[..., [2, 1, 0]].permute(2, 0, 1)
        out.append(Sample((x - mean) / std, torch.tensor([float(p.label)])))
    return out


def run(args):
    dev = device_of(args.device)
    classes = args.classNum
    model, side = zoo(args.model, classes)
    model.evaluate()
    with tempfile.TemporaryDirectory() as d:
        if not args.modelPath:
            export(model, args, d)
        loaded = load(args)
    loaded.evaluate()
    if args.folder:
        data = image_samples(args.folder, side, "inception" if "inception" in args.model else "default", args.limit)
    else:
        g = torch.Generator().manual_seed(0)
        data = [Sample(torch.randn(3, side, side, generator=g), torch.tensor([float(1 + i % classes)]))
                for i in range(args.limit or 2 * args.batchSize)]
    if args.engine == "dnn":
        from ..utils.intermediate import ConversionUtils

        net = ConversionUtils.convert(loaded, "dnn", device=dev, train=False)
    elif args.engine == "int8":
        from ..quantized.quantizer import quantize

        calib = torch.stack([s.feature() for s in data[:min(len(data), 16)]]).to(dev)
        net = quantize(loaded.to(dev), calibration=calib)
    else:
        net = loaded.to(dev)
    t0 = time.perf_counter()
    res = evaluate_dataset(net, DataSet.array(data), [Top1Accuracy(), Top5Accuracy()], args.batchSize, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"images": len(data), "top1": res[0].result()[0], "top5": res[1].result()[0],
            "images_per_sec": len(data) / dt, "engine": args.engine}


def build_parser():
    p = argparse.ArgumentParser(prog="loadmodel")
    p.add_argument("--modelType", choices=["bigdl", "caffe", "torch", "tf"], default="caffe")
    p.add_argument("--modelPath", default=None)
    p.add_argument("--caffeDefPath", default=None)
    p.add_argument("--tfInputs", default="input")
    p.add_argument("--tfOutputs", default="output")
    p.add_argument("--model", default="resnet50", help="zoo architecture (when no --modelPath is given)")
    p.add_argument("--classNum", type=int, default=1000)
    p.add_argument("--folder", default=None)
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--limit", type=int, default=None)
    p.add_argument("--engine", choices=["blas", "dnn", "int8"], default="dnn")
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
