"""Int8 inference: generate calibrated activation scales, then run the quantized model and compare with fp32.

Reference: S/example/mkldnn/int8/GenerateInt8Scales.scala (``model.calcScales(batch)`` over calibration images, the
model saved with its scales) and ImageNetInference.scala (the scaled model converted to int8 and validated with
Top-1 / Top-5). Here the scales are written as JSON (layer name -> input range), applied with ``setInputScales``
and consumed by ``quantize`` (static per-tensor ranges; on the GPU the i8-MFMA kernels of csrc/quant.hip).

    python -m bigdl_amd.examples int8 --mode genscales --scales scales.json
    python -m bigdl_amd.examples int8 --mode inference --scales scales.json
    python -m bigdl_amd.examples int8 --mode both                      (default: both in one run)
"""
import argparse
import json
import os
import tempfile

import torch

from ._common import device_of


def _model_and_data(args, dev):
    from ..models.cli import build_model

    if args.modelPath:
        from ..nn.module import Module

        model = Module.loadModule(args.modelPath)
        shape = (3, args.imageSize, args.imageSize)
    else:
        torch.manual_seed(0)
        model, shape = build_model("resnet", args.classNum, 20)
    g = torch.Generator().manual_seed(1)
    calib = torch.randn((args.calibSize,) + tuple(shape), generator=g)
    val = torch.randn((args.valSize,) + tuple(shape), generator=g)
    model.evaluate()
    return model.to(dev), calib.to(dev), val.to(dev)


def generate_scales(model, calib, path):
    from ..quantized.quantizer import REGISTRY

    probe = model.cloneModule()
    probe.calcScales(calib)
    scales = {m.getName(): m.getInputScales() for m in probe.flattened_layers()
              if type(m) in REGISTRY and m.getInputScales()}
    with open(path, "w") as f:
        json.dump(scales, f, indent=1)
    return scales


def int8_inference(model, scales_path, val, batch):
    from ..quantized.quantizer import quantize

    with open(scales_path) as f:
        scales = json.load(f)
    for m in model.flattened_layers():
        if m.getName() in scales:
            m.setInputScales(scales[m.getName()])
    q = quantize(model)
    with torch.no_grad():
        ref = torch.cat([model.forward(val[i:i + batch]).float() for i in range(0, val.shape[0], batch)])
        out = torch.cat([q.forward(val[i:i + batch]).float() for i in range(0, val.shape[0], batch)])
    top1_ref, top1_q = ref.argmax(1), out.argmax(1)
    top5_q = out.topk(min(5, out.shape[1]), 1).indices
    return {"top1_agreement": float((top1_ref == top1_q).float().mean()),
            "top5_contains_fp32_top1": float((top5_q == top1_ref[:, None]).any(1).float().mean()),
            "rel_output_error": float((out - ref).norm() / ref.norm())}


def run(args):
    dev = device_of(args.device)
    model, calib, val = _model_and_data(args, dev)
    tmp = None
    path = args.scales
    if path is None:
        tmp = tempfile.TemporaryDirectory()
        path = os.path.join(tmp.name, "scales.json")
    out = {}
    if args.mode in ("genscales", "both"):
        out["layers_with_scales"] = len(generate_scales(model, calib, path))
    if args.mode in ("inference", "both"):
        out.update(int8_inference(model, path, val, args.batchSize))
    if tmp is not None:
        tmp.cleanup()
    return out


def build_parser():
    p = argparse.ArgumentParser(prog="int8")
    p.add_argument("--mode", choices=["genscales", "inference", "both"], default="both")
    p.add_argument("--modelPath", default=None)
    p.add_argument("--scales", default=None, help="scales JSON written by genscales / read by inference")
    p.add_argument("--imageSize", type=int, default=224)
    p.add_argument("--classNum", type=int, default=10)
    p.add_argument("--calibSize", type=int, default=16)
    p.add_argument("--valSize", type=int, default=32)
    p.add_argument("--batchSize", type=int, default=16)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
