"""Inference throughput (BASELINE.json config 4: Inception-v3 through the Caffe loader, int8 path replacing
DL-Boost) on N GPUs of one node, one process per GPU (data-parallel inference, reference Predictor /
DistriValidator: the model is broadcast once and every rank scores its own batches).

    python tools/bench_inference.py --model inception_v3 --mode int8 [--caffe 1] [--batch 256 --steps 20]

Pipeline: build the model (random-init weights of that architecture), optionally persist it as
prototxt + caffemodel and load it back through ``Module.loadCaffeModel`` (the reference's Caffe path), then
  bf16: lower through the engine-neutral IR to the GPU engine (BN folded into conv, ReLU in conv epilogues);
  int8: ``quantize()`` (BN folded, per-channel int8 weights, per-sample int8 activations, i8 MFMA convs).
Prints one JSON line (rank 0): images/sec for the whole job.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(name):
    from bigdl_amd.models.inception import Inception_v3
    from bigdl_amd.models.resnet import DatasetType, ResNet

    if name == "inception_v3":
        return Inception_v3(1000), 299
    if name == "resnet50":
        return ResNet(1000, 50, dataSet=DatasetType.ImageNet), 224
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--mode", default="int8", choices=["int8", "bf16"])
    ap.add_argument("--caffe", type=int, default=1, help="round-trip the model through prototxt + caffemodel")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--calibrate", type=int, default=1, help="int8: calibrated static activation ranges")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from bigdl_amd.utils.engine import Engine

    Engine.init(master=f"local[{world}]", dist=world > 1)
    from bigdl_amd.nn.module import Module
    from bigdl_amd.utils.intermediate import ConversionUtils
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(7)
    model, side = build(args.model)
    model.evaluate()
    if args.caffe:
        d = tempfile.mkdtemp(prefix=f"caffe_{rank}_")
        proto, weights = os.path.join(d, "net.prototxt"), os.path.join(d, "net.caffemodel")
        model.saveCaffe(proto, weights, overwrite=True)
        model = Module.loadCaffeModel(proto, weights)
        model.evaluate()
    if args.mode == "int8":
        from bigdl_amd.quantized.quantizer import quantize

        model = model.to(dev)
        calib = torch.randn(8, 3, side, side, device=dev) if args.calibrate else None
        model = quantize(model, calibration=calib)
    else:
        model = ConversionUtils.convert(model, "dnn", device=dev, train=False)
    B = args.batch
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    x = torch.randn(B, 3, side, side, device=dev, generator=g)

    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            out = model.forward(x)
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = model.forward(x)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ips = B * world * args.steps / dt
    if rank == 0:
        print(json.dumps({
            "metric": f"images/sec (whole node) {args.model} inference", "value": round(ips, 1),
            "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.mode, "data": "synthetic images; random-init weights",
            "config": {"model": args.model, "global_batch": B * world, "image": side, "parallelism": f"dp{world}",
                       "caffe_loader": bool(args.caffe), "calibrated": bool(args.calibrate and args.mode == "int8"),
                       "out_shape": list(out.shape)},
        }), flush=True)
    Engine.shutdown()


if __name__ == "__main__":
    main()
