"""Throughput of the device image pipeline (dataset/device_pipeline.py) on an ImageNet-shaped batch: 256 decoded
BGR images of 500x375 / 375x500 / 400x400, random-resized crop to 224, flip, full colour jitter, normalise, fp32
NCHW. Reports the kernel-only time (batch already resident), the end-to-end call (pack + H2D + kernel) and the host
transformer chain for a few images (extrapolated per batch)."""
import json
import time

import torch

from bigdl_amd.dataset.device_pipeline import DeviceImagePipeline
from bigdl_amd.ops import native
from bigdl_amd.utils.random_generator import RNG


def main():
    RNG.setSeed(1)
    shapes = [(500, 375, 3), (375, 500, 3), (400, 400, 3)]
    imgs = [torch.randint(0, 256, shapes[i % 3], dtype=torch.uint8) for i in range(256)]
    pipe = DeviceImagePipeline(224, 224, (123.68, 116.78, 103.94), (58.4, 57.1, 57.4))
    jit = dict(brightnessProb=1.0, contrastProb=1.0, saturationProb=1.0, hueProb=1.0)
    params = pipe.random_params([im.shape for im in imgs], jitter=jit)
    out = pipe(imgs, params)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        out = pipe(imgs, params)
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t) / 5 * 1e3
    # kernel only: reuse device-resident inputs
    flat = torch.cat([im.reshape(-1) for im in imgs]).cuda()
    offs = torch.tensor([0] + [im.numel() for im in imgs[:-1]]).cumsum(0).cuda()
    prm = torch.zeros(256, 16)
    for i, (im, p) in enumerate(zip(imgs, params)):
        row = [im.shape[0], im.shape[1], p.y0, p.x0, p.ch, p.cw, float(p.flip), len(p.ops)]
        for c, a in p.ops:
            row += [c, a]
        prm[i, :len(row)] = torch.tensor(row)
    prm = prm.cuda()
    C = native.get()
    C.image_pipeline(flat, offs, prm, out, pipe.mean, pipe.std, True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        C.image_pipeline(flat, offs, prm, out, pipe.mean, pipe.std, True)
    e.record()
    torch.cuda.synchronize()
    kern = s.elapsed_time(e) / 20
    t = time.perf_counter()
    for i in range(4):
        pipe.host_reference(imgs[i], params[i])
    host = (time.perf_counter() - t) / 4 * 256 * 1e3
    print(json.dumps({"batch": 256, "out": "3x224x224 fp32", "kernel_ms": round(kern, 3),
                      "end_to_end_ms": round(e2e, 2), "host_chain_ms_per_batch_1thread": round(host, 1),
                      "kernel_images_per_s": round(256 / kern * 1e3)}))


if __name__ == "__main__":
    main()
