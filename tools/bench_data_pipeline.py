"""ImageNet-from-SeqFile input throughput on one GPU (dataset/seqfile_stream.py + optim/device_feed.py).

Writes synthetic SequenceFiles of BGR records shaped like the reference's ImageNet SeqFile generator output (short
side 256, long side 256-400, random pixels, labels 1..1000), then measures:
  host      : native index + pinned gather + crop-parameter draws, images/s per gather-thread count
  feed      : host + host->device copy + the preprocessing kernel (DeviceFeed, no training), images/s
  train     : Optimizer.optimize() on ResNet-50 b256 fed by the stream, images/s over the timed iterations
and the number of host gather threads 8 such GPUs need. One JSON line."""
import argparse
import json
import math
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_files(root, n, per_file, seed=0):
    from bigdl_amd.dataset.image import encode_bgr_record
    from bigdl_amd.dataset.seqfile import SequenceFileWriter

    g = torch.Generator().manual_seed(seed)
    paths = []
    for f in range((n + per_file - 1) // per_file):
        p = os.path.join(root, f"imagenet_{f}.seq")
        with SequenceFileWriter(p) as w:
            for i in range(min(per_file, n - f * per_file)):
                long = int(torch.randint(256, 401, (1,), generator=g))
                h, wd = (256, long) if i % 2 else (long, 256)
                im = torch.randint(0, 256, (h, wd, 3), generator=g, dtype=torch.uint8)
                w.append(f"{1 + (f * per_file + i) % 1000}", encode_bgr_record(im))
        paths.append(p)
    return paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=1536)
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--train-iters", type=int, default=10)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--feed-threads", default="8,16", help="gather threads of the host -> device feed runs")
    a = ap.parse_args()
    from bigdl_amd.dataset.seqfile_stream import SeqFileImageStream
    from bigdl_amd.optim.device_feed import DeviceFeed

    tmp = tempfile.mkdtemp(prefix="bigdl_seq_")
    t0 = time.perf_counter()
    paths = write_files(tmp, a.images, 512)
    gen_s = time.perf_counter() - t0
    mb_bytes = sum(os.path.getsize(p) for p in paths)
    res = {"images": a.images, "seqfile_MB": round(mb_bytes / 2**20, 1), "write_s": round(gen_s, 1)}
    B = 256
    host = {}
    t0 = time.perf_counter()
    ds = SeqFileImageStream(paths, B, threads=1, rank=0, world=1)
    res["index_s"] = round(time.perf_counter() - t0, 3)
    for T in [int(v) for v in a.threads.split(",")]:
        ds.threads = T
        it = ds.data(train=True)
        next(it)
        t0 = time.perf_counter()
        nb = 8
        for _ in range(nb):
            next(it)
        host[T] = round(nb * B / (time.perf_counter() - t0), 1)
        print(f"host threads={T}: {host[T]} img/s", file=sys.stderr, flush=True)
    res["host_img_s_by_threads"] = host
    # feed: host (T threads) -> pinned -> H2D on the copy stream -> preprocessing kernel
    res["feed_img_s_by_threads"] = {}
    for T in [int(v) for v in a.feed_threads.split(",")]:
        ds.threads = T
        feed = DeviceFeed(iter(ds.data(train=True)), torch.device("cuda"))
        next(feed)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nb = 16
        for _ in range(nb):
            mb = next(feed)
        torch.cuda.synchronize()
        res["feed_img_s_by_threads"][T] = round(nb * B / (time.perf_counter() - t0), 1)
        res["feed_batch"] = list(mb.getInput().shape)
        feed.close()
        print(f"feed threads={T}: {res['feed_img_s_by_threads'][T]} img/s", file=sys.stderr, flush=True)
    res["feed_img_s"] = max(res["feed_img_s_by_threads"].values())
    ds.threads = 8
    if not a.no_train:
        from bigdl_amd import nn
        from bigdl_amd.models.resnet import DatasetType, ResNet
        from bigdl_amd.optim.optimizer import Optimizer
        from bigdl_amd.optim.sgd import SGD
        from bigdl_amd.optim.trigger import Trigger
        from bigdl_amd.utils.engine import Engine

        Engine.init(master="local[1]", dist=False)
        model = ResNet(1000, 50, dataSet=DatasetType.ImageNet)
        W, K = 6, a.train_iters
        marks = {}

        def hook(neval):
            if neval in (W, W + K):
                torch.cuda.synchronize()
                marks[neval] = time.perf_counter()

        opt = Optimizer(model, ds, nn.CrossEntropyCriterion(), batchSize=None,
                        optimMethod=SGD(learningRate=0.1, momentum=0.9, dampening=0.0),
                        endTrigger=Trigger.maxIteration(W + K))
        opt.device = torch.device("cuda", 0)
        opt._iteration_hook = hook
        opt.optimize()
        dt = marks[W + K] - marks[W]
        res["train_img_s"] = round(K * B / dt, 1)
        res["train_ms_per_step"] = round(dt / K * 1e3, 3)
        res["train_loss"] = float(opt.state.get("Loss", float("nan")))
        res["graph_vs_eager"] = getattr(opt, "graph_decision", None)
        per_thread = max(v / k for k, v in host.items())
        res["host_img_s_per_thread_best"] = round(per_thread, 1)
        res["gather_threads_for_8_gpus"] = math.ceil(8 * res["train_img_s"] / per_thread)
    for p in paths:
        os.remove(p)
    os.rmdir(tmp)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
