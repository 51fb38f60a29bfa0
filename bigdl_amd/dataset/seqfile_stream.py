"""SequenceFile ImageNet stream for GPU training: native record index + parallel gather on the host, resized crop /
flip / normalise on the device.

Reference: the ImageNet training input of the reference reads Hadoop SequenceFiles of pre-scaled BGR records
(S/dataset/DataSet.scala SeqFileFolder.filesToImageFrame / files, S/models/utils/ImageNetSeqFileGenerator), then
runs the per-image host chain BGRImgCropper -> HFlip -> BGRImgNormalizer -> MTLabeledBGRImgToBatch on a thread
pool (S/dataset/image/MTLabeledBGRImgToBatch.scala). MI355X design:
  * every .seq file is read once into one uint8 tensor and indexed in C++ (``_C.seqfile_index``: pixel offset,
    height, width, label per record) — no per-record Python;
  * a batch is a gather of the chosen records' raw BGR bytes into one pinned staging buffer by the native thread
    pool with the GIL released (``_C.gather_bytes``), plus one float32 parameter row per image (crop box, flip)
    drawn vectorised on the host;
  * the device feed (optim/device_feed.py) copies the staging buffer to the GPU on its copy stream and
    ``on_device`` turns it into the training batch with ONE kernel launch (csrc/image.hip: resized crop, flip,
    BGR->RGB, normalisation, fp32 NCHW) — the host never touches a float pixel.
Records are sharded over ranks (record i belongs to rank i % world), so each rank reads its own 1/world of the
data per epoch, and the per-rank batch is batchSize / world as in the reference's distributed dataset.
"""
import math

import numpy as np
import torch

from ..ops import native
from .core import MiniBatch

_NP = 16   # parameter row width of the image_pipeline kernel (dataset/device_pipeline.py)


class RawImageMiniBatch(MiniBatch):
    """A batch still in raw form: input = [flat uint8 BGR bytes, int64 byte offsets, float32 [N, 16] params],
    target = labels. ``on_device()`` (called by the device feed after the host->device copy) returns the training
    MiniBatch of normalised fp32 NCHW crops."""

    def __init__(self, input, target=None, cfg=None):
        super().__init__(input, target)
        self.cfg = cfg

    def size(self):
        return int(self.input[1].shape[0])

    def rebuild(self, input, target):
        return RawImageMiniBatch(input, target, self.cfg)

    def on_device(self):
        flat, offs, prm = self.input
        oh, ow, mean, std, to_rgb = self.cfg
        n = offs.shape[0]
        if flat.is_cuda:
            out = torch.empty(n, 3, oh, ow, dtype=torch.float32, device=flat.device)
            native.get().image_pipeline(flat, offs, prm, out, list(mean), list(std), bool(to_rgb))
            return MiniBatch(out, self.target)
        return MiniBatch(_host_pipeline(flat, offs, prm, oh, ow, mean, std, to_rgb), self.target)


def _host_pipeline(flat, offs, prm, oh, ow, mean, std, to_rgb):
    """CPU engine: the same resized crop / flip / normalisation with the host transformer math."""
    from ..transform.vision.image.augmentation import _resize

    out = torch.empty(offs.shape[0], 3, oh, ow)
    m = torch.tensor(mean)
    s = torch.tensor(std)
    for i in range(offs.shape[0]):
        H, W, y0, x0, ch, cw, flip = (int(v) for v in prm[i, :7].tolist())
        o = int(offs[i])
        img = flat[o:o + H * W * 3].reshape(H, W, 3).float()[y0:y0 + ch, x0:x0 + cw]
        img = _resize(img, ow, oh)
        if flip:
            img = img.flip(1)
        if to_rgb:
            img = img[..., [2, 1, 0]]
        out[i] = ((img - m) / s).permute(2, 0, 1)
    return out


class SeqFileImageStream:
    """DataSet of BGR image SequenceFiles for ``Optimizer``: ``data(train=True)`` yields RawImageMiniBatches
    forever (reshuffled every epoch), ``data(train=False)`` one pass of centre crops.

    ``paths``: .seq files (``SeqFileFolder.paths(folder)``); ``batchSize``: global batch; ``crop``: (h, w);
    ``area`` / ``aspect``: random-resized-crop ranges (area=(1, 1), aspect=(1, 1) with ``scale_crop=False`` gives
    the reference's fixed-size BGRImgCropper crop); ``threads``: native gather threads."""

    def __init__(self, paths, batchSize, crop=(224, 224), mean=(123.68, 116.78, 103.94), std=(58.4, 57.1, 57.4),
                 to_rgb=True, area=(0.08, 1.0), aspect=(3.0 / 4.0, 4.0 / 3.0), scale_crop=True, flip_prob=0.5,
                 threads=8, classNum=None, seed=1, rank=None, world=None, pin=None):
        if rank is None or world is None:
            from ..utils.engine import Engine

            rank = Engine.rank() if rank is None else rank
            world = Engine.world_size() if world is None else world
        self.rank, self.world = int(rank), max(1, int(world))
        if batchSize % self.world:
            raise ValueError(f"batchSize {batchSize} is not a multiple of the {self.world} ranks")
        self.batch = batchSize // self.world
        self.crop = (int(crop[0]), int(crop[1]))
        self.cfg = (self.crop[0], self.crop[1], tuple(float(v) for v in mean), tuple(float(v) for v in std),
                    bool(to_rgb))
        self.area, self.aspect, self.scale_crop, self.flip_prob = area, aspect, scale_crop, flip_prob
        self.threads = int(threads)
        self.pin = torch.cuda.is_available() if pin is None else bool(pin)
        self.gen = torch.Generator().manual_seed(int(seed) * 1000003 + self.rank)
        C = native.get()
        bufs, recs, labs, fids = [], [], [], []
        for i, p in enumerate(paths):
            b = torch.from_numpy(np.fromfile(p, dtype=np.uint8))
            r, lab = C.seqfile_index(b)
            bufs.append(b)
            recs.append(r)
            labs.append(lab)
            fids.append(torch.full((r.shape[0],), i, dtype=torch.int64))
        if not bufs:
            raise ValueError("SeqFileImageStream: no files")
        self.bufs = bufs
        rec = torch.cat(recs)
        lab = torch.cat(labs)
        fid = torch.cat(fids)
        keep = torch.ones(rec.shape[0], dtype=torch.bool) if classNum is None else lab <= classNum
        small = (rec[:, 1] < self.crop[0]) | (rec[:, 2] < self.crop[1])
        if bool((keep & small).any()) and not scale_crop:
            raise ValueError("a record is smaller than the fixed crop")
        mine = torch.arange(rec.shape[0]) % self.world == self.rank
        sel = keep & mine
        self.rec, self.lab, self.fid = rec[sel], lab[sel], fid[sel]
        self.total = int(keep.sum())

    def size(self):
        return self.total

    def shuffle(self):
        pass

    # ------------------------------------------------------------------------------------------------ params
    def _params(self, H, W, train):
        """Vectorised crop boxes: Inception random-resized crop (10 tries, centre square fallback) or the fixed
        random / centre crop of the reference's BGRImgCropper."""
        n = H.shape[0]
        Hf, Wf = H.double(), W.double()
        ch, cw = self.crop
        if train and self.scale_crop:
            t = torch.empty(10, n, dtype=torch.float64)
            target = t.uniform_(self.area[0], self.area[1], generator=self.gen) * Hf * Wf
            logr = torch.empty(10, n, dtype=torch.float64).uniform_(math.log(self.aspect[0]), math.log(self.aspect[1]),
                                                                    generator=self.gen)
            r = logr.exp()
            cws = (target * r).sqrt().round()
            chs = (target / r).sqrt().round()
            ok = (cws > 0) & (chs > 0) & (cws <= Wf) & (chs <= Hf)
            first = torch.where(ok.any(0), ok.double().argmax(0), torch.full((n,), -1, dtype=torch.int64))
            idx = first.clamp(min=0)
            bw = cws.gather(0, idx[None])[0]
            bh = chs.gather(0, idx[None])[0]
            s = torch.minimum(Hf, Wf)
            bh = torch.where(first >= 0, bh, s)
            bw = torch.where(first >= 0, bw, s)
            u = torch.rand(2, n, dtype=torch.float64, generator=self.gen)
            y0 = torch.where(first >= 0, (u[0] * (Hf - bh + 1e-9)).floor(), ((Hf - s) / 2).floor())
            x0 = torch.where(first >= 0, (u[1] * (Wf - bw + 1e-9)).floor(), ((Wf - s) / 2).floor())
            y0 = torch.minimum(y0, Hf - bh)
            x0 = torch.minimum(x0, Wf - bw)
        else:
            bh = torch.full((n,), float(ch), dtype=torch.float64).minimum(Hf)
            bw = torch.full((n,), float(cw), dtype=torch.float64).minimum(Wf)
            if train:
                u = torch.rand(2, n, dtype=torch.float64, generator=self.gen)
                y0 = (u[0] * (Hf - bh + 1)).floor().minimum(Hf - bh)
                x0 = (u[1] * (Wf - bw + 1)).floor().minimum(Wf - bw)
            else:
                y0, x0 = ((Hf - bh) / 2).floor(), ((Wf - bw) / 2).floor()
        flip = (torch.rand(n, generator=self.gen) < self.flip_prob) if train else torch.zeros(n, dtype=torch.bool)
        prm = torch.zeros(n, _NP, dtype=torch.float32)
        prm[:, 0], prm[:, 1] = H.float(), W.float()
        prm[:, 2], prm[:, 3], prm[:, 4], prm[:, 5] = y0.float(), x0.float(), bh.float(), bw.float()
        prm[:, 6] = flip.float()
        return prm

    # ------------------------------------------------------------------------------------------------ batches
    def _batch(self, ids, train):
        C = native.get()
        rec, fid = self.rec[ids], self.fid[ids]
        nbytes = rec[:, 1] * rec[:, 2] * 3
        dst = torch.zeros_like(nbytes)
        if ids.numel() > 1:
            dst[1:] = nbytes[:-1].cumsum(0)
        total = int(nbytes.sum())
        flat = torch.empty(total, dtype=torch.uint8, pin_memory=self.pin)
        for f in fid.unique().tolist():
            m = fid == f
            C.gather_bytes(self.bufs[f], rec[m, 0].contiguous(), nbytes[m].contiguous(), dst[m].contiguous(), flat,
                           self.threads)
        prm = self._params(rec[:, 1], rec[:, 2], train)
        return RawImageMiniBatch([flat, dst, prm], self.lab[ids].clone(), self.cfg)

    def data(self, train=True):
        n = self.rec.shape[0]
        if n == 0:
            return
        bs = min(self.batch, n)
        while True:
            order = torch.randperm(n, generator=self.gen) if train else torch.arange(n)
            starts = range(0, n - bs + 1, bs) if train else range(0, n, bs)    # training drops the partial tail
            for b0 in starts:
                yield self._batch(order[b0:b0 + bs], train)
            if not train:
                return


__all__ = ["SeqFileImageStream", "RawImageMiniBatch"]
