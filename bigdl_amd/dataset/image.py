"""Image datasets and transformers (reference S/dataset/image/*: Types.scala, BytesToBGRImg, BytesToGreyImg,
BGRImgCropper, BGRImgRdmCropper, BGRImgNormalizer, BGRImgPixelNormalizer, ColorJitter, Lighting, HFlip,
GreyImgCropper, GreyImgNormalizer, GreyImgToBatch, GreyImgToSample, BGRImgToBatch, BGRImgToSample,
LocalImgReader, LocalImageFiles, MTLabeledBGRImgToBatch).

Images are torch tensors: grey [H, W], BGR [H, W, 3] (interleaved, channel order B, G, R as in the reference).
Every transformer works on whole tensors (no per-pixel loops), so it runs on host tensors in the loader
threads or on device tensors. ``MTLabeledBGRImgToBatch`` assembles batches with a host thread pool (PIL's
decoders release the GIL); ``GpuImageAugment`` (ops/image.py, csrc/image.hip) does crop + flip + normalise +
layout/dtype conversion of a whole uint8 batch in one HIP kernel on the device.
"""
import math
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import torch

from ..utils.random_generator import RNG
from .core import MiniBatch, Sample, Transformer

__all__ = ["ByteRecord", "LocalLabeledImagePath", "GreyImage", "LabeledGreyImage", "BGRImage", "LabeledBGRImage",
           "BytesToGreyImg", "BytesToBGRImg", "GreyImgCropper", "GreyImgNormalizer", "GreyImgToBatch",
           "GreyImgToSample", "BGRImgCropper", "CropRandom", "CropCenter", "BGRImgRdmCropper", "BGRImgNormalizer",
           "BGRImgPixelNormalizer", "HFlip", "ColorJitter", "Lighting", "BGRImgToBatch", "BGRImgToSample",
           "LocalImgReader", "LocalImageFiles", "MTLabeledBGRImgToBatch", "read_image", "GpuImageAugment"]


class ByteRecord:
    def __init__(self, data, label):
        self.data, self.label = data, float(label)


class LocalLabeledImagePath:
    def __init__(self, label, path):
        self.label, self.path = float(label), path


# ---------------------------------------------------------------------------------------------- images
class GreyImage:
    def __init__(self, content=None, width=0, height=0, label=0.0):
        self.content = content if content is not None else torch.zeros(height, width)
        self._label = float(label)

    def width(self):
        return self.content.shape[1]

    def height(self):
        return self.content.shape[0]

    def label(self):
        return self._label

    def setLabel(self, label):
        self._label = float(label)
        return self

    def copy(self, data, normalize=1.0):
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if isinstance(data, (bytes, bytearray)) else data
        self.content = t.reshape(self.height(), self.width()).float() / normalize
        return self


LabeledGreyImage = GreyImage


class BGRImage:
    def __init__(self, content=None, width=0, height=0, label=0.0):
        self.content = content if content is not None else torch.zeros(height, width, 3)
        self._label = float(label)

    def width(self):
        return self.content.shape[1]

    def height(self):
        return self.content.shape[0]

    def label(self):
        return self._label

    def setLabel(self, label):
        self._label = float(label)
        return self

    def hflip(self):
        self.content = self.content.flip(1)
        return self

    def copy(self, data, normalize=1.0):
        """``data``: width(int32 BE) + height(int32 BE) + BGR bytes (the reference's record layout)."""
        if isinstance(data, (bytes, bytearray)):
            w = int.from_bytes(data[0:4], "big")
            h = int.from_bytes(data[4:8], "big")
            t = torch.frombuffer(bytearray(data[8:8 + w * h * 3]), dtype=torch.uint8).reshape(h, w, 3)
        else:
            t = data
        self.content = t.float() / normalize
        return self

    def toTensor(self, toRGB=True):
        """[3, H, W] float (RGB order when ``toRGB``), the layout of BGRImage.copyTo."""
        c = self.content.flip(2) if toRGB else self.content
        return c.permute(2, 0, 1).contiguous()


LabeledBGRImage = BGRImage


def read_image(path, scaleTo=-1, resizeW=-1, resizeH=-1):
    """Decode an image file to a BGR uint8 [H, W, 3] tensor; ``scaleTo`` resizes the short side
    (BGRImage.readImage :371), ``resizeW/H`` resizes to a fixed size (:378)."""
    from PIL import Image

    with Image.open(path) as im:
        im = im.convert("RGB")
        if resizeW > 0 and resizeH > 0:
            im = im.resize((resizeW, resizeH), Image.BILINEAR)
        elif scaleTo > 0:
            w, h = im.size
            if w < h:
                im = im.resize((scaleTo, int(round(h * scaleTo / w))), Image.BILINEAR)
            else:
                im = im.resize((int(round(w * scaleTo / h)), scaleTo), Image.BILINEAR)
        t = torch.frombuffer(bytearray(im.tobytes()), dtype=torch.uint8).reshape(im.size[1], im.size[0], 3)
    return t.flip(2).contiguous()


def encode_bgr_record(img_bgr_uint8):
    """Inverse of BGRImage.copy's record layout."""
    h, w, _ = img_bgr_uint8.shape
    return w.to_bytes(4, "big") + h.to_bytes(4, "big") + bytes(img_bgr_uint8.contiguous().numpy().tobytes())


# ---------------------------------------------------------------------------------------------- converters
class BytesToGreyImg(Transformer):
    def __init__(self, row, col):
        self.row, self.col = row, col

    def apply(self, it):
        for r in it:
            yield GreyImage(width=self.col, height=self.row).copy(r.data, 255.0).setLabel(r.label)


class BytesToBGRImg(Transformer):
    def __init__(self, normalize=255.0, resizeW=-1, resizeH=-1):
        self.normalize, self.resizeW, self.resizeH = normalize, resizeW, resizeH

    def apply(self, it):
        for r in it:
            img = BGRImage().copy(r.data, 1.0)
            if self.resizeW > 0:
                x = img.content.permute(2, 0, 1).unsqueeze(0)
                x = torch.nn.functional.interpolate(x, size=(self.resizeH, self.resizeW), mode="bilinear",
                                                    align_corners=False)
                img.content = x[0].permute(1, 2, 0).round().clamp(0, 255)
            img.content = img.content / self.normalize
            yield img.setLabel(r.label)


# ---------------------------------------------------------------------------------------------- grey
class GreyImgCropper(Transformer):
    def __init__(self, cropWidth, cropHeight):
        self.cw, self.ch = cropWidth, cropHeight

    def apply(self, it):
        for img in it:
            sw = int(RNG.uniform(0, img.width() - self.cw))
            sh = int(RNG.uniform(0, img.height() - self.ch))
            yield GreyImage(img.content[sh:sh + self.ch, sw:sw + self.cw].clone(), label=img.label())


class GreyImgNormalizer(Transformer):
    def __init__(self, mean, std):
        self.mean, self.std = float(mean), float(std)

    @staticmethod
    def fromDataSet(dataSet, samples=2 ** 31 - 1):
        it = dataSet.toLocal().data(False) if hasattr(dataSet, "toLocal") else iter(dataSet)
        n = min(samples, dataSet.size()) if hasattr(dataSet, "size") else samples
        imgs = [next(it).content for _ in range(n)]
        allv = torch.stack(imgs).double()
        return GreyImgNormalizer(allv.mean().item(), allv.std(unbiased=False).item())

    def apply(self, it):
        for img in it:
            yield GreyImage((img.content - self.mean) / self.std, label=img.label())


class GreyImgToSample(Transformer):
    def apply(self, it):
        for img in it:
            yield Sample(img.content.clone(), torch.tensor([img.label()]))


class GreyImgToBatch(Transformer):
    def __init__(self, batchSize):
        self.batchSize = batchSize

    def apply(self, it):
        from .core import SampleToMiniBatch

        bs = SampleToMiniBatch(self.batchSize)._per_rank()
        buf_x, buf_y = [], []
        for img in it:
            buf_x.append(img.content)
            buf_y.append(img.label())
            if len(buf_x) == bs:
                yield MiniBatch(torch.stack(buf_x), torch.tensor(buf_y))
                buf_x, buf_y = [], []
        if buf_x:
            yield MiniBatch(torch.stack(buf_x), torch.tensor(buf_y))


# ---------------------------------------------------------------------------------------------- BGR
CropRandom, CropCenter = "CropRandom", "CropCenter"


class BGRImgCropper(Transformer):
    def __init__(self, cropWidth, cropHeight, cropperMethod=CropRandom):
        self.cw, self.ch, self.method = cropWidth, cropHeight, cropperMethod

    def apply(self, it):
        for img in it:
            w, h = img.width(), img.height()
            if self.method == CropRandom:
                sh = int(math.ceil(RNG.uniform(1e-2, h - self.ch)))
                sw = int(math.ceil(RNG.uniform(1e-2, w - self.cw)))
            else:
                sh, sw = (h - self.ch) // 2, (w - self.cw) // 2
            yield BGRImage(img.content[sh:sh + self.ch, sw:sw + self.cw].clone(), label=img.label())


class BGRImgRdmCropper(Transformer):
    """Zero-pad by ``padding`` then random crop (CIFAR augmentation)."""

    def __init__(self, cropWidth, cropHeight, padding):
        self.cw, self.ch, self.padding = cropWidth, cropHeight, padding

    def apply(self, it):
        p = self.padding
        for img in it:
            c = img.content
            if p > 0:
                c = torch.nn.functional.pad(c.permute(2, 0, 1), (p, p, p, p)).permute(1, 2, 0)
            h, w = c.shape[:2]
            sw = int(RNG.uniform(0, w - self.cw))
            sh = int(RNG.uniform(0, h - self.ch))
            yield BGRImage(c[sh:sh + self.ch, sw:sw + self.cw].clone(), label=img.label())


class BGRImgNormalizer(Transformer):
    """(x - mean) / std per channel; constructor args are in R, G, B order as in the reference."""

    def __init__(self, meanR, meanG, meanB, stdR, stdG, stdB):
        self.mean = torch.tensor([meanB, meanG, meanR], dtype=torch.float32)
        self.std = torch.tensor([stdB, stdG, stdR], dtype=torch.float32)

    @staticmethod
    def fromDataSet(dataSet, samples=-1):
        it = dataSet.toLocal().data(False) if hasattr(dataSet, "toLocal") else iter(dataSet)
        n = dataSet.size() if samples < 0 else samples
        px = torch.cat([next(it).content.reshape(-1, 3).double() for _ in range(n)])
        mean = px.mean(0)
        std = ((px - mean) ** 2).mean(0).sqrt()
        return BGRImgNormalizer(mean[2].item(), mean[1].item(), mean[0].item(), std[2].item(), std[1].item(),
                                std[0].item())

    def apply(self, it):
        for img in it:
            yield BGRImage((img.content - self.mean.to(img.content.device)) / self.std.to(img.content.device),
                           label=img.label())


class BGRImgPixelNormalizer(Transformer):
    """Subtract a per-pixel mean image (BGR interleaved float array of H*W*3)."""

    def __init__(self, means):
        self.means = torch.as_tensor(means, dtype=torch.float32)

    def apply(self, it):
        for img in it:
            yield BGRImage(img.content - self.means.reshape(img.content.shape).to(img.content.device),
                           label=img.label())


class HFlip(Transformer):
    def __init__(self, threshold=0.0):
        self.threshold = threshold

    def apply(self, it):
        for img in it:
            if RNG.uniform(0, 1) >= self.threshold:
                img = BGRImage(img.content.flip(1), label=img.label())
            yield img


def _gray(c):
    # the reference applies 0.299/0.587/0.114 to storage order (B, G, R) — kept for parity
    g = c[..., 0] * 0.299 + c[..., 1] * 0.587 + c[..., 2] * 0.114
    return g.unsqueeze(-1).expand_as(c)


class ColorJitter(Transformer):
    """Brightness / contrast / saturation (variance 0.4 each) in random order (ColorJitter.scala)."""

    def __init__(self, brightness=0.4, contrast=0.4, saturation=0.4):
        self.b, self.c, self.s = brightness, contrast, saturation

    def _one(self, c):
        order = torch.randperm(3).tolist()
        for o in order:
            if o == 0:
                alpha = 1.0 + RNG.uniform(-self.b, self.b)
                c = c * alpha
            elif o == 1:
                mean = _gray(c).mean()
                alpha = 1.0 + RNG.uniform(-self.c, self.c)
                c = c * alpha + (1 - alpha) * mean
            else:
                alpha = 1.0 + RNG.uniform(-self.s, self.s)
                c = c * alpha + (1 - alpha) * _gray(c)
        return c

    def apply(self, it):
        for img in it:
            yield BGRImage(self._one(img.content.float()), label=img.label())


class Lighting(Transformer):
    """AlexNet-style PCA lighting noise (Lighting.scala)."""

    eigval = torch.tensor([0.2175, 0.0188, 0.0045])
    eigvec = torch.tensor([[-0.5675, 0.7192, 0.4009], [-0.5808, -0.0045, -0.8140], [-0.5836, -0.6948, 0.4203]])

    def __init__(self, alphastd=0.1):
        self.alphastd = alphastd

    def apply(self, it):
        for img in it:
            if self.alphastd != 0:
                alpha = torch.tensor([RNG.uniform(0, self.alphastd) for _ in range(3)])
                rgb = (self.eigvec * alpha.view(1, 3) * self.eigval.view(1, 3)).sum(1)
                img = BGRImage(img.content + rgb.to(img.content.device), label=img.label())
            yield img


class BGRImgToSample(Transformer):
    def __init__(self, toRGB=True):
        self.toRGB = toRGB

    def apply(self, it):
        for img in it:
            yield Sample(img.toTensor(self.toRGB), torch.tensor([img.label()]))


class BGRImgToBatch(Transformer):
    """Stack images into an NCHW float MiniBatch (RGB order when ``toRGB``) of the per-rank batch size."""

    def __init__(self, batchSize, toRGB=True):
        self.batchSize, self.toRGB = batchSize, toRGB

    def apply(self, it):
        from .core import SampleToMiniBatch

        bs = SampleToMiniBatch(self.batchSize)._per_rank()
        xs, ys = [], []
        for img in it:
            xs.append(img.toTensor(self.toRGB))
            ys.append(img.label())
            if len(xs) == bs:
                yield MiniBatch(torch.stack(xs), torch.tensor(ys))
                xs, ys = [], []
        if xs:
            yield MiniBatch(torch.stack(xs), torch.tensor(ys))


class LocalImgReader(Transformer):
    """LocalLabeledImagePath -> BGRImage (LocalImgReader.scala: scaleTo short side, or fixed resize)."""

    NO_SCALE = -1

    def __init__(self, scaleTo=NO_SCALE, normalize=255.0, resizeW=-1, resizeH=-1):
        self.scaleTo, self.normalize, self.resizeW, self.resizeH = scaleTo, normalize, resizeW, resizeH

    def apply(self, it):
        for p in it:
            t = read_image(p.path, self.scaleTo, self.resizeW, self.resizeH)
            yield BGRImage(t.float() / self.normalize, label=p.label)


class LocalImageFiles:
    """Folder-per-class image tree -> sorted LocalLabeledImagePath list with 1-based labels
    (LocalImageFiles.scala readPaths)."""

    EXT = (".jpg", ".jpeg", ".png", ".bmp", ".ppm", ".JPEG")

    @staticmethod
    def readPaths(root, hasLabel=True):
        out = []
        if not hasLabel:
            for f in sorted(os.listdir(root)):
                if f.endswith(LocalImageFiles.EXT):
                    out.append(LocalLabeledImagePath(-1, os.path.join(root, f)))
            return out
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        for i, c in enumerate(classes):
            for f in sorted(os.listdir(os.path.join(root, c))):
                if f.endswith(LocalImageFiles.EXT):
                    out.append(LocalLabeledImagePath(i + 1, os.path.join(root, c, f)))
        return out


class MTLabeledBGRImgToBatch(Transformer):
    """Multi-threaded decode/augment + batch assembly (MTLabeledBGRImgToBatch.scala): each worker runs its own
    clone of ``transformer`` over records pulled from the shared source and writes into its slot of one
    preallocated pinned NCHW batch buffer."""

    def __init__(self, width, height, batchSize, transformer, toRGB=True, threads=None, pin_memory=False):
        self.width, self.height, self.batchSize = width, height, batchSize
        self.transformer, self.toRGB = transformer, toRGB
        self.threads = threads or min(16, os.cpu_count() or 4)
        self.pin_memory = pin_memory

    def apply(self, it):
        from .core import SampleToMiniBatch

        bs = SampleToMiniBatch(self.batchSize)._per_rank()
        lock = threading.Lock()
        src = iter(it)
        done = [False]

        def pull(pos):
            """Reserve the next slot and its record atomically, so no record is dropped at a batch edge."""
            with lock:
                if done[0] or pos[0] >= bs:
                    return None, -1
                try:
                    rec = next(src)
                except StopIteration:
                    done[0] = True
                    return None, -1
                p = pos[0]
                pos[0] += 1
                return rec, p

        tfs = [self.transformer.cloneTransformer() for _ in range(self.threads)]
        pool = ThreadPoolExecutor(self.threads)
        try:
            while not done[0]:
                feat = torch.empty(bs, 3, self.height, self.width, pin_memory=self.pin_memory)
                lab = torch.empty(bs)
                pos = [0]

                def work(tid):
                    while True:
                        rec, p = pull(pos)
                        if rec is None:
                            return
                        img = next(iter(tfs[tid].apply(iter([rec]))))
                        feat[p].copy_(img.toTensor(self.toRGB))
                        lab[p] = img.label()

                list(pool.map(work, range(self.threads)))
                n = min(pos[0], bs)
                if n == 0:
                    break
                yield MiniBatch(feat[:n], lab[:n])
        finally:
            pool.shutdown(wait=True)


class GpuImageAugment(Transformer):
    """MiniBatch of decoded uint8 [N, H, W, 3] BGR images -> normalised training batch produced on the device
    by one HIP kernel (ops/image.py): random (train) or center crop, random horizontal flip, BGR->RGB,
    per-channel (x - mean) / std. ``mean``/``std`` are given in R, G, B order on the 0..255 scale."""

    def __init__(self, cropWidth, cropHeight, mean, std, train=True, device="cuda", nhwc_bf16=False):
        self.cw, self.ch = cropWidth, cropHeight
        self.mean, self.std = list(mean), list(std)
        self.train, self.device, self.nhwc_bf16 = train, device, nhwc_bf16

    def apply(self, it):
        from ..ops.image import augment_batch, center_crop_params, random_crop_params

        for mb in it:
            x = mb.getInput().to(self.device, non_blocking=True)
            N, H, W, _ = x.shape
            p = random_crop_params(N, H, W, self.ch, self.cw) if self.train else \
                center_crop_params(N, H, W, self.ch, self.cw)
            yield MiniBatch(augment_batch(x, p, self.ch, self.cw, self.mean, self.std, True, self.nhwc_bf16),
                            mb.getTarget().to(self.device) if mb.getTarget() is not None else None)
