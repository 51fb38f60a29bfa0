"""ImageFeature / ImageFrame / FeatureTransformer and the convertors (reference
S/transform/vision/image/{ImageFeature.scala:36, ImageFrame.scala, FeatureTransformer.scala:27, Convertor.scala,
MTImageFeatureToBatch.scala}).

A ``mat`` is a float32 torch tensor [H, W, C] in BGR channel order holding 0..255 pixel values (the
OpenCV CV_8UC3 / CV_32FC3 mats of the reference); colour operations saturate to [0, 255] like 8-bit mats.
"""
import logging
import os

import torch

from ....dataset.core import MiniBatch, Sample, Transformer

logger = logging.getLogger("bigdl_amd.transform")


class ImageFeature(dict):
    uri, mat, bytes, floats, size, originalSize = "uri", "mat", "bytes", "floats", "size", "originalSize"
    label, predict, boundingBox, sample, imageTensor = "label", "predict", "boundingBox", "sample", "imageTensor"

    def __init__(self, bytes=None, label=None, uri=None):
        super().__init__()
        self._valid = True
        if bytes is not None:
            self[ImageFeature.bytes] = bytes
        if label is not None:
            self[ImageFeature.label] = label
        if uri is not None:
            self[ImageFeature.uri] = uri

    def apply(self, key):
        return self.get(key)

    def update(self, key, value=None):
        if value is None and isinstance(key, dict):
            return super().update(key)
        self[key] = value
        return self

    def contains(self, key):
        return key in self

    def opencvMat(self):
        return self.get(ImageFeature.mat)

    def isValid(self):
        return self._valid

    def setValid(self, v):
        self._valid = v

    def getSize(self):
        m = self.opencvMat()
        if m is not None:
            return (m.shape[0], m.shape[1], m.shape[2] if m.dim() == 3 else 1)
        return self.get(ImageFeature.size)

    def getHeight(self):
        return self.getSize()[0]

    def getWidth(self):
        return self.getSize()[1]

    def getChannel(self):
        return self.getSize()[2]

    def getOriginalSize(self):
        return self.get(ImageFeature.originalSize)

    def getOriginalWidth(self):
        return self.getOriginalSize()[1]

    def getOriginalHeight(self):
        return self.getOriginalSize()[0]

    def getLabel(self):
        return self.get(ImageFeature.label)

    def getUri(self):
        return self.get(ImageFeature.uri)

    def getImInfo(self):
        h, w, _ = self.getSize()
        oh, ow, _ = self.getOriginalSize()
        return torch.tensor([h, w, h / oh, w / ow], dtype=torch.float32)

    def toTensor(self, key=None):
        return self.get(key or ImageFeature.imageTensor)

    def clone(self):
        f = ImageFeature()
        for k, v in self.items():
            f[k] = v.clone() if isinstance(v, torch.Tensor) else v
        f._valid = self._valid
        return f


class FeatureTransformer(Transformer):
    """Per-feature transformer; failures mark the feature invalid instead of killing the pipeline
    (FeatureTransformer.scala transform + ignoreImageException)."""

    def transformMat(self, feature):
        pass

    def transform(self, feature):
        if not feature.isValid():
            return feature
        try:
            self.transformMat(feature)
        except Exception as e:  # noqa: BLE001
            logger.warning("failed in transform %s: %s", type(self).__name__, e)
            feature.setValid(False)
        return feature

    def __call__(self, x):
        if isinstance(x, ImageFeature):
            return self.transform(x)
        if isinstance(x, ImageFrame):
            return x.transform(self)
        return super().__call__(x)

    def apply(self, it):
        for f in it:
            yield self.transform(f)

    def __rshift__(self, other):
        return ChainedFeatureTransformer(self, other)


class ChainedFeatureTransformer(FeatureTransformer):
    def __init__(self, first, last):
        self.first, self.last = first, last

    def transform(self, feature):
        return self.last.transform(self.first.transform(feature))


# ---------------------------------------------------------------------------------------------- frames
class ImageFrame:
    @staticmethod
    def array(features):
        return LocalImageFrame(list(features))

    @staticmethod
    def rdd(features, rank=None, world=None):
        return DistributedImageFrame(list(features), rank, world)

    @staticmethod
    def read(path, minPartitions=1):
        """Read an image file or a folder tree into a LocalImageFrame of raw-bytes features."""
        files = []
        if os.path.isdir(path):
            for root, _, names in os.walk(path):
                for n in sorted(names):
                    files.append(os.path.join(root, n))
        else:
            files = [path]
        feats = []
        for f in sorted(files):
            with open(f, "rb") as fh:
                feats.append(ImageFeature(fh.read(), uri=f))
        return LocalImageFrame(feats)

    def isLocal(self):
        return isinstance(self, LocalImageFrame) and not isinstance(self, DistributedImageFrame)

    def isDistributed(self):
        return isinstance(self, DistributedImageFrame)


class LocalImageFrame(ImageFrame):
    def __init__(self, array):
        self.array = array

    def transform(self, transformer):
        self.array = [transformer.transform(f) for f in self.array]
        return self

    def __rshift__(self, transformer):
        return self.transform(transformer)

    def toLocal(self):
        return self

    def size(self):
        return len(self.array)


class DistributedImageFrame(LocalImageFrame):
    """One rank's shard (rank::world) of the frame — the analog of an RDD partition set."""

    def __init__(self, array, rank=None, world=None):
        import torch.distributed as dist

        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
            world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        super().__init__(array[rank::world])
        self.rank, self.world = rank, world

    def toDistributed(self):
        return self


# ---------------------------------------------------------------------------------------------- convertors
def _decode(b):
    import io

    from PIL import Image

    with Image.open(io.BytesIO(b)) as im:
        im = im.convert("RGB")
        t = torch.frombuffer(bytearray(im.tobytes()), dtype=torch.uint8).reshape(im.size[1], im.size[0], 3)
    return t.flip(2).float().contiguous()


class BytesToMat(FeatureTransformer):
    """Decode encoded image bytes (JPEG/PNG/...) to a BGR mat."""

    def __init__(self, byteKey=ImageFeature.bytes):
        self.byteKey = byteKey

    def transformMat(self, feature):
        m = _decode(feature[self.byteKey])
        feature[ImageFeature.mat] = m
        feature[ImageFeature.originalSize] = tuple(m.shape)


class PixelBytesToMat(FeatureTransformer):
    """Raw BGR pixel bytes + originalSize (h, w, c) -> mat."""

    def __init__(self, byteKey=ImageFeature.bytes):
        self.byteKey = byteKey

    def transformMat(self, feature):
        h, w, c = feature[ImageFeature.originalSize]
        t = torch.frombuffer(bytearray(feature[self.byteKey]), dtype=torch.uint8).reshape(h, w, c)
        feature[ImageFeature.mat] = t.float()


class MatToFloats(FeatureTransformer):
    def __init__(self, validHeight=300, validWidth=300, validChannels=3, outKey=ImageFeature.floats,
                 shareBuffer=True):
        self.h, self.w, self.c, self.outKey = validHeight, validWidth, validChannels, outKey

    def transformMat(self, feature):
        m = feature.opencvMat()
        if m is None:
            m = torch.zeros(self.h, self.w, self.c)
        feature[self.outKey] = m.reshape(-1).float().clone()
        feature[ImageFeature.size] = tuple(m.shape)


class MatToTensor(FeatureTransformer):
    """mat [H, W, C] -> CHW float tensor (RGB order when ``toRGB``)."""

    def __init__(self, toRGB=False, tensorKey=ImageFeature.imageTensor, shareBuffer=True, greyToRGB=False):
        self.toRGB, self.tensorKey, self.greyToRGB = toRGB, tensorKey, greyToRGB

    def transformMat(self, feature):
        m = feature.opencvMat().float()
        if m.dim() == 2:
            m = m.unsqueeze(-1)
        if self.greyToRGB and m.shape[2] == 1:
            m = m.expand(-1, -1, 3)
        if self.toRGB and m.shape[2] == 3:
            m = m.flip(2)
        feature[self.tensorKey] = m.permute(2, 0, 1).contiguous()


class ImageFrameToSample(FeatureTransformer):
    def __init__(self, inputKeys=(ImageFeature.imageTensor,), targetKeys=None, sampleKey=ImageFeature.sample):
        self.inputKeys, self.targetKeys, self.sampleKey = list(inputKeys), targetKeys, sampleKey

    def transformMat(self, feature):
        feats = [feature[k] for k in self.inputKeys]
        labels = None
        if self.targetKeys:
            labels = [torch.as_tensor(feature[k], dtype=torch.float32).reshape(-1) for k in self.targetKeys]
        feature[self.sampleKey] = Sample(feats if len(feats) > 1 else feats[0],
                                         labels if labels is None or len(labels) > 1 else labels[0])


class ImageFeatureToMiniBatch(Transformer):
    def __init__(self, batchSize, featurePaddingParam=None, labelPaddingParam=None, partitionNum=None,
                 sampleKey=ImageFeature.sample):
        from ....dataset.core import SampleToMiniBatch

        self.s2b = SampleToMiniBatch(batchSize, featurePaddingParam, labelPaddingParam, partitionNum)
        self.sampleKey = sampleKey

    def apply(self, it):
        return self.s2b.apply(f[self.sampleKey] for f in it if f.isValid())


class MTImageFeatureToBatch(Transformer):
    """Multi-threaded ImageFeature -> MiniBatch of ``imageTensor`` (ClassificationMTImageFeatureToBatch)."""

    def __init__(self, width, height, batchSize, transformer, toRGB=True, threads=None):
        from ....dataset.image import MTLabeledBGRImgToBatch

        self.width, self.height, self.batchSize = width, height, batchSize
        self.transformer, self.toRGB, self.threads = transformer, toRGB, threads
        self._mt = MTLabeledBGRImgToBatch

    def apply(self, it):
        from ....dataset.image import BGRImage

        outer = self

        class _Adapter(Transformer):
            def apply(self, inner):
                for f in inner:
                    f = outer.transformer.transform(f)
                    lab = f.get(ImageFeature.label, 0.0)
                    yield BGRImage(f.opencvMat(), label=float(torch.as_tensor(lab).reshape(-1)[0]))

        return self._mt(self.width, self.height, self.batchSize, _Adapter(), self.toRGB, self.threads).apply(it)
