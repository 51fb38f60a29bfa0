"""Hadoop SequenceFile image records and the native batch-assembly path.

Reference: DataSet.SeqFileFolder (S/dataset/DataSet.scala:500-600; ``readLabel`` :512), BGRImgToLocalSeqFile
(S/dataset/image/BGRImgToLocalSeqFile.scala: Text key = "label" or "name\\nlabel", Text value = big-endian
int width, int height, then BGR HWC bytes), LocalSeqFileToBytes (S/dataset/image/LocalSeqFileToBytes.scala),
ImageNetSeqFileGenerator (S/models/utils/ImageNetSeqFileGenerator.scala), DataSet.ImageFolder
(S/dataset/DataSet.scala ImageFolder.paths / images), MTLabeledBGRImgToBatch (batch assembly).

The SequenceFile codec is the uncompressed version-6 format (Text keys and values) written by Hadoop's
``SequenceFile.Writer`` - written and read here without a JVM. ``NativeBGRImgToBatch`` hands decoded uint8
images to the C++ thread pool in ``bigdl_amd._C.assemble_batch`` (csrc/host_runtime.cpp), which crops, flips,
swaps BGR->RGB and normalises straight into a pinned fp32 NCHW batch with the GIL released.
"""
import glob
import os
import random
import struct

import torch

from .core import LocalArrayDataSet, MiniBatch, Transformer
from .image import ByteRecord, LocalImageFiles, LocalLabeledImagePath, encode_bgr_record, read_image

_TEXT = "org.apache.hadoop.io.Text"
_BYTES = "org.apache.hadoop.io.BytesWritable"
SYNC_INTERVAL = 100 * 20          # Hadoop SequenceFile.SYNC_INTERVAL (bytes between sync markers)


# ---------------------------------------------------------------------------------------------- Hadoop vints
def write_vlong(i):
    """org.apache.hadoop.io.WritableUtils.writeVLong."""
    if -112 <= i <= 127:
        return bytes([i & 0xFF])
    ln = -112
    if i < 0:
        i ^= -1
        ln = -120
    tmp = i
    while tmp != 0:
        tmp >>= 8
        ln -= 1
    out = bytearray([ln & 0xFF])
    n = -(ln + 120) if ln < -120 else -(ln + 112)
    for idx in range(n, 0, -1):
        out.append((i >> ((idx - 1) * 8)) & 0xFF)
    return bytes(out)


def read_vlong(buf, pos):
    first = struct.unpack_from("b", buf, pos)[0]
    pos += 1
    if first >= -112:
        return first, pos
    neg = first < -120
    n = -(first + 120) if neg else -(first + 112)
    v = 0
    for _ in range(n):
        v = (v << 8) | buf[pos]
        pos += 1
    return (v ^ -1) if neg else v, pos


def _text(b):
    b = b.encode("utf-8") if isinstance(b, str) else bytes(b)
    return write_vlong(len(b)) + b


# ---------------------------------------------------------------------------------------------- writer / reader
def _writable(cls, b):
    """Hadoop serialisation of one key / value: Text = vlong length + UTF-8, BytesWritable = int32 length + bytes."""
    if cls == _BYTES:
        b = bytes(b)
        return struct.pack(">i", len(b)) + b
    return _text(b)


class SequenceFileWriter:
    """Uncompressed SequenceFile (version 6); keys / values are Text (default) or BytesWritable (``_BYTES``, the
    COCO generator's record type)."""

    def __init__(self, path, key_class=_TEXT, value_class=_TEXT):
        self.f = open(path, "wb")
        self.sync = os.urandom(16)
        self.key_class, self.value_class = key_class, value_class
        hdr = (b"SEQ" + bytes([6]) + _text(key_class) + _text(value_class) + b"\x00\x00" + struct.pack(">i", 0)
               + self.sync)
        self.f.write(hdr)
        self._last_sync = self.f.tell()

    def append(self, key, value):
        k, v = _writable(self.key_class, key), _writable(self.value_class, value)
        if self.f.tell() >= self._last_sync + SYNC_INTERVAL:
            self.f.write(struct.pack(">i", -1) + self.sync)
            self._last_sync = self.f.tell()
        self.f.write(struct.pack(">ii", len(k) + len(v), len(k)) + k + v)

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_sequence_file(path):
    """Yield (key bytes, value bytes) of an uncompressed SequenceFile of Text / BytesWritable pairs."""
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:3] != b"SEQ":
        raise ValueError(f"{path}: not a SequenceFile")
    version = buf[3]
    pos = 4
    if version < 6:
        raise ValueError(f"{path}: SequenceFile version {version} not supported")
    names = []
    for _ in range(2):
        n, pos = read_vlong(buf, pos)
        names.append(buf[pos:pos + n].decode())
        pos += n
    compressed, block = buf[pos], buf[pos + 1]
    pos += 2
    if compressed or block:
        raise ValueError(f"{path}: compressed SequenceFiles are not supported")
    (nmeta,) = struct.unpack_from(">i", buf, pos)
    pos += 4
    for _ in range(nmeta * 2):
        n, pos = read_vlong(buf, pos)
        pos += n
    sync = buf[pos:pos + 16]
    pos += 16
    while pos < len(buf):
        (rec_len,) = struct.unpack_from(">i", buf, pos)
        pos += 4
        if rec_len == -1:
            if buf[pos:pos + 16] != sync:
                raise ValueError(f"{path}: corrupt sync marker at {pos}")
            pos += 16
            continue
        (key_len,) = struct.unpack_from(">i", buf, pos)
        pos += 4
        kb = buf[pos:pos + key_len]
        vb = buf[pos + key_len:pos + rec_len]
        pos += rec_len
        yield _unwritable(names[0], kb), _unwritable(names[1], vb)


def _unwritable(cls, b):
    if cls == _BYTES:
        (n,) = struct.unpack_from(">i", b, 0)
        return b[4:4 + n]
    n, p = read_vlong(b, 0)
    return b[p:p + n]


def read_label(key):
    """SeqFileFolder.readLabel: the key is "label" or "name\\nlabel"."""
    s = key.decode() if isinstance(key, (bytes, bytearray)) else str(key)
    return s.split("\n")[-1]


def read_name(key):
    s = key.decode() if isinstance(key, (bytes, bytearray)) else str(key)
    parts = s.split("\n")
    return parts[0] if len(parts) > 1 else None


# ---------------------------------------------------------------------------------------------- transformers
class BGRImgToLocalSeqFile(Transformer):
    """(LabeledBGRImage | uint8 HWC tensor with label, name) -> written seq file names, ``blockSize`` records
    per file named ``{baseFileName}_{index}.seq``."""

    def __init__(self, blockSize, baseFileName, hasName=False):
        self.blockSize, self.baseFileName, self.hasName = blockSize, baseFileName, hasName
        self.index = 0

    def apply(self, it):
        it = iter(it)
        while True:
            name = f"{self.baseFileName}_{self.index}.seq"
            n = 0
            w = None
            for img, img_name in it:
                if w is None:
                    w = SequenceFileWriter(name)
                content = img.content if hasattr(img, "content") else img
                label = img.label() if callable(getattr(img, "label", None)) else getattr(img, "label", 0)
                u8 = content if content.dtype == torch.uint8 else content.round().clamp(0, 255).to(torch.uint8)
                key = f"{img_name}\n{int(label)}" if self.hasName else f"{int(label)}"
                w.append(key, encode_bgr_record(u8))
                n += 1
                if n >= self.blockSize:
                    break
            if w is None:
                return
            w.close()
            self.index += 1
            yield name
            if n < self.blockSize:
                return


class LocalSeqFileToBytes(Transformer):
    """seq file paths -> ByteRecord(value bytes, label)."""

    def apply(self, it):
        for p in it:
            path = p.path if hasattr(p, "path") else p
            for k, v in read_sequence_file(path):
                yield ByteRecord(v, float(read_label(k)))


def decode_bgr_record(data):
    """ByteRecord bytes (int width, int height big-endian, BGR HWC) -> uint8 [H, W, 3]."""
    w, h = struct.unpack_from(">ii", data, 0)
    return torch.frombuffer(bytearray(data[8:8 + w * h * 3]), dtype=torch.uint8).reshape(h, w, 3)


class NativeBGRImgToBatch(Transformer):
    """ByteRecords (BGR records) or (uint8 HWC tensor, label) pairs -> MiniBatch of normalised fp32 NCHW crops,
    assembled by the native C++ pool (``_C.assemble_batch``). Training: random crop + random horizontal flip
    (BGRImgRdmCropper + HFlip); evaluation: center crop. ``mean`` / ``std`` in R, G, B order on 0..255."""

    def __init__(self, cropWidth, cropHeight, batchSize, mean=(123.0, 117.0, 104.0), std=(58.4, 57.1, 57.4),
                 train=True, toRGB=True, threads=0, pin_memory=False, seed=None):
        self.cw, self.ch, self.batchSize = cropWidth, cropHeight, batchSize
        self.mean, self.std, self.train, self.toRGB = list(mean), list(std), train, toRGB
        self.threads, self.pin_memory = threads, pin_memory
        self.rng = random.Random(seed)

    def _params(self, imgs):
        ps = []
        for im in imgs:
            H, W = im.shape[0], im.shape[1]
            if H < self.ch or W < self.cw:
                raise ValueError(f"image {H}x{W} smaller than the crop {self.ch}x{self.cw}")
            if self.train:
                ps.append([self.rng.randint(0, H - self.ch), self.rng.randint(0, W - self.cw), self.rng.random() < 0.5])
            else:
                ps.append([(H - self.ch) // 2, (W - self.cw) // 2, 0])
        return torch.tensor(ps, dtype=torch.int32)

    def _flush(self, imgs, labels):
        from ..ops import native

        out = torch.empty(len(imgs), 3, self.ch, self.cw, pin_memory=self.pin_memory)
        native.get().assemble_batch(imgs, self._params(imgs), out, self.mean, self.std, self.toRGB, self.threads)
        return MiniBatch(out, torch.tensor(labels, dtype=torch.float32))

    def apply(self, it):
        from .core import SampleToMiniBatch

        bs = SampleToMiniBatch(self.batchSize)._per_rank()
        imgs, labels = [], []
        for r in it:
            if isinstance(r, ByteRecord):
                im, lab = decode_bgr_record(r.data), r.label
            else:
                im, lab = r
            imgs.append(im.contiguous())
            labels.append(float(lab))
            if len(imgs) == bs:
                yield self._flush(imgs, labels)
                imgs, labels = [], []
        if imgs:
            yield self._flush(imgs, labels)


# ---------------------------------------------------------------------------------------------- datasets
class SeqFileFolder:
    """DataSet.SeqFileFolder: a folder of ``*.seq`` files of BGR image records."""

    @staticmethod
    def paths(folder):
        return sorted(glob.glob(os.path.join(folder, "*.seq")))

    @staticmethod
    def files(folder, classNum=None, shuffle=True):
        """All records as an in-memory ByteRecord dataset (labels 1-based, filtered to ``classNum``)."""
        recs = []
        for p in SeqFileFolder.paths(folder):
            for k, v in read_sequence_file(p):
                lab = float(read_label(k))
                if classNum is None or lab <= classNum:
                    recs.append(ByteRecord(v, lab))
        return LocalArrayDataSet(recs, shuffle)


class ImageFolder:
    """DataSet.ImageFolder: a folder-per-class tree of image files."""

    @staticmethod
    def paths(root, hasLabel=True, shuffle=True):
        return LocalArrayDataSet(LocalImageFiles.readPaths(root, hasLabel), shuffle)

    @staticmethod
    def images(root, scaleTo=256, shuffle=True):
        """Decoded uint8 BGR images (short side scaled to ``scaleTo``) as ByteRecords."""
        recs = [ByteRecord(encode_bgr_record(read_image(p.path, scaleTo)), p.label)
                for p in LocalImageFiles.readPaths(root, True)]
        return LocalArrayDataSet(recs, shuffle)


def generate_seq_files(image_root, out_dir, blockSize=12800, scaleTo=256, hasName=False, prefix="imagenet"):
    """ImageNetSeqFileGenerator: image tree -> seq files of scaled BGR records; returns the file names."""
    os.makedirs(out_dir, exist_ok=True)
    paths = LocalImageFiles.readPaths(image_root, True)

    def items():
        for p in paths:
            img = read_image(p.path, scaleTo)
            yield _Labeled(img, p.label), os.path.basename(p.path)

    return list(BGRImgToLocalSeqFile(blockSize, os.path.join(out_dir, prefix), hasName).apply(items()))


class _Labeled:
    def __init__(self, content, label):
        self.content, self._label = content, label

    def label(self):
        return self._label


__all__ = ["SequenceFileWriter", "read_sequence_file", "read_label", "read_name", "BGRImgToLocalSeqFile",
           "LocalSeqFileToBytes", "decode_bgr_record", "NativeBGRImgToBatch", "SeqFileFolder", "ImageFolder",
           "generate_seq_files", "write_vlong", "read_vlong", "LocalLabeledImagePath"]
