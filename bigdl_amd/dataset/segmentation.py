"""Segmentation masks (COCO RLE / polygons) and the COCO detection dataset.

Reference: S/dataset/segmentation/MaskUtils.scala:23-593 (RLEMasks, PolyMasks, compact RLE string codec,
polygon rasterisation, RLE merge / area / IoU / bbox, binary mask -> RLE) and COCODataset.scala:29-351
(COCO json loading, category id <-> index mapping, image / annotation records).

RLE convention (COCO "uncompressed" RLE): run lengths over the column-major flattening of an h x w mask,
starting with a run of zeros. All functions are host-side numpy: masks are produced once per detection and
serialised, the GPU never sees them.
"""
import glob
import json
import math
import os
import struct

import numpy as np
import torch


class SegmentationMasks:
    def toRLE(self):
        raise NotImplementedError


class RLEMasks(SegmentationMasks):
    """Uncompressed COCO RLE (reference MaskUtils.scala:68)."""

    def __init__(self, counts, height, width):
        self.counts = [int(c) for c in counts]
        self.height, self.width = int(height), int(width)
        self._bbox = None

    def toRLE(self):
        return self

    def get(self, idx):
        return self.counts[idx] & 0xFFFFFFFF      # counts are unsigned in COCO

    @property
    def bbox(self):
        if self._bbox is None:
            self._bbox = rle_to_bbox(self)
        return self._bbox

    @property
    def area(self):
        return rle_area(self)

    def __eq__(self, other):
        return isinstance(other, RLEMasks) and self.counts == other.counts and \
            (self.height, self.width) == (other.height, other.width)

    def __hash__(self):
        return hash((tuple(self.counts), self.height, self.width))

    def __repr__(self):
        return f"RLEMasks({len(self.counts)} runs, {self.height}x{self.width})"


class PolyMasks(SegmentationMasks):
    """Polygon masks (reference MaskUtils.scala:37): ``poly`` is a list of flat [x0, y0, x1, y1, ...] lists."""

    def __init__(self, poly, height, width):
        self.poly = [list(map(float, p)) for p in poly]
        self.height, self.width = int(height), int(width)

    def toRLE(self):
        assert self.height > 0 and self.width > 0, "PolyMasks.toRLE needs the image size"
        return poly_to_single_rle(self, self.height, self.width)


# ----------------------------------------------------------------------------------- compact string codec
def rle_to_string(rle):
    """Compact COCO RLE string (LEB128-like, 5 bits per char, ascii 48..111; counts delta-coded from i-2)."""
    out = []
    c = rle.counts
    for i in range(len(c)):
        x = c[i] & 0xFFFFFFFF
        if i > 2:
            x -= c[i - 2] & 0xFFFFFFFF
        more = True
        while more:
            ch = x & 0x1F
            x >>= 5                      # python ints shift arithmetically, like the C long
            more = (x != -1) if (ch & 0x10) else (x != 0)
            if more:
                ch |= 0x20
            out.append(chr(ch + 48))
    return "".join(out)


def string_to_rle(s, h, w):
    cnts = []
    p = 0
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            k += 1
            p += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(cnts) > 2:
            x += cnts[-2] & 0xFFFFFFFF
        cnts.append(((x + 2 ** 31) % 2 ** 32) - 2 ** 31)   # wrap to int32 like x.toInt
    return RLEMasks(cnts, h, w)


# ------------------------------------------------------------------------------------- polygon -> RLE
def poly_to_rle(poly, height, width):
    """One RLE per polygon (not merged) — COCO rleFrPoly."""
    return [_one_poly(xy, height, width) for xy in poly.poly]


def _one_poly(xy, h, w):
    scale = 5.0
    k = len(xy) // 2
    x = [int(math.floor(scale * xy[2 * j] + 0.5)) for j in range(k)]
    y = [int(math.floor(scale * xy[2 * j + 1] + 0.5)) for j in range(k)]
    x.append(x[0])
    y.append(y[0])
    u, v = [], []
    for j in range(k):
        xs, xe, ys, ye = x[j], x[j + 1], y[j], y[j + 1]
        dx, dy = abs(xe - xs), abs(ys - ye)
        flip = (dx >= dy and xs > xe) or (dx < dy and ys > ye)
        if flip:
            xs, xe, ys, ye = xe, xs, ye, ys
        if dx >= dy:
            s = (ye - ys) / dx if dx else 0.0
            for d in range(dx + 1):
                t = dx - d if flip else d
                u.append(t + xs)
                v.append(int(math.floor(ys + s * t + 0.5)))
        else:
            s = (xe - xs) / dy
            for d in range(dy + 1):
                t = dy - d if flip else d
                v.append(t + ys)
                u.append(int(math.floor(xs + s * t + 0.5)))
    # y-boundary points, downsampled
    bx, by = [], []
    for j in range(1, len(u)):
        if u[j] == u[j - 1]:
            continue
        xd = u[j] if u[j] < u[j - 1] else u[j] - 1
        xd = (xd + 0.5) / scale - 0.5
        if math.floor(xd) != xd or xd < 0 or xd > w - 1:
            continue
        yd = float(v[j] if v[j] < v[j - 1] else v[j - 1])
        yd = (yd + 0.5) / scale - 0.5
        yd = min(max(yd, 0.0), float(h))
        bx.append(int(xd))
        by.append(int(math.ceil(yd)))
    a = sorted([bx[j] * h + by[j] for j in range(len(bx))] + [h * w])
    prev = 0
    for j in range(len(a)):
        a[j], prev = a[j] - prev, a[j]
    b = [a[0]]
    j = 1
    while j < len(a):
        if a[j] > 0:
            b.append(a[j])
            j += 1
        else:
            j += 1
            if j < len(a):
                b[-1] += a[j]
                j += 1
    return RLEMasks(b, h, w)


def poly_to_single_rle(poly, height, width):
    return merge_rles(poly_to_rle(poly, height, width), False)


# --------------------------------------------------------------------------------- RLE set operations
def merge_rles(rles, intersect):
    """Union (or intersection) of RLEs of the same size — COCO rleMerge."""
    if len(rles) == 1:
        return rles[0]
    h, w = rles[0].height, rles[0].width
    cnts = [c & 0xFFFFFFFF for c in rles[0].counts]
    for B in rles[1:]:
        assert (B.height, B.width) == (h, w), "The height and width of the merged RLEs must be the same"
        A = cnts
        cnts = []
        ca, cb = A[0], B.get(0)
        v = va = vb = False
        a = b = 1
        cc, ct = 0, 1
        while ct > 0:
            c = min(ca, cb)
            cc += c
            ct = 0
            ca -= c
            if ca == 0 and a < len(A):
                ca = A[a]
                a += 1
                va = not va
            ct += ca
            cb -= c
            if cb == 0 and b < len(B.counts):
                cb = B.get(b)
                b += 1
                vb = not vb
            ct += cb
            vp = v
            v = (va and vb) if intersect else (va or vb)
            if v != vp or ct == 0:
                cnts.append(cc)
                cc = 0
    return RLEMasks(cnts, h, w)


def rle_area(rle):
    return int(sum(rle.get(j) for j in range(1, len(rle.counts), 2)))


def bbox_iou(gt, dt, is_crowd):
    """IoU of inclusive pixel boxes (x1, y1, x2, y2) (reference MaskUtils.bboxIOU)."""
    f = np.float32
    xmin, ymin, xmax, ymax = map(f, gt)
    x1, y1, x2, y2 = map(f, dt)
    area = (xmax - xmin + 1) * (ymax - ymin + 1)
    inter = max(min(xmax, x2) - max(xmin, x1) + 1, f(0)) * max(min(ymax, y2) - max(ymin, y1) + 1, f(0))
    darea = (x2 - x1 + 1) * (y2 - y1 + 1)
    union = darea if is_crowd else darea + area - inter
    return f(inter / union)


def rle_to_bbox(rle):
    m = len(rle.counts) // 2 * 2
    h = rle.height
    if m == 0:
        return (0.0, 0.0, 0.0, 0.0)
    xs, ys, xe, ye = rle.width, rle.height, 0, 0
    xp, cc = 0, 0
    for j in range(m):
        cc += rle.get(j)
        t = cc - j % 2
        y = t % h
        x = (t - y) // h
        if j % 2 == 0:
            xp = x
        elif xp < x:
            ys, ye = 0, h - 1
        xs, xe = min(xs, x), max(xe, x)
        ys, ye = min(ys, y), max(ye, y)
    return (float(xs), float(ys), float(xe), float(ye))


def rle_iou(detection, ground_truth, is_crowd):
    assert (detection.width, detection.height) == (ground_truth.width, ground_truth.height), \
        "The sizes of RLEs must be the same to compute IOU"
    iou = bbox_iou(ground_truth.bbox, detection.bbox, is_crowd)
    if iou <= 0:
        return iou
    a = b = 1
    ca, cb = detection.get(0), ground_truth.get(0)
    ka, kb = len(detection.counts), len(ground_truth.counts)
    va = vb = False
    i = u = 0
    ct = 1
    while ct > 0:
        c = min(ca, cb)
        if va or vb:
            u += c
            if va and vb:
                i += c
        ct = 0
        ca -= c
        if ca == 0 and a < ka:
            ca = detection.get(a)
            a += 1
            va = not va
        ct += ca
        cb -= c
        if cb == 0 and b < kb:
            cb = ground_truth.get(b)
            b += 1
            vb = not vb
        ct += cb
    if i == 0:
        u = 1
    elif is_crowd:
        u = detection.area
    return np.float32(i) / np.float32(u)


def binary_to_rle(mask):
    """Binary (h, w) mask (tensor / array of 0/1) -> RLEMasks (column-major runs, first run of zeros)."""
    m = np.asarray(mask.detach().cpu() if isinstance(mask, torch.Tensor) else mask)
    h, w = m.shape
    flat = (m.T.reshape(-1) != 0).astype(np.int8)
    if flat.size == 0:
        return RLEMasks([0], h, w)
    change = np.flatnonzero(np.diff(flat)) + 1
    bounds = np.concatenate([[0], change, [flat.size]])
    runs = np.diff(bounds).tolist()
    if flat[0] == 1:
        runs = [0] + runs
    return RLEMasks(runs, h, w)


def rle_to_binary(rle):
    flat = np.zeros(rle.height * rle.width, dtype=np.uint8)
    pos, val = 0, 0
    for c in rle.counts:
        c &= 0xFFFFFFFF
        if val:
            flat[pos: pos + c] = 1
        pos += c
        val ^= 1
    return flat.reshape(rle.width, rle.height).T


class MaskUtils:
    """Namespace mirroring the reference object's method names."""
    RLE2String = staticmethod(rle_to_string)
    string2RLE = staticmethod(string_to_rle)
    poly2RLE = staticmethod(poly_to_rle)
    polyToSingleRLE = staticmethod(poly_to_single_rle)
    mergeRLEs = staticmethod(merge_rles)
    rleArea = staticmethod(rle_area)
    rleIOU = staticmethod(rle_iou)
    bboxIOU = staticmethod(bbox_iou)
    rleToOneBbox = staticmethod(rle_to_bbox)
    binaryToRLE = staticmethod(binary_to_rle)
    rleToBinary = staticmethod(rle_to_binary)


# ------------------------------------------------------------------------------------------ COCO dataset
class COCOImage:
    def __init__(self, d, root):
        self.id, self.height, self.width = int(d["id"]), int(d["height"]), int(d["width"])
        self.fileName = d.get("file_name")
        self.imgRootPath = root
        self.annotations = []

    @property
    def path(self):
        return os.path.join(self.imgRootPath, self.fileName)

    def data(self):
        with open(self.path, "rb") as f:
            return f.read()


class COCOAnnotation:
    """Object-detection annotation; ``bbox`` is inclusive (x1, y1, x1 + w - 1, y1 + h - 1)."""

    def __init__(self, d):
        self.id, self.imageId, self.categoryId = int(d["id"]), int(d["image_id"]), int(d["category_id"])
        self.area = float(d["area"])
        x1, y1, w, h = [float(v) for v in d["bbox"]]
        self.bbox = (x1, y1, x1 + w - 1, y1 + h - 1)
        self.isCrowd = int(d.get("iscrowd", 0)) == 1
        seg = d["segmentation"]
        if self.isCrowd:
            self.segmentation = RLEMasks(seg["counts"], seg["size"][0], seg["size"][1])
        else:
            self.segmentation = PolyMasks(seg, -1, -1)
        self.image = None


class COCODataset:
    """COCO instances json (reference COCODataset.scala:138). Category index 0 is background."""

    def __init__(self, d, image_root="."):
        self.info = d.get("info", {})
        self.licenses = d.get("licenses", [])
        self.categories = d.get("categories", [])
        self.images = [COCOImage(i, image_root) for i in d.get("images", [])]
        self.annotations = [COCOAnnotation(a) for a in d.get("annotations", [])]
        self._img = {im.id: im for im in self.images}
        self._cat = {int(c["id"]): i + 1 for i, c in enumerate(self.categories)}
        for a in self.annotations:
            assert a.imageId in self._img, f"Cannot find image_id {a.imageId}"
            img = self._img[a.imageId]
            a.image = img
            img.annotations.append(a)
            if isinstance(a.segmentation, PolyMasks):
                a.segmentation = PolyMasks(a.segmentation.poly, img.height, img.width)

    @staticmethod
    def load(json_path, image_root="."):
        with open(json_path) as f:
            return COCODataset(json.load(f), image_root)

    def getImageById(self, i):
        return self._img[int(i)]

    def categoryId2Idx(self, i):
        return self._cat[int(i)]

    def getCategoryByIdx(self, idx):
        return self.categories[idx - 1]

    def to_targets(self, image):
        """(bboxes (n, 4), class indices (n), masks [RLEMasks], is_crowd (n)) of one image."""
        anns = image.annotations
        boxes = torch.tensor([a.bbox for a in anns], dtype=torch.float32).reshape(-1, 4)
        cls = torch.tensor([self.categoryId2Idx(a.categoryId) for a in anns], dtype=torch.float32)
        masks = [a.segmentation.toRLE() for a in anns]
        crowd = torch.tensor([1.0 if a.isCrowd else 0.0 for a in anns])
        return boxes, cls, masks, crowd


# ------------------------------------------------------------------------------------------ COCO sequence files
COCO_MAGIC = 0x1F3D4E5A


class COCOSerializeContext:
    """Big-endian record writer of the COCO sequence-file key (reference COCODataset.scala:29-77)."""

    def __init__(self):
        self.buf = bytearray()

    def clear(self):
        self.buf = bytearray()

    def dump_int(self, v):
        self.buf += struct.pack(">i", int(v))

    def dump_float(self, v):
        self.buf += struct.pack(">f", float(v))

    def dump_bool(self, v):
        self.buf += b"\x01" if v else b"\x00"

    def dump_bytes(self, b):
        self.dump_int(len(b))
        self.buf += bytes(b)

    def dump_string(self, s):
        self.dump_bytes(s.encode("utf-8"))

    def toByteArray(self):
        return bytes(self.buf)


def dump_image_meta(ctx, image, dataset):
    """fileName, height, width, then per annotation: category index, area, bbox (4 floats, inclusive x1 y1 x2 y2),
    isCrowd, and the RLE counts (crowd) or polygons (reference COCOImage / COCOAnotationOD / COCORLE / COCOPoly
    dumpTo), closed by the magic number."""
    ctx.dump_string(image.fileName)
    ctx.dump_int(image.height)
    ctx.dump_int(image.width)
    ctx.dump_int(len(image.annotations))
    for a in image.annotations:
        ctx.dump_int(dataset.categoryId2Idx(a.categoryId))
        ctx.dump_float(a.area)
        for v in a.bbox:
            ctx.dump_float(v)
        ctx.dump_bool(a.isCrowd)
        seg = a.segmentation
        if isinstance(seg, RLEMasks):
            ctx.dump_int(len(seg.counts))
            for c in seg.counts:
                ctx.dump_int(c if c < 2 ** 31 else c - 2 ** 32)
        else:
            ctx.dump_int(len(seg.poly))
            for p in seg.poly:
                ctx.dump_int(len(p))
                for v in p:
                    ctx.dump_float(v)
    ctx.dump_int(COCO_MAGIC)


class COCODeserializer:
    """Reader of the record key (reference COCODeserializer, COCODataset.scala:80-136)."""

    def __init__(self, buf):
        self.b, self.p = bytes(buf), 0

    def _u(self, fmt, n):
        (v,) = struct.unpack_from(fmt, self.b, self.p)
        self.p += n
        return v

    def getInt(self):
        return self._u(">i", 4)

    def getFloat(self):
        return self._u(">f", 4)

    def getBoolean(self):
        v = self.b[self.p] != 0
        self.p += 1
        return v

    def getString(self):
        n = self.getInt()
        s = self.b[self.p:self.p + n].decode("utf-8")
        self.p += n
        return s

    def getAnnotations(self):
        h, w, n = self.getInt(), self.getInt(), self.getInt()
        anns = []
        for _ in range(n):
            cat, area = self.getInt(), self.getFloat()
            bbox = tuple(self.getFloat() for _ in range(4))
            crowd = self.getBoolean()
            if crowd:
                counts = [self.getInt() & 0xFFFFFFFF for _ in range(self.getInt())]
                masks = RLEMasks(counts, h, w)
            else:
                polys = []
                for _ in range(self.getInt()):
                    polys.append([self.getFloat() for _ in range(self.getInt())])
                masks = PolyMasks(polys, h, w)
            anns.append({"categoryId": cat, "area": area, "bbox": bbox, "isCrowd": crowd, "masks": masks})
        return h, w, anns


def generate_coco_seq_files(meta_path, image_root, out_dir, blockSize=12800, prefix="coco-seq"):
    """COCO instances json + image folder -> ``{prefix}-{block}.seq`` files of (metadata key, encoded image bytes)
    BytesWritable records (reference models/utils/COCOSeqFileGenerator.scala; written uncompressed here rather than
    BZip2 block-compressed). Images whose file is missing are skipped with a warning, as in the reference."""
    from .seqfile import _BYTES, SequenceFileWriter

    meta = COCODataset.load(meta_path, image_root)
    imgs = [im for im in meta.images if os.path.isfile(im.path)]
    os.makedirs(out_dir, exist_ok=True)
    ctx = COCOSerializeContext()
    paths = []
    for blk in range(0, len(imgs), blockSize):
        path = os.path.join(out_dir, f"{prefix}-{blk // blockSize}.seq")
        with SequenceFileWriter(path, _BYTES, _BYTES) as w:
            for im in imgs[blk:blk + blockSize]:
                ctx.clear()
                dump_image_meta(ctx, im, meta)
                w.append(ctx.toByteArray(), im.data())
        paths.append(path)
    return paths


def read_coco_seq_files(folder):
    """Yield one detection sample per record: {"fileName", "image" (uint8 BGR H x W x 3 tensor), "classes" (n),
    "bboxes" (n, 4), "isCrowd" (n), "masks" [SegmentationMasks], "originalSize"} (reference
    DataSet.SeqFileFolder.filesToRoiImageFrame)."""
    import io

    from PIL import Image

    from .seqfile import read_sequence_file

    for path in sorted(glob.glob(os.path.join(folder, "*.seq"))):
        for key, value in read_sequence_file(path):
            d = COCODeserializer(key)
            name = d.getString()
            h, w, anns = d.getAnnotations()
            if d.getInt() != COCO_MAGIC:
                raise ValueError(f"{path}: corrupted metadata for {name}")
            rgb = np.asarray(Image.open(io.BytesIO(value)).convert("RGB"))
            if rgb.shape[0] != h or rgb.shape[1] != w:
                raise ValueError(f"{path}: {name} decodes to {rgb.shape[:2]}, metadata says {(h, w)}")
            yield {"fileName": name, "image": torch.from_numpy(rgb[..., ::-1].copy()),
                   "classes": torch.tensor([a["categoryId"] for a in anns], dtype=torch.float32),
                   "bboxes": torch.tensor([a["bbox"] for a in anns], dtype=torch.float32).reshape(-1, 4),
                   "isCrowd": torch.tensor([1.0 if a["isCrowd"] else 0.0 for a in anns]),
                   "masks": [a["masks"] for a in anns], "originalSize": (h, w, 3)}
