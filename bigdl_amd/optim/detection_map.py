"""Mean average precision for object detection / instance segmentation (Pascal VOC 2007 11-point, VOC 2010
all-points, COCO 101-point over several IoU thresholds).

Reference: S/optim/ValidationMethod.scala:290-560 (MAPUtil.gtTablesToGroundTruthRegions / parseDetection /
parseSegmentationTensorResult, MAPValidationResult, GroundTruthBBox / GroundTruthRLE), :596-650
(MAPMultiIOUValidationResult), :674-798 (MeanAveragePrecisionObjectDetection) and :800-840
(MeanAveragePrecision.pascalVOC / cocoBBox / cocoSegmentation factories).

Class labels are 0-based, as in the reference. The output is either a [batch, 1 + 6 * maxDet] tensor
(per image: count, then (label, score, x1, y1, x2, y2) per detection) or a Table of per-image Tables with
``classes`` / ``bboxes`` / ``scores`` (and ``masks`` as RLEs for segmentation); the target is a Table of
per-image Tables with ``classes`` ([n] or [2, n] with the difficult flag), ``bboxes``, ``is_crowd``
(and ``masks``). This runs on the host: it is bookkeeping over a few hundred boxes per image.
"""
from ..utils.table import Table
from .validation import ValidationMethod, ValidationResult

MAPPascalVoc2007, MAPPascalVoc2010, MAPCOCO = "voc2007", "voc2010", "coco"
CLASSES, BBOXES, MASKS, ISCROWD, SCORES = "classes", "bboxes", "masks", "is_crowd", "scores"


class _GT:
    """One ground-truth region; ``occupied[i]`` marks a match at IoU threshold i."""

    def __init__(self, coco, n_iou, label, diff, box=None, rle=None):
        self.coco, self.label, self.diff = coco, label, diff
        self.occupied = [False] * n_iou
        self.box, self.rle = box, rle
        if box is not None:
            x1, y1, x2, y2 = box
            self.area = (x2 - x1 + 1) * (y2 - y1 + 1)

    def can_occupy(self, i):
        return (self.coco and self.diff == 1) or not self.occupied[i]

    def iou(self, x1, y1, x2, y2, rle=None):
        if self.rle is not None:
            from ..dataset.segmentation import rle_iou

            return float(rle_iou(rle, self.rle, self.diff != 0))
        gx1, gy1, gx2, gy2 = self.box
        iw = max(min(gx2, x2) - max(gx1, x1) + 1, 0.0)
        ih = max(min(gy2, y2) - max(gy1, y1) + 1, 0.0)
        inter = iw * ih
        det = (x2 - x1 + 1) * (y2 - y1 + 1)
        union = det if (self.coco and self.diff != 0) else det + self.area - inter
        return inter / union


def _get(t, key):
    if isinstance(t, Table):
        return t.get(key) if key in t.keys() else None
    return t.get(key) if isinstance(t, dict) else None


def _images(tbl):
    if isinstance(tbl, Table):
        return [tbl[i] for i in range(1, tbl.length() + 1)]
    return list(tbl)


def _ground_truth(target, classes, n_iou, coco, seg):
    cnt = [0] * classes
    images = []
    for img in _images(target):
        regions = []
        bb = _get(img, BBOXES)
        if bb is not None and bb.numel() > 0:
            bb = bb.reshape(-1, 4).float()
            cl = _get(img, CLASSES).float()
            crowd = _get(img, ISCROWD)
            masks = _get(img, MASKS) if seg else None
            n = bb.shape[0]
            if (cl.shape[1] if cl.dim() == 2 else cl.numel()) != n:
                raise ValueError("CLASSES of target tables should have the same size of the bbox counts")
            if crowd is None or crowd.numel() != n:
                raise ValueError("ISCROWD of target tables should have the same size of the bbox counts")
            for j in range(n):
                if cl.dim() == 2:
                    label, d = int(cl[0, j]), float(cl[1, j])
                else:
                    label, d = int(cl[j]), 0.0
                diff = 1.0 if (float(crowd.reshape(-1)[j]) != 0 or d != 0) else 0.0
                if not 0 <= label < classes:
                    raise ValueError(f"Bad label id {label}")
                if seg:
                    regions.append(_GT(True, n_iou, label, diff, rle=masks[j]))
                else:
                    regions.append(_GT(coco, n_iou, label, diff, box=[float(v) for v in bb[j]]))
                if diff == 0:
                    cnt[label] += 1
        images.append(regions)
    return images, cnt


def _parse_detection(gts, label, score, box, rle, classes, ious, preds):
    if not 0 <= label < classes:
        raise ValueError(f"Bad label id {label}")
    for i, thr in enumerate(ious):
        best = None
        for gt in gts:
            if gt.label != label or not gt.can_occupy(i):
                continue
            r = gt.iou(*box, rle)
            if r < thr:
                continue
            if best is None:
                best = (gt, r)
            elif best[0].diff != gt.diff:
                if best[0].diff > gt.diff:   # prefer the non-difficult region
                    best = (gt, r)
            elif r >= best[1]:
                best = (gt, r)
        if best is not None:
            best[0].occupied[i] = True
        if best is None or best[0].diff == 0:
            preds[i][label].append((score, best is not None))
        # a match with a "difficult" region is neither a true nor a false positive


class MAPValidationResult(ValidationResult):
    def __init__(self, nClass, k, predictForClass, gtCntForClass, theType=MAPPascalVoc2010, skipClass=-1,
                 isSegmentation=False):
        if skipClass < -1 or skipClass >= nClass:
            raise ValueError(f"Invalid skipClass {skipClass}")
        self.nClass, self.k, self.theType, self.skipClass, self.isSegmentation = \
            nClass, k, theType, skipClass, isSegmentation
        self.predictForClass = [list(p) for p in predictForClass]
        self.gtCntForClass = list(gtCntForClass)

    def _sorted(self, p):
        return sorted(p, key=lambda v: -v[0])     # stable: ties keep insertion order, like sortBy

    def calculateClassAP(self, c):
        pos = self.gtCntForClass[c]
        preds = self._sorted(self.predictForClass[c])
        kk = self.k if self.k > 0 else len(preds)
        pr, tp = [], 0
        for j, (_, hit) in enumerate(preds[:kk]):
            if hit:
                tp += 1
                pr.append((tp / pos if pos else float("inf"), tp / (j + 1)))

        def pmax(recall):
            vals = [p for r, p in pr if r >= recall]
            return max(vals) if vals else 0.0

        if self.theType == MAPPascalVoc2007:
            return sum(pmax(0.1 * r) for r in range(11)) / 11
        if self.theType == MAPPascalVoc2010:
            if pos == 0:
                return 0.0
            return sum(pmax(r / pos) for r in range(1, pos + 1)) / pos
        if pos == 0:
            return -1.0
        return sum(pmax(0.01 * r) for r in range(101)) / 101

    def result(self):
        aps = [self.calculateClassAP(c) for c in range(self.nClass) if c != self.skipClass]
        if self.theType == MAPCOCO:
            aps = [a for a in aps if a != -1.0]
            return (sum(aps) / len(aps) if aps else 0.0), 1
        return sum(aps) / (self.nClass - (0 if self.skipClass == -1 else 1)), 1

    def _merge_preds(self, o):
        for i in range(len(self.predictForClass)):
            merged = self.predictForClass[i] + o.predictForClass[i]
            self.predictForClass[i] = merged if self.k < 0 else self._sorted(merged)[:self.k]

    def __add__(self, o):
        self._merge_preds(o)
        self.gtCntForClass = [a + b for a, b in zip(self.gtCntForClass, o.gtCntForClass)]
        return self

    def format(self):
        kind = "segm" if self.isSegmentation else "bbox"
        per = "".join(f"AP of class {c} = {self.calculateClassAP(c)}\n" for c in range(self.nClass))
        return f"MeanAveragePrecision_{kind}@{self.k}({self.result()[0]})\n {per}"

    def __repr__(self):
        return self.format()


class MAPMultiIOUValidationResult(ValidationResult):
    def __init__(self, nClass, k, predictForClassIOU, gtCntForClass, iouRange, theType=MAPPascalVoc2010,
                 skipClass=-1, isSegmentation=False):
        self.iouRange, self.isSegmentation = iouRange, isSegmentation
        self.gtCntForClass = list(gtCntForClass)
        self.impl = [MAPValidationResult(nClass, k, p, self.gtCntForClass, theType, skipClass, isSegmentation)
                     for p in predictForClassIOU]

    def result(self):
        return sum(r.result()[0] for r in self.impl) / len(self.impl), 1

    def __add__(self, o):
        if len(o.impl) != len(self.impl):
            raise ValueError("To merge MAPMultiIOUValidationResult, the number of IoU thresholds must match")
        for a, b in zip(self.impl, o.impl):
            a._merge_preds(b)
        self.gtCntForClass = [a + b for a, b in zip(self.gtCntForClass, o.gtCntForClass)]
        for r in self.impl:
            r.gtCntForClass = self.gtCntForClass
        return self

    def format(self):
        lo, hi = self.iouRange
        step = (hi - lo) / (len(self.impl) - 1)
        res = [r.result()[0] for r in self.impl]
        lines = "".join(f"\t IOU({lo + i * step}) = {v}\n" for i, v in enumerate(res))
        kind = "segm" if self.isSegmentation else "bbox"
        return f"MAP_{kind}@IOU({lo:1.3f}:{step:1.3f}:{hi:1.3f})={sum(res) / len(res)}\n{lines}"

    def __repr__(self):
        return self.format()


class MeanAveragePrecisionObjectDetection(ValidationMethod):
    def __init__(self, classes, topK=-1, iouThres=(0.5,), theType=MAPPascalVoc2010, skipClass=-1,
                 isSegmentation=False):
        self.classes, self.topK, self.iouThres = classes, topK, [float(t) for t in iouThres]
        self.theType, self.skipClass, self.isSegmentation = theType, skipClass, isSegmentation

    def apply(self, output, target):
        n_iou = len(self.iouThres)
        gt_images, gt_cnt = _ground_truth(target, self.classes, n_iou, self.theType == MAPCOCO,
                                          self.isSegmentation)
        preds = [[[] for _ in range(self.classes)] for _ in range(n_iou)]
        if not isinstance(output, Table) and hasattr(output, "dim"):
            if self.isSegmentation:
                raise ValueError("Cannot get segmentation data from tensor output for MAP")
            out = output.float().cpu()
            if out.dim() != 2:
                raise ValueError("the output tensor should have 2 dimensions")
            for img in range(out.shape[0]):
                row = out[img]
                n, off = int(row[0]), 1
                for _ in range(n):
                    label, score = int(row[off]), float(row[off + 1])
                    box = [float(v) for v in row[off + 2:off + 6]]
                    _parse_detection(gt_images[img], label, score, box, None, self.classes, self.iouThres,
                                     preds)
                    off += 6
        else:
            imgs = _images(output)
            if len(imgs) != len(gt_images):
                raise ValueError("The number of images in the output and in the target should be the same")
            for gts, img in zip(gt_images, imgs):
                bb = _get(img, BBOXES)
                if bb is None or bb.numel() == 0:
                    continue
                bb = bb.reshape(-1, 4).float().cpu()
                sc = _get(img, SCORES).reshape(-1).float().cpu()
                cl = _get(img, CLASSES).reshape(-1).float().cpu()
                masks = _get(img, MASKS) if self.isSegmentation else None
                if not (bb.shape[0] == cl.numel() == sc.numel()):
                    raise ValueError("bboxes, classes and scores must have the same count")
                dets = [(int(cl[j]), float(sc[j]), [float(v) for v in bb[j]], masks[j] if masks else None)
                        for j in range(bb.shape[0])]
                dets.sort(key=lambda d: -d[1])
                for label, score, box, rle in dets:
                    _parse_detection(gts, label, score, box, rle, self.classes, self.iouThres, preds)
        if n_iou != 1:
            return MAPMultiIOUValidationResult(self.classes, self.topK, preds, gt_cnt,
                                               (self.iouThres[0], self.iouThres[-1]), self.theType,
                                               self.skipClass, self.isSegmentation)
        return MAPValidationResult(self.classes, self.topK, preds[0], gt_cnt, self.theType, self.skipClass,
                                   self.isSegmentation)

    def format(self):
        return "MAPObjectDetection"


def _coco(nClasses, topK, skipClass, iouThres, seg):
    start, step, n = iouThres
    return MeanAveragePrecisionObjectDetection(nClasses, topK, [start + i * step for i in range(n)], MAPCOCO,
                                               skipClass, seg)


def pascalVOC(nClasses, useVoc2007=False, topK=-1, skipClass=0):
    return MeanAveragePrecisionObjectDetection(nClasses, topK, theType=MAPPascalVoc2007 if useVoc2007
                                               else MAPPascalVoc2010, skipClass=skipClass)


def cocoBBox(nClasses, topK=-1, skipClass=0, iouThres=(0.5, 0.05, 10)):
    return _coco(nClasses, topK, skipClass, iouThres, False)


def cocoSegmentation(nClasses, topK=-1, skipClass=0, iouThres=(0.5, 0.05, 10)):
    return _coco(nClasses, topK, skipClass, iouThres, True)
