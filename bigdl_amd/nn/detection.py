"""Object-detection layers: anchors, priors, proposals, RoI pooling / align, FPN, Faster/Mask R-CNN heads, SSD and
Faster R-CNN detection outputs.

Reference: S/nn/Anchor.scala:25-233, PriorBox.scala:42-346, Nms.scala:26-242, Proposal.scala:34-204,
RoiPooling.scala:42-366, RoiAlign.scala:45-500, Pooler.scala:33-182, FPN.scala:41-153, BoxHead.scala:30-387,
MaskHead.scala:24-174, RegionProposal.scala:40-358, DetectionOutputSSD.scala:49-308,
DetectionOutputFrcnn.scala:48-260, BaseModule.scala:25-85.

Compute mapping: the per-RoI inner loops (RoiAlign sampling, RoiPooling max + argmax scatter, NMS IoU tests)
run in HIP kernels (csrc/detection.hip) when the feature maps live on the GPU; the surrounding bookkeeping
(top-k, per-class filtering, concatenation) is vectorised torch on the same device. All boxes are fp32 —
box arithmetic is not a bandwidth problem and bf16 boxes would shift pixel coordinates.
"""
import math

import numpy as np
import torch

from ..ops import detection as D
from ..utils.table import Table
from .abstractnn import AbstractModule
from .activation import ReLU, Sigmoid, SoftMax
from .containers import Container, Sequential
from .conv import SpatialConvolution, SpatialFullConvolution
from .graph import Graph, Input
from .init_methods import MsraFiller, RandomNormal, Xavier, Zeros
from .linear import Linear
from .pooling import SpatialMaxPooling
from .shape_ops import InferReshape, UpSampling2D
from .table_ops import CAddTable


def _jround(v):
    return math.floor(v + 0.5)   # Java Math.round


def _t(x):
    return x if isinstance(x, torch.Tensor) else torch.as_tensor(x, dtype=torch.float32)


# ------------------------------------------------------------------------------------------ Anchor / Nms
class Anchor:
    """Faster R-CNN anchor generator (reference Anchor.scala:25): basic anchors from ratios x scales around a
    ``baseSize`` window, shifted over the feature-map grid. ``generateAnchors`` returns (H*W*A, 4) in (y, x, a)
    order."""

    def __init__(self, ratios, scales):
        self.ratios = [float(r) for r in ratios]
        self.scales = [float(s) for s in scales]
        self.baseSize = 16.0
        self.anchorNum = len(self.ratios) * len(self.scales)
        self.basicAnchors = self._basic(self.baseSize)

    @staticmethod
    def _info(a):
        w = a[2] - a[0] + 1
        h = a[3] - a[1] + 1
        return w, h, a[0] + 0.5 * (w - 1), a[1] + 0.5 * (h - 1)

    @staticmethod
    def _mk(ws, hs, xc, yc):
        return [[xc - (w / 2 - 0.5), yc - (h / 2 - 0.5), xc + (w / 2 - 0.5), yc + (h / 2 - 0.5)] for w, h in zip(ws, hs)]

    def _basic(self, base):
        f32 = np.float32
        w, h, xc, yc = self._info([0.0, 0.0, base - 1, base - 1])
        area = w * h
        ws = [float(_jround(math.sqrt(area / r))) for r in self.ratios]
        hs = [float(_jround(f32(w_) * f32(r))) for w_, r in zip(ws, self.ratios)]
        ratio_anchors = self._mk(ws, hs, xc, yc)
        out = []
        for ra in ratio_anchors:
            rw, rh, rx, ry = self._info(ra)
            out += self._mk([s * rw for s in self.scales], [s * rh for s in self.scales], rx, ry)
        return torch.tensor(out, dtype=torch.float32)

    def generateAnchors(self, width, height, featStride=16.0, device=None):
        if featStride != self.baseSize:
            self.basicAnchors = self._basic(float(featStride))
            self.baseSize = float(featStride)
        sx = torch.arange(width, dtype=torch.float32) * featStride
        sy = torch.arange(height, dtype=torch.float32) * featStride
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        shifts = torch.stack([xx, yy, xx, yy], dim=-1).reshape(-1, 1, 4)
        out = (shifts + self.basicAnchors.reshape(1, -1, 4)).reshape(-1, 4)
        return out if device is None else out.to(device)


class Nms:
    """Reference Nms.scala API: ``nms`` / ``nmsFast`` write 1-based indices into ``indices`` and return the
    count. Backed by ops.detection (HIP bitmask NMS for device tensors)."""

    def nms(self, scores, boxes, thresh, indices=None, sorted=False, orderWithBBox=False):
        keep = D.nms(_t(scores), _t(boxes), thresh, sorted=sorted, orderWithBBox=orderWithBBox)
        if indices is not None:
            for i, k in enumerate(keep.tolist()):
                indices[i] = k + 1
        return keep.numel()

    def nmsFast(self, scores, boxes, nmsThresh, scoreThresh, indices=None, topk=-1, eta=1.0, normalized=True):
        keep = D.nms_fast(_t(scores), _t(boxes), nmsThresh, scoreThresh, topk, eta, normalized)
        if indices is not None:
            for i, k in enumerate(keep.tolist()):
                indices[i] = k + 1
        return keep.numel()


# ----------------------------------------------------------------------------------------------- PriorBox
class PriorBox(AbstractModule):
    """SSD prior boxes (reference PriorBox.scala:42). Output (1, 2, H*W*numPriors*4): normalised boxes, then
    their variances."""

    def __init__(self, minSizes, maxSizes=None, aspectRatios=None, isFlip=True, isClip=False, variances=None,
                 offset=0.5, imgH=0, imgW=0, imgSize=0, stepH=0.0, stepW=0.0, step=0.0):
        super().__init__()
        assert minSizes, "must provide minSize"
        self.minSizes = [float(v) for v in minSizes]
        self.maxSizes = [float(v) for v in maxSizes] if maxSizes else []
        self.isFlip, self.isClip, self.offset = isFlip, isClip, offset
        ars = [1.0]
        for ar in (aspectRatios or []):
            if not any(abs(ar - a) < 1e-6 for a in ars):
                ars.append(float(ar))
            if isFlip:
                ars.append(1.0 / ar)
        self.aspectRatios = ars
        self.numPriors = len(ars) * len(self.minSizes) + len(self.maxSizes)
        if self.maxSizes:
            assert len(self.maxSizes) == len(self.minSizes)
        self.variances = [float(v) for v in variances] if variances else [0.1]
        assert len(self.variances) in (1, 4), "Must and only provide 4 variance."
        if imgSize and not (imgH and imgW):
            imgH = imgW = imgSize
        if step and not (stepH and stepW):
            stepH = stepW = step
        self.imgH, self.imgW, self.stepH, self.stepW = imgH, imgW, stepH, stepW

    def updateOutput(self, input):
        feat = input if isinstance(input, torch.Tensor) else input[1]
        assert self.imgW > 0 and self.imgH > 0, "imgW and imgH must > 0"
        lh, lw = feat.shape[2], feat.shape[3]
        stepW = self.stepW or self.imgW / float(lw)
        stepH = self.stepH or self.imgH / float(lh)
        f32 = np.float32
        boxes = []
        for s, ms in enumerate(self.minSizes):
            m = int(ms)
            half = [(m / 2.0, m / 2.0)]
            if self.maxSizes:
                hb = f32(math.sqrt(m * int(self.maxSizes[s]))) / 2
                half.append((hb, hb))
            for ar in self.aspectRatios:
                if abs(ar - 1) >= 1e-6:
                    v = f32(math.sqrt(ar))
                    half.append((m * v / 2, m / v / 2))
            boxes += half
        hw = torch.tensor(boxes, dtype=torch.float32)                      # (numPriors, 2) half w, half h
        cx = (torch.arange(lw, dtype=torch.float32) + self.offset) * stepW
        cy = (torch.arange(lh, dtype=torch.float32) + self.offset) * stepH
        yy, xx = torch.meshgrid(cy, cx, indexing="ij")
        cxy = torch.stack([xx, yy], -1).reshape(lh, lw, 1, 2)
        lo = (cxy - hw.reshape(1, 1, -1, 2)) / torch.tensor([self.imgW, self.imgH], dtype=torch.float32)
        hi = (cxy + hw.reshape(1, 1, -1, 2)) / torch.tensor([self.imgW, self.imgH], dtype=torch.float32)
        pri = torch.cat([lo, hi], -1).reshape(-1)
        if self.isClip:
            pri = pri.clamp(0, 1)
        var = torch.tensor(self.variances, dtype=torch.float32)
        var = var.repeat(pri.numel() // 4) if var.numel() == 4 else var.expand(pri.numel()).clone()
        return torch.stack([pri, var]).reshape(1, 2, -1).to(feat.device)

    def updateGradInput(self, input, gradOutput):
        return None


# -------------------------------------------------------------------------------------- RoiPooling/Align
class RoiPooling(AbstractModule):
    """Fast R-CNN RoI max pooling (reference RoiPooling.scala:42). Input Table(data (N,C,H,W), rois (R,5) with
    0-based batch index)."""

    def __init__(self, pooledW, pooledH, spatialScale):
        super().__init__()
        self.pooledW, self.pooledH, self.spatialScale = pooledW, pooledH, float(spatialScale)
        self._argmax = None

    def updateOutput(self, input):
        data, rois = input[1], input[2]
        assert rois.dim() > 1 and rois.shape[1] == 5, "roi input shape should be (R, 5)"
        out, self._argmax = D.roi_pool_forward(data, rois, self.spatialScale, self.pooledH, self.pooledW)
        return out.to(data.dtype)

    def updateGradInput(self, input, gradOutput):
        data, rois = input[1], input[2]
        g = D.roi_pool_backward(gradOutput.float(), self._argmax, rois, tuple(data.shape)).to(data.dtype)
        return Table(g, torch.zeros_like(rois))


class RoiAlign(AbstractModule):
    """Mask R-CNN RoiAlign (reference RoiAlign.scala:45). Input Table(data, rois (R,4) of image 0, or (R,5))."""

    def __init__(self, spatialScale, samplingRatio, pooledH, pooledW):
        super().__init__()
        self.spatialScale, self.samplingRatio = float(spatialScale), int(samplingRatio)
        self.pooledH, self.pooledW = pooledH, pooledW

    def updateOutput(self, input):
        data, rois = input[1], input[2]
        out = D.roi_align(data, rois, self.spatialScale, self.samplingRatio, self.pooledH, self.pooledW)
        assert out.numel() != 0, "Output contains no elements"
        return out

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("Not support backward propagation")


class Pooler(AbstractModule):
    """Multi-level RoiAlign over FPN maps (reference Pooler.scala:33): each box goes to the level
    ``floor(4 + log2(sqrt(area) / 224 + 1e-6))`` clamped to the available levels."""

    def __init__(self, resolution, scales, samplingRatio):
        super().__init__()
        self.resolution, self.scales, self.samplingRatio = resolution, [float(s) for s in scales], samplingRatio
        self.lvl_min = int(-math.log(self.scales[0]) / math.log(2.0))
        self.lvl_max = int(-math.log(self.scales[-1]) / math.log(2.0))

    def _levels(self, rois):
        area = (rois[:, 2] - rois[:, 0] + 1) * (rois[:, 3] - rois[:, 1] + 1)
        s = torch.sqrt(area.double())
        lvl = torch.floor(4 + torch.log(s / 224 + 1e-6) / math.log(2))
        return (lvl.clamp(self.lvl_min, self.lvl_max) - self.lvl_min).long()

    def updateOutput(self, input):
        fmaps = input[1]
        roi_batch = input[2]
        roi_list = [roi_batch] if isinstance(roi_batch, torch.Tensor) else [roi_batch[i + 1] for i in
                                                                           range(roi_batch.length())]
        first = fmaps[1]
        C, dev = first.shape[1], first.device
        res = self.resolution
        outs = []
        for b, rois in enumerate(roi_list):
            rois = rois.to(dev).float()
            out = torch.zeros(rois.shape[0], C, res, res, device=dev)
            if rois.shape[0]:
                lv = self._levels(rois)
                for level in range(len(self.scales)):
                    idx = torch.nonzero(lv == level).reshape(-1)
                    if idx.numel() == 0:
                        continue
                    r5 = torch.cat([torch.full((idx.numel(), 1), float(b), device=dev), rois[idx]], 1)
                    out[idx] = D.roi_align(fmaps[level + 1], r5, self.scales[level], self.samplingRatio, res, res)
            outs.append(out)
        return torch.cat(outs, 0) if len(outs) > 1 else outs[0]

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("Not support backward propagation")


# ----------------------------------------------------------------------------------------- BaseModule
class BaseModule(Container):
    """A module whose body is a model built by ``buildModel()`` (reference BaseModule.scala:25)."""

    def __init__(self):
        super().__init__()
        self.model = self.buildModel()
        self.modules = [self.model]

    def buildModel(self):
        raise NotImplementedError

    def _set_children(self, children):
        self.model = children[0]
        self.modules = [self.model]

    def updateOutput(self, input):
        return self.model.forward(input)

    def updateGradInput(self, input, gradOutput):
        return self.model.updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        self.model.accGradParameters(input, gradOutput)

    def backward(self, input, gradOutput):
        self.gradInput = self.model.backward(input, gradOutput)
        return self.gradInput


class FPN(BaseModule):
    """Feature Pyramid Network (reference FPN.scala:41): lateral 1x1 convs, nearest 2x top-down path, 3x3 output
    convs; ``topBlocks`` 1 adds a stride-2 max-pool P6, 2 adds P6/P7 convs (RetinaNet)."""

    def __init__(self, inChannels, outChannels, topBlocks=0, inChannelsOfP6P7=0, outChannelsOfP6P7=0):
        self.inChannels, self.outChannels, self.topBlocks = list(inChannels), outChannels, topBlocks
        self.inChannelsOfP6P7, self.outChannelsOfP6P7 = inChannelsOfP6P7, outChannelsOfP6P7
        super().__init__()

    def buildModel(self):
        n = len(self.inChannels)
        inner, layer = [None] * n, [None] * n
        for i, c in enumerate(self.inChannels):
            if c != 0:
                inner[i] = SpatialConvolution(c, self.outChannels, 1, 1, 1, 1).setName(f"fpn_inner{i + 1}")
                layer[i] = SpatialConvolution(self.outChannels, self.outChannels, 3, 3, 1, 1, 1, 1).setName(
                    f"fpn_layer{i + 1}")
        inputs = [Input() for _ in range(n)]
        inner_nodes = [inner[i].inputs(inputs[i]) for i in range(n)]
        results = [None] * (n + self.topBlocks)
        count = len(results) - 1 - self.topBlocks
        last = inner_nodes[n - 1]
        results[count] = layer[n - 1].inputs(last)
        for i in range(n - 2, -1, -1):
            if layer[i] is not None:
                top_down = UpSampling2D([2, 2]).inputs(last)
                last = CAddTable().setName(f"number_{i}_{n}").inputs(inner_nodes[i], top_down)
                count -= 1
                results[count] = layer[i].inputs(last)
        if self.topBlocks == 1:
            results[-1] = SpatialMaxPooling(1, 1, 2, 2).inputs(results[n - 1])
        if self.topBlocks == 2:
            p6 = SpatialConvolution(self.inChannelsOfP6P7, self.outChannelsOfP6P7, 3, 3, 2, 2, 1, 1)
            p7 = SpatialConvolution(self.outChannelsOfP6P7, self.outChannelsOfP6P7, 3, 3, 2, 2, 1, 1)
            src = results[n - 1] if self.inChannelsOfP6P7 == self.outChannelsOfP6P7 else inputs[n - 1]
            results[-2] = p6.inputs(src)
            results[-1] = p7.inputs(ReLU().inputs(results[-2]))
        return Graph(inputs, results)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("Not support backward propagation")

    def __repr__(self):
        return f"FPN({self.outChannels})"


# ------------------------------------------------------------------------------------------ Box head
def _per_class_nms(scores, boxes, n_classes, score_thresh, nms_thresh, order_with_bbox):
    """[(label, scores_k, boxes_k)] for classes 1..n_classes-1 (reference postProcessOneClass)."""
    res = [None] * n_classes
    for c in range(1, n_classes):
        inds = torch.nonzero(scores[:, c] > score_thresh).reshape(-1)
        if inds.numel() == 0:
            continue
        cs = scores[inds, c]
        cb = boxes[inds, 4 * c: 4 * c + 4]
        keep = D.nms(cs, cb, nms_thresh, orderWithBBox=order_with_bbox)
        res[c] = (cs[keep], cb[keep])
    return res


def _limit_max_per_image(res, max_per_image):
    scores = [r[0] for r in res if r is not None]
    total = sum(int(s.numel()) for s in scores)
    if max_per_image <= 0 or total <= max_per_image:
        return res
    allsc = torch.sort(torch.cat(scores)).values
    thresh = allsc[total - max_per_image]
    out = list(res)
    for c, r in enumerate(res):
        if r is None:
            continue
        keep = r[0] >= thresh
        out[c] = (r[0][keep], r[1][keep])
    return out


class BoxPostProcessor(AbstractModule):
    """Mask R-CNN box post-processing (reference BoxHead.scala BoxPostProcessor): softmax, weighted box decode,
    clip, per-class NMS, top-``maxPerImage``. Output Table(labels, Table(per-image boxes), scores)."""

    def __init__(self, scoreThresh, nmsThresh, maxPerImage, nClasses, weight=(10.0, 10.0, 5.0, 5.0)):
        super().__init__()
        self.scoreThresh, self.nmsThresh, self.maxPerImage = scoreThresh, nmsThresh, maxPerImage
        self.nClasses, self.weight = nClasses, tuple(weight)

    def updateOutput(self, input):
        if self.train:
            return input
        logits, reg, bbox, info = input[1], input[2], input[3], input[4]
        per_img = [bbox] if isinstance(bbox, torch.Tensor) else [bbox[i + 1] for i in range(bbox.length())]
        counts = [int(b.shape[0]) for b in per_img]
        concat = torch.cat([b.float() for b in per_img], 0).to(reg.device)
        prob = torch.softmax(logits.float(), dim=1)
        boxes = D.decode_with_weight(reg.float(), concat, self.weight)
        D.clip_boxes(boxes, float(info.reshape(-1)[0]), float(info.reshape(-1)[1]))
        labels, scores, out_boxes = [], [], Table()
        start = 0
        for i, n in enumerate(counts):
            res = _per_class_nms(prob[start:start + n], boxes[start:start + n], self.nClasses, self.scoreThresh,
                                 self.nmsThresh, True)
            res = _limit_max_per_image(res, self.maxPerImage)
            start += n
            bl, ls, ss = [], [], []
            for c, r in enumerate(res):
                if r is None:
                    continue
                bl.append(r[1])
                ss.append(r[0])
                ls.append(torch.full((r[0].numel(),), float(c), device=r[0].device))
            out_boxes[i + 1] = torch.cat(bl, 0) if bl else torch.zeros(0, 4, device=reg.device)
            labels += ls
            scores += ss
        lab = torch.cat(labels) if labels else torch.zeros(0, device=reg.device)
        sco = torch.cat(scores) if scores else torch.zeros(0, device=reg.device)
        return Table(lab, out_boxes, sco)

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class BoxHead(BaseModule):
    """Mask R-CNN box head (reference BoxHead.scala:30): Pooler -> fc1 -> ReLU -> fc2 -> ReLU -> (cls, bbox) ->
    BoxPostProcessor. Graph inputs (features, proposals, imageInfo); outputs (boxFeatures, result)."""

    def __init__(self, inChannels, resolution=7, scales=(0.25, 0.125, 0.0625, 0.03125), samplingRatio=2,
                 scoreThresh=0.05, nmsThresh=0.5, maxPerImage=100, outputSize=1024, numClasses=81):
        self.inChannels, self.resolution, self.scales = inChannels, resolution, list(scales)
        self.samplingRatio, self.scoreThresh, self.nmsThresh = samplingRatio, scoreThresh, nmsThresh
        self.maxPerImage, self.outputSize, self.numClasses = maxPerImage, outputSize, numClasses
        super().__init__()

    def buildModel(self):
        fe = Sequential().add(Pooler(self.resolution, self.scales, self.samplingRatio)).add(InferReshape([0, -1]))
        fc1 = Linear(self.inChannels * self.resolution ** 2, self.outputSize).setInitMethod(Xavier(), Zeros())
        fc2 = Linear(self.outputSize, self.outputSize).setInitMethod(Xavier(), Zeros())
        fe.add(fc1).add(ReLU()).add(fc2).add(ReLU())
        cls = Linear(self.outputSize, self.numClasses).setInitMethod(RandomNormal(0, 0.01), Zeros())
        box = Linear(self.outputSize, self.numClasses * 4).setInitMethod(RandomNormal(0, 0.001), Zeros())
        post = BoxPostProcessor(self.scoreThresh, self.nmsThresh, self.maxPerImage, self.numClasses)
        features, proposals, info = Input(), Input(), Input()
        feats = fe.inputs(features, proposals)
        result = post.inputs(cls.inputs(feats), box.inputs(feats), proposals, info)
        return Graph([features, proposals, info], [feats, result])


# ----------------------------------------------------------------------------------------- Mask head
class MaskPostProcessor(AbstractModule):
    """sigmoid(mask logits) of each RoI's predicted class (reference MaskHead.scala MaskPostProcessor)."""

    def updateOutput(self, input):
        logits, labels = input[1], input[2]
        assert labels.dim() == 1, "Labels should be tensor with one dimension"
        assert labels.numel() == logits.shape[0], "number of masks should be same with labels"
        prob = torch.sigmoid(logits.float())
        idx = labels.long().to(prob.device)
        return prob[torch.arange(prob.shape[0], device=prob.device), idx].unsqueeze(1)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("MaskPostProcessor only support inference")


class MaskHead(BaseModule):
    """Mask R-CNN mask head (reference MaskHead.scala:24): Pooler -> 4 x (3x3 conv + ReLU) -> 2x2/2 deconv ->
    ReLU -> 1x1 class conv -> per-class sigmoid selection."""

    def __init__(self, inChannels, resolution=14, scales=(0.25, 0.125, 0.0625, 0.03125), samplingRatio=2,
                 layers=(256, 256, 256, 256), dilation=1, numClasses=81, useGn=False):
        assert dilation == 1, f"Only support dilation = 1, but got {dilation}"
        self.inChannels, self.resolution, self.scales = inChannels, resolution, list(scales)
        self.samplingRatio, self.layers, self.dilation = samplingRatio, list(layers), dilation
        self.numClasses, self.useGn = numClasses, useGn
        super().__init__()

    def buildModel(self):
        fe = Sequential().add(Pooler(self.resolution, self.scales, self.samplingRatio))
        nxt = self.inChannels
        for i, f in enumerate(self.layers):
            conv = SpatialConvolution(nxt, f, 3, 3, 1, 1, self.dilation, self.dilation,
                                      withBias=not self.useGn).setName(f"mask_fcn{i + 1}")
            conv.setInitMethod(MsraFiller(False), Zeros())
            fe.add(conv).add(ReLU())
            nxt = f
        dim = self.layers[-1]
        deconv = SpatialFullConvolution(dim, dim, 2, 2, 2, 2).setInitMethod(MsraFiller(False), Zeros())
        logits = SpatialConvolution(dim, self.numClasses, 1, 1, 1, 1).setInitMethod(MsraFiller(False), Zeros())
        pred = Sequential().add(deconv).add(ReLU()).add(logits)
        features, proposals, labels = Input(), Input(), Input()
        feats = fe.inputs(features, proposals)
        result = MaskPostProcessor().inputs(pred.inputs(feats), labels)
        return Graph([features, proposals, labels], [feats, result])


# ----------------------------------------------------------------------------------- Region proposal
class ProposalPostProcessor(AbstractModule):
    """Per-level RPN box selection (reference RegionProposal.scala ProposalPostProcessor): sigmoid objectness,
    pre-NMS top-k, decode against anchors, clip, NMS(0.7). Output Table(boxes (K,4), scores (K))."""

    def __init__(self, preNmsTopNTest=1000, postNmsTopNTest=1000, preNmsTopNTrain=2000, postNmsTopNTrain=2000,
                 nmsThread=0.7, minSize=0):
        super().__init__()
        self.preNmsTopNTest, self.postNmsTopNTest = preNmsTopNTest, postNmsTopNTest
        self.preNmsTopNTrain, self.postNmsTopNTrain = preNmsTopNTrain, postNmsTopNTrain
        self.nmsThread, self.minSize = nmsThread, minSize

    def updateOutput(self, input):
        anchors, obj, reg, size = input[1], input[2], input[3], input[4]
        N, A, H, W = obj.shape
        assert N == 1, "ProposalPostProcessor processes one image"
        obj = torch.sigmoid(obj.float().permute(0, 2, 3, 1).reshape(-1))        # (h, w, a)
        reg = reg.float().reshape(A, 4, H, W).permute(2, 3, 0, 1).reshape(-1, 4)
        top = min(self.preNmsTopNTrain if self.train else self.preNmsTopNTest, obj.numel())
        sc, ind = torch.topk(obj, top, sorted=True)
        props = D.bbox_transform_inv(anchors.to(reg.device)[ind], reg[ind], normalized=True)
        sc_clip = sc.clone()
        size = size.reshape(-1)
        D.clip_boxes(props, float(size[0]), float(size[1]), self.minSize, self.minSize, sc_clip)
        keep = D.nms_sorted(props, self.nmsThread)
        return Table(props[keep], sc[keep])

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("ProposalPostProcessor only support inference")


class RegionProposal(Container):
    """FPN region proposal network (reference RegionProposal.scala:40). Input Table(features Table, image size
    (h, w)); output Table of per-image proposals (postNmsTopN, 4)."""

    def __init__(self, inChannels, anchorSizes=(32, 64, 128, 256, 512), aspectRatios=(0.5, 1.0, 2.0),
                 anchorStride=(4, 8, 16, 32, 64), preNmsTopNTest=1000, postNmsTopNTest=1000, preNmsTopNTrain=2000,
                 postNmsTopNTrain=2000, nmsThread=0.7, minSize=0):
        super().__init__()
        assert len(anchorSizes) == len(anchorStride), "length of anchor size and stride should be same"
        self.inChannels, self.anchorSizes, self.aspectRatios = inChannels, list(anchorSizes), list(aspectRatios)
        self.anchorStride = list(anchorStride)
        self.postNmsTopNTest, self.postNmsTopNTrain = postNmsTopNTest, postNmsTopNTrain
        self.anchors = [Anchor(self.aspectRatios, [s / st]) for s, st in zip(self.anchorSizes, self.anchorStride)]
        self.numAnchors = self.anchors[0].anchorNum
        self.head = self._rpn_head(inChannels, self.numAnchors)
        self.modules = [self.head]
        self.boxSelector = ProposalPostProcessor(preNmsTopNTest, postNmsTopNTest, preNmsTopNTrain, postNmsTopNTrain,
                                                 nmsThread, minSize)

    def _set_children(self, children):
        self.head = children[0]
        self.modules = [self.head]

    @staticmethod
    def _rpn_head(c, a):
        conv = SpatialConvolution(c, c, 3, 3, 1, 1, 1, 1).setInitMethod(RandomNormal(0.0, 0.01), Zeros())
        cls = SpatialConvolution(c, a, 1, 1, 1, 1).setInitMethod(RandomNormal(0.0, 0.01), Zeros())
        box = SpatialConvolution(c, a * 4, 1, 1, 1, 1).setInitMethod(RandomNormal(0.0, 0.01), Zeros())
        inp = Input()
        r = ReLU().inputs(conv.inputs(inp))
        return Graph(inp, [cls.inputs(r), box.inputs(r)])

    def anchorGenerator(self, features):
        res = []
        for i in range(min(len(self.anchorSizes), features.length())):
            f = features[i + 1]
            res.append(self.anchors[i].generateAnchors(f.shape[3], f.shape[2], self.anchorStride[i], f.device))
        return res

    def updateOutput(self, input):
        features, size = input[1], input[2]
        anchors = self.anchorGenerator(features)
        self.boxSelector.train = self.train
        batch = features[1].shape[0]
        out = Table()
        for b in range(batch):
            boxes, scores = [], []
            for i, anc in enumerate(anchors):
                ho = self.head.forward(features[i + 1][b:b + 1])
                sel = self.boxSelector.forward(Table(anc, ho[1], ho[2], size))
                boxes.append(sel[1])
                scores.append(sel[2])
            allb, alls = torch.cat(boxes), torch.cat(scores)
            post = min(self.postNmsTopNTrain if self.train else self.postNmsTopNTest, alls.numel())
            _, idx = torch.topk(alls, post, sorted=True)
            out[b + 1] = allb[idx]
        return out

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("RegionProposal only support inference")

    def accGradParameters(self, input, gradOutput):
        raise NotImplementedError("RegionProposal only support inference")


# -------------------------------------------------------------------------------------------- Proposal
class Proposal(AbstractModule):
    """Faster R-CNN (VGG / PVANet) proposal layer (reference Proposal.scala:34). Input Table(scores (1, 2A, H, W),
    bbox deltas (1, 4A, H, W), imInfo (1, 4)); output (K, 5) rois with batch index 0."""

    def __init__(self, preNmsTopN, postNmsTopN, ratios, scales, rpnPreNmsTopNTrain=12000, rpnPostNmsTopNTrain=2000):
        super().__init__()
        self.preNmsTopNTest, self.postNmsTopNTest = preNmsTopN, postNmsTopN
        self.rpnPreNmsTopNTrain, self.rpnPostNmsTopNTrain = rpnPreNmsTopNTrain, rpnPostNmsTopNTrain
        self.ratios, self.scales = list(ratios), list(scales)
        self.anchorUtil = Anchor(self.ratios, self.scales)
        self.minSize = 16

    def updateOutput(self, input):
        score, deltas, info = input[1].float(), input[2].float(), input[3].float()
        assert score.shape[0] == 1 and info.shape[0] == 1, "currently only support single batch"
        A = self.anchorUtil.anchorNum
        bbox_deltas = deltas[0].permute(1, 2, 0).reshape(-1, 4)
        scores = score[0, A:2 * A].permute(1, 2, 0).reshape(-1).clone()
        anchors = self.anchorUtil.generateAnchors(score.shape[3], score.shape[2], device=score.device)
        props = D.bbox_transform_inv(anchors, bbox_deltas)
        iv = info.reshape(-1)
        keep_n = D.clip_boxes(props, float(iv[0]), float(iv[1]), self.minSize * float(iv[2]),
                              self.minSize * float(iv[3]), scores)
        pre = self.rpnPreNmsTopNTrain if self.train else self.preNmsTopNTest
        post = self.rpnPostNmsTopNTrain if self.train else self.postNmsTopNTest
        top = min(pre, keep_n)
        sc, ind = torch.topk(scores, top, sorted=True)
        filtered = props[ind]
        keep = D.nms_sorted(filtered, 0.7)
        if post > 0:
            keep = keep[:post]
        rois = filtered[keep]
        return torch.cat([torch.zeros(rois.shape[0], 1, device=rois.device), rois], 1)

    def updateGradInput(self, input, gradOutput):
        return None


# --------------------------------------------------------------------------------- detection outputs
class DetectionOutputSSD(AbstractModule):
    """SSD detection output (reference DetectionOutputSSD.scala:49). Input Table(loc, conf, priors); output
    (batch, 1 + maxDet * 6) rows: [numDet, (label, score, x1, y1, x2, y2) * numDet]."""

    def __init__(self, nClasses=21, shareLocation=True, bgLabel=0, nmsThresh=0.45, nmsTopk=400, keepTopK=200,
                 confThresh=0.01, varianceEncodedInTarget=False, confPostProcess=True):
        super().__init__()
        self.nClasses, self.shareLocation, self.bgLabel = nClasses, shareLocation, bgLabel
        self.nmsThresh, self.nmsTopk, self.keepTopK, self.confThresh = nmsThresh, nmsTopk, keepTopK, confThresh
        self.varianceEncodedInTarget, self.confPostProcess = varianceEncodedInTarget, confPostProcess

    def setTopK(self, topK):
        self.keepTopK = topK
        return self

    def updateOutput(self, input):
        if self.train:
            return input
        loc, conf, prior = input[1].float(), input[2].float(), input[3].float()
        B = loc.shape[0]
        nP = prior.shape[2] // 4
        nl = 1 if self.shareLocation else self.nClasses
        if self.confPostProcess:
            conf = torch.softmax(conf.reshape(B, -1, self.nClasses), dim=2).reshape(B, -1)
        locs = loc.reshape(B, nP, nl, 4)
        confs = conf.reshape(B, nP, self.nClasses)
        pboxes, pvars = prior[0, 0].reshape(nP, 4), prior[0, 1].reshape(nP, 4)
        results, counts = [], []
        for b in range(B):
            decoded = [D.decode_boxes(pboxes, pvars, False, locs[b, :, c], self.varianceEncodedInTarget)
                       for c in range(nl)]
            dets = []
            for c in range(self.nClasses):
                if c == self.bgLabel:
                    continue
                bx = decoded[0 if self.shareLocation else c]
                keep = D.nms_fast(confs[b, :, c], bx, self.nmsThresh, self.confThresh, self.nmsTopk, 1.0, True)
                dets.append((c, confs[b, keep, c], bx[keep]))
            num = sum(int(d[1].numel()) for d in dets)
            if -1 < self.keepTopK < num:
                allsc = torch.cat([d[1] for d in dets])
                thr_idx = torch.sort(allsc, descending=True, stable=True).indices[: self.keepTopK]
                mask = torch.zeros(allsc.numel(), dtype=torch.bool, device=allsc.device)
                mask[thr_idx] = True
                off, nd = 0, []
                for c, s, bx in dets:
                    m = mask[off: off + s.numel()]
                    off += s.numel()
                    o = torch.sort(s[m], descending=True, stable=True).indices
                    nd.append((c, s[m][o], bx[m][o]))
                dets, num = nd, self.keepTopK
            rows = [torch.cat([torch.full((s.numel(), 1), float(c), device=s.device), s[:, None], bx], 1)
                    for c, s, bx in dets if s.numel()]
            results.append(torch.cat(rows) if rows else torch.zeros(0, 6, device=loc.device))
            counts.append(num)
        maxd = max(counts) if counts else 0
        out = torch.zeros(B, 1 + maxd * 6, device=loc.device)
        if sum(counts) > 0:
            for b in range(B):
                out[b, 0] = counts[b]
                out[b, 1: 1 + counts[b] * 6] = results[b].reshape(-1)
        return out

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class DetectionOutputFrcnn(AbstractModule):
    """Faster R-CNN detection output (reference DetectionOutputFrcnn.scala:48). Input Table(imInfo (1,4), rois
    (R,5), box deltas (R, 4*nClasses), scores (R, nClasses)); output (1, 1 + numDet * 6)."""

    def __init__(self, nmsThresh=0.3, nClasses=21, bboxVote=False, maxPerImage=100, thresh=0.05):
        super().__init__()
        self.nmsThresh, self.nClasses, self.bboxVote = nmsThresh, nClasses, bboxVote
        self.maxPerImage, self.thresh = maxPerImage, thresh

    def process(self, scores, deltas, rois, info):
        iv = info.reshape(-1).float()
        boxes = rois[:, 1:5].float().clone()
        D.scale_bbox(boxes, 1.0 / float(iv[2]), 1.0 / float(iv[3]))
        pred = D.bbox_transform_inv(boxes, deltas.float())
        D.clip_boxes(pred, float(iv[0] / iv[2]), float(iv[1] / iv[3]))
        res = [None] * self.nClasses
        for c in range(1, self.nClasses):
            inds = torch.nonzero(scores[:, c] > self.thresh).reshape(-1)
            if inds.numel() == 0:
                continue
            cs, cb = scores[inds, c].float(), pred[inds, 4 * c: 4 * c + 4]
            keep = D.nms(cs, cb, self.nmsThresh)
            ks, kb = cs[keep], cb[keep]
            if self.bboxVote:
                ks, kb = D.bbox_vote(ks, kb, cs, cb)
            res[c] = (ks, kb)
        # reference filters on the last box column (a bug); the score threshold is what is meant
        return _limit_max_per_image(res, self.maxPerImage)

    def updateOutput(self, input):
        if self.train:
            return input
        info, rois_d, deltas, scores = input[1], input[2], input[3], input[4]
        rois = rois_d if isinstance(rois_d, torch.Tensor) else rois_d[1]
        assert info.dim() == 2 and tuple(info.shape) == (1, 4), "imInfo should be a 1x4 tensor"
        assert rois.shape[1] == 5, "rois is a Nx5 tensor"
        assert deltas.shape[1] == self.nClasses * 4 and scores.shape[1] == self.nClasses
        res = self.process(scores.float(), deltas, rois, info)
        rows = [torch.cat([torch.full((r[0].numel(), 1), float(c), device=r[0].device), r[0][:, None], r[1]], 1)
                for c, r in enumerate(res) if r is not None and r[0].numel()]
        det = torch.cat(rows) if rows else torch.zeros(0, 6, device=scores.device)
        out = torch.zeros(1, 1 + det.shape[0] * 6, device=scores.device)
        out[0, 0] = det.shape[0]
        out[0, 1:] = det.reshape(-1)
        return out

    def updateGradInput(self, input, gradOutput):
        return gradOutput


__all__ = ["Anchor", "Nms", "PriorBox", "RoiPooling", "RoiAlign", "Pooler", "BaseModule", "FPN", "BoxPostProcessor",
           "BoxHead", "MaskPostProcessor", "MaskHead", "ProposalPostProcessor", "RegionProposal", "Proposal",
           "DetectionOutputSSD", "DetectionOutputFrcnn"]
