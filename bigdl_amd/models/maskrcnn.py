"""Mask R-CNN (ResNet-50-FPN) inference model.

Reference: S/models/maskrcnn/MaskRCNN.scala:38-443 (MaskRCNNParams, ResNet-50 C2-C5 backbone + FPN(topBlocks=1),
RegionProposal, BoxHead, MaskHead, per-image post-processing into RLE masks) and models/maskrcnn/Utils.scala:28-213
(expandBoxes / expandMasks / decodeMaskInImage / bilinear paste).

Input: Table(images (N, 3, H, W), imageInfo (N, 4) = [scaled h, scaled w, original h, original w]).
Eval output: Table of per-image Tables {"masks": [RLEMasks], "bboxes": (k, 4), "classes": (k), "scores": (k)}.
The backbone / FPN / heads run on the GPU engine (implicit-GEMM convs, HIP RoiAlign and NMS); mask pasting
and RLE encoding are host-side per detection.
"""
import math

import torch
import torch.nn.functional as F

from .. import nn
from ..dataset.segmentation import binary_to_rle
from ..nn.containers import Container
from ..nn.detection import FPN, BoxHead, MaskHead, RegionProposal
from ..ops import detection as D
from ..utils.table import Table
from .resnet import Convolution, Sbn

MASKS, BBOXES, CLASSES, SCORES = "masks", "bboxes", "classes", "scores"


class MaskRCNNParams:
    def __init__(self, anchorSizes=(32, 64, 128, 256, 512), aspectRatios=(0.5, 1.0, 2.0),
                 anchorStride=(4, 8, 16, 32, 64), preNmsTopNTest=1000, postNmsTopNTest=1000, preNmsTopNTrain=2000,
                 postNmsTopNTrain=2000, rpnNmsThread=0.7, minSize=0, boxResolution=7, maskResolution=14,
                 scales=(0.25, 0.125, 0.0625, 0.03125), samplingRatio=2, boxScoreThresh=0.05, boxNmsThread=0.5,
                 maxPerImage=100, outputSize=1024, layers=(256, 256, 256, 256), dilation=1, useGn=False):
        self.__dict__.update({k: (list(v) if isinstance(v, tuple) else v) for k, v in locals().items()
                              if k != "self"})


def _bottleneck(nin, internal, nout, stride, use_conv):
    s = nn.Sequential()
    s.add(Convolution(nin, internal, 1, 1, stride, stride, 0, 0)).add(Sbn(internal)).add(nn.ReLU(True))
    s.add(Convolution(internal, internal, 3, 3, 1, 1, 1, 1)).add(Sbn(internal)).add(nn.ReLU(True))
    s.add(Convolution(internal, nout, 1, 1, 1, 1, 0, 0)).add(Sbn(nout))
    short = (nn.Sequential().add(Convolution(nin, nout, 1, 1, stride, stride)).add(Sbn(nout)) if use_conv
             else nn.Identity())
    return nn.Sequential().add(nn.ConcatTable().add(s).add(short)).add(nn.CAddTable(True)).add(nn.ReLU(True))


def _layer(count, nin, planes, nout, stride=1):
    s = nn.Sequential().add(_bottleneck(nin, planes, nout, stride, True))
    for _ in range(2, count + 1):
        s.add(_bottleneck(nout, planes, nout, 1, False))
    return s


def build_resnet50_c2c5(in_channels):
    stem = nn.Sequential()
    stem.add(Convolution(3, 64, 7, 7, 2, 2, 3, 3, optnet=False, propagateBack=False)).add(Sbn(64))
    stem.add(nn.ReLU(True)).add(nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1))
    inp = nn.Input()
    n0 = stem.inputs(inp)
    n1 = _layer(3, 64, 64, in_channels, 1).inputs(n0)
    n2 = _layer(4, in_channels, 128, in_channels * 2, 2).inputs(n1)
    n3 = _layer(6, in_channels * 2, 256, in_channels * 4, 2).inputs(n2)
    n4 = _layer(3, in_channels * 4, 512, in_channels * 8, 2).inputs(n3)
    return nn.Graph(inp, [n1, n2, n3, n4])


def expand_boxes(box, scale):
    w_half = (box[2] - box[0]) * 0.5 * scale
    h_half = (box[3] - box[1]) * 0.5 * scale
    xc, yc = (box[2] + box[0]) * 0.5, (box[3] + box[1]) * 0.5
    return torch.stack([xc - w_half, yc - h_half, xc + w_half, yc + h_half])


def decode_mask_in_image(mask, box, img_h, img_w, thresh=0.5, padding=1):
    """Paste one (1, M, M) mask probability map into an (img_h, img_w) binary mask (reference
    Utils.decodeMaskInImage: pad by 1, expand the box by the same ratio, bilinear resize, threshold)."""
    m = mask.reshape(mask.shape[-2], mask.shape[-1]).float().cpu()
    M = m.shape[-1]
    padded = F.pad(m, (padding, padding, padding, padding))
    scale = (M + 2 * padding) / M
    b = expand_boxes(box.float().cpu(), scale)
    bx = [int(v) for v in b.tolist()]          # toInt truncates toward zero
    w = max(bx[2] - bx[0] + 1, 1)
    h = max(bx[3] - bx[1] + 1, 1)
    interp = F.interpolate(padded[None, None], size=(h, w), mode="bilinear", align_corners=False)[0, 0]
    interp = (interp > thresh).float() if thresh >= 0 else interp * 255.0
    out = torch.zeros(img_h, img_w)
    x0, x1 = max(bx[0], 0), min(bx[2] + 1, img_w)
    y0, y1 = max(bx[1], 0), min(bx[3] + 1, img_h)
    if x1 > x0 and y1 > y0:
        out[y0:y1, x0:x1] = interp[y0 - bx[1]: y1 - bx[1], x0 - bx[0]: x1 - bx[0]]
    return out


class MaskRCNN(Container):
    """Mask R-CNN (reference MaskRCNN.scala:68). ``inChannels`` is the C2 width (256), ``outChannels`` the FPN
    width (256)."""

    def __init__(self, inChannels, outChannels, numClasses=81, config=None):
        super().__init__()
        c = config or MaskRCNNParams()
        self.inChannels, self.outChannels, self.numClasses, self.config = inChannels, outChannels, numClasses, c
        backbone = nn.Sequential().add(build_resnet50_c2c5(inChannels)).add(
            FPN([inChannels, inChannels * 2, inChannels * 4, inChannels * 8], outChannels, topBlocks=1))
        rpn = RegionProposal(inChannels, c.anchorSizes, c.aspectRatios, c.anchorStride, c.preNmsTopNTest,
                             c.postNmsTopNTest, c.preNmsTopNTrain, c.postNmsTopNTrain, c.rpnNmsThread, c.minSize)
        box = BoxHead(inChannels, c.boxResolution, c.scales, c.samplingRatio, c.boxScoreThresh, c.boxNmsThread,
                      c.maxPerImage, c.outputSize, numClasses)
        mask = MaskHead(inChannels, c.maskResolution, c.scales, c.samplingRatio, c.layers, c.dilation, numClasses,
                        c.useGn)
        self.modules = [backbone, rpn, box, mask]

    def _set_children(self, children):
        self.modules = list(children)

    @property
    def backbone(self):
        return self.modules[0]

    @property
    def rpn(self):
        return self.modules[1]

    @property
    def boxHead(self):
        return self.modules[2]

    @property
    def maskHead(self):
        return self.modules[3]

    def updateOutput(self, input):
        images, info = input[1], input[2]
        size = torch.tensor([float(images.shape[2]), float(images.shape[3])], device=images.device)
        features = self.backbone.forward(images)
        proposals = self.rpn.forward(Table(features, size))
        box_out = self.boxHead.forward(Table(features, proposals, size))
        post = box_out[2]
        labels, boxes, scores = post[1], post[2], post[3]
        masks = self.maskHead.forward(Table(features, boxes, labels))
        if self.train:
            return Table(boxes, labels, masks, scores)
        return self._post_process(boxes, labels, masks[2], scores, info)

    def _post_process(self, bboxes, labels, masks, scores, info):
        out = Table()
        start = 0
        for i in range(bboxes.length()):
            iv = info[i].tolist() if info.dim() == 2 else info.tolist()
            h, w, oh, ow = int(iv[0]), int(iv[1]), int(iv[2]), int(iv[3])
            b = bboxes[i + 1].float().clone()
            n = b.shape[0]
            if (h, w) != (oh, ow):
                D.scale_bbox(b, oh / h, ow / w)
            rles = [binary_to_rle(decode_mask_in_image(masks[start + j], b[j], oh, ow)) for j in range(n)]
            res = Table()
            res[MASKS] = rles
            res[BBOXES] = b
            res[CLASSES] = labels[start: start + n]
            res[SCORES] = scores[start: start + n]
            out[i + 1] = res
            start += n
        return out

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("MaskRCNN model only support inference now")
