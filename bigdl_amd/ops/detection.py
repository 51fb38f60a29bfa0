"""Detection primitives: NMS, RoiAlign, RoiPooling (device dispatch) and the bounding-box utilities.

Reference: S/nn/Nms.scala:26-236, S/nn/RoiAlign.scala:45-420, S/nn/RoiPooling.scala:42-366,
S/transform/vision/image/util/BboxUtil.scala:26-581.

On a GPU tensor the HIP kernels in csrc/detection.hip run (IoU bitmask NMS with a single-wave greedy scan,
one-thread-per-output RoiAlign / RoiPooling); on the CPU the same arithmetic runs in numpy / torch. Box
conventions follow the reference: pixel boxes use ``+1`` widths (``(x2 - x1 + 1)``) unless ``normalized``.
"""
import math

import numpy as np
import torch

from . import native


def _on_gpu(t):
    return t.is_cuda


# ------------------------------------------------------------------------------------------------ NMS
def nms_sorted(boxes, thresh, normalized=False, max_keep=-1):
    """Greedy NMS over boxes already sorted by descending score. Returns 0-based kept positions (int64)."""
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    if _on_gpu(boxes):
        b = boxes.float().contiguous()
        keep = torch.empty(n, dtype=torch.int32, device=b.device)
        cnt = torch.empty(1, dtype=torch.int32, device=b.device)
        native.get().nms(b, float(thresh), bool(normalized), int(max_keep), keep, cnt)
        return keep[: int(cnt.item())].long()
    b = boxes.detach().double().cpu().numpy()
    one = 0.0 if normalized else 1.0
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    areas = (x2 - x1 + one) * (y2 - y1 + one)
    w = np.minimum(x2[:, None], x2[None, :]) - np.maximum(x1[:, None], x1[None, :]) + one
    h = np.minimum(y2[:, None], y2[None, :]) - np.maximum(y1[:, None], y1[None, :]) + one
    inter = w * h
    with np.errstate(divide="ignore", invalid="ignore"):
        iou = inter / (areas[:, None] + areas[None, :] - inter)
    sup = (w >= 0) & (h >= 0) & (iou > thresh)
    removed = np.zeros(n, dtype=bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        if 0 < max_keep <= len(keep):
            break
        removed |= sup[i]
    return torch.as_tensor(keep, dtype=torch.long, device=boxes.device)


def nms(scores, boxes, thresh, sorted=False, orderWithBBox=False, normalized=False, max_keep=-1):
    """Reference ``Nms.nms``: returns 0-based indices of kept boxes (score order, or box order with
    ``orderWithBBox``)."""
    scores = scores.reshape(-1)
    if scores.numel() == 0:
        return torch.zeros(0, dtype=torch.long, device=scores.device)
    order = torch.arange(scores.numel(), device=scores.device) if sorted else \
        torch.sort(scores, descending=True, stable=True).indices
    kept = order[nms_sorted(boxes[order], thresh, normalized, max_keep)]
    if orderWithBBox:
        kept = torch.sort(kept).values
    return kept


def nms_fast(scores, boxes, nms_thresh, score_thresh, topk=-1, eta=1.0, normalized=True):
    """Reference ``Nms.nmsFast`` (SSD): score threshold, top-k pre-selection, greedy NMS with an optional
    adaptive threshold (``eta < 1``). Returns 0-based indices in descending-score order."""
    s = scores.reshape(-1)
    cand = torch.nonzero(s >= score_thresh).reshape(-1) if score_thresh > 0 else torch.arange(s.numel(),
                                                                                              device=s.device)
    if cand.numel() == 0:
        return cand
    order = cand[torch.sort(s[cand], descending=True, stable=True).indices]
    if topk > 0:
        order = order[:topk]
    if eta >= 1.0:
        return order[nms_sorted(boxes[order], nms_thresh, normalized)]
    b = boxes[order].double().cpu().numpy()
    one = 0.0 if normalized else 1.0
    areas = (b[:, 2] - b[:, 0] + one) * (b[:, 3] - b[:, 1] + one)
    keep, thr = [], nms_thresh
    for i in range(b.shape[0]):
        ok = True
        for k in keep:
            w = min(b[i, 2], b[k, 2]) - max(b[i, 0], b[k, 0]) + one
            h = min(b[i, 3], b[k, 3]) - max(b[i, 1], b[k, 1]) + one
            if w >= 0 and h >= 0:
                inter = w * h
                if inter / (areas[i] + areas[k] - inter) > thr:
                    ok = False
                    break
        if ok:
            keep.append(i)
            if eta < 1 and thr > 0.5:
                thr *= eta
    return order[torch.as_tensor(keep, dtype=torch.long, device=order.device)]


# ------------------------------------------------------------------------------------------- RoiAlign
def roi_align(x, rois, spatial_scale, sampling_ratio, pooled_h, pooled_w):
    """x: (N, C, H, W); rois: (R, 4) boxes of image 0 (reference) or (R, 5) (batch, x1, y1, x2, y2)."""
    R, C = rois.shape[0], x.shape[1]
    if _on_gpu(x):
        out = torch.empty(R, C, pooled_h, pooled_w, dtype=torch.float32, device=x.device)
        if R:
            native.get().roi_align_fwd(x.float().contiguous(), rois.float().contiguous(), out, float(spatial_scale),
                                       int(sampling_ratio))
        return out
    return _roi_align_cpu(x.float(), rois.float(), spatial_scale, sampling_ratio, pooled_h, pooled_w)


def _roi_align_cpu(x, rois, scale, sampling, PH, PW):
    N, C, H, W = x.shape
    R = rois.shape[0]
    out = torch.zeros(R, C, PH, PW)
    f32 = np.float32
    for r in range(R):
        roi = rois[r].tolist()
        b = int(roi[0]) if len(roi) == 5 else 0
        x1, y1, x2, y2 = [f32(v) * f32(scale) for v in (roi[-4:])]
        rw, rh = max(x2 - x1, f32(1.0)), max(y2 - y1, f32(1.0))
        bh, bw = f32(rh / f32(PH)), f32(rw / f32(PW))
        gh = sampling if sampling > 0 else int(math.ceil(rh / PH))
        gw = sampling if sampling > 0 else int(math.ceil(rw / PW))
        # sampling positions of the whole (PH * gh) x (PW * gw) grid
        iy = np.arange(PH * gh)
        ys = (y1 + (iy // gh).astype(f32) * bh + ((iy % gh).astype(f32) + f32(0.5)) * bh / f32(gh)).astype(f32)
        ix = np.arange(PW * gw)
        xs = (x1 + (ix // gw).astype(f32) * bw + ((ix % gw).astype(f32) + f32(0.5)) * bw / f32(gw)).astype(f32)

        def axis(v, size):
            valid = (v >= -1.0) & (v <= size)
            v = np.maximum(v, 0)
            lo = v.astype(np.int64)
            edge = lo >= size - 1
            lo = np.where(edge, size - 1, lo)
            hi = np.where(edge, lo, lo + 1)
            v = np.where(edge, lo.astype(f32), v)
            l = (v - lo).astype(f32)
            return valid, lo, hi, l

        vy, yl, yh, ly = axis(ys, H)
        vx, xl, xh, lx = axis(xs, W)
        img = x[b]
        wy_l = torch.as_tensor((1 - ly) * vy, dtype=torch.float32)
        wy_h = torch.as_tensor(ly * vy, dtype=torch.float32)
        wx_l = torch.as_tensor((1 - lx) * vx, dtype=torch.float32)
        wx_h = torch.as_tensor(lx * vx, dtype=torch.float32)
        yl_t, yh_t = torch.as_tensor(yl), torch.as_tensor(yh)
        xl_t, xh_t = torch.as_tensor(xl), torch.as_tensor(xh)
        # separable bilinear: rows then columns
        rows = img[:, yl_t, :] * wy_l[None, :, None] + img[:, yh_t, :] * wy_h[None, :, None]   # C, PH*gh, W
        val = rows[:, :, xl_t] * wx_l[None, None, :] + rows[:, :, xh_t] * wx_h[None, None, :]  # C, PH*gh, PW*gw
        out[r] = val.reshape(C, PH, gh, PW, gw).sum(dim=(2, 4)) / float(gh * gw)
    return out


# ----------------------------------------------------------------------------------------- RoiPooling
def _jround(v):
    return int(math.floor(v + 0.5))          # Java Math.round


def roi_pool_forward(x, rois, spatial_scale, PH, PW):
    """Returns (out (R, C, PH, PW), argmax int32 (flat h*W+w within the map, -1 for empty bins))."""
    R, C = rois.shape[0], x.shape[1]
    if _on_gpu(x):
        out = torch.empty(R, C, PH, PW, dtype=torch.float32, device=x.device)
        arg = torch.empty(R, C, PH, PW, dtype=torch.int32, device=x.device)
        if R:
            native.get().roi_pool_fwd(x.float().contiguous(), rois.float().contiguous(), out, arg,
                                      float(spatial_scale))
        return out, arg
    x = x.float()
    H, W = x.shape[2], x.shape[3]
    out = torch.zeros(R, C, PH, PW)
    arg = torch.full((R, C, PH, PW), -1, dtype=torch.int32)
    for r in range(R):
        b, rx1, ry1, rx2, ry2 = rois[r].tolist()
        sw, sh = _jround(np.float32(rx1) * np.float32(spatial_scale)), _jround(np.float32(ry1) * np.float32(spatial_scale))
        ew, eh = _jround(np.float32(rx2) * np.float32(spatial_scale)), _jround(np.float32(ry2) * np.float32(spatial_scale))
        bh = np.float32(max(eh - sh + 1, 1)) / np.float32(PH)
        bw = np.float32(max(ew - sw + 1, 1)) / np.float32(PW)
        fmap = x[int(b)].reshape(C, H * W)
        for ph in range(PH):
            hs = min(max(int(math.floor(ph * bh)) + sh, 0), H)
            he = min(max(int(math.ceil((ph + 1) * bh)) + sh, 0), H)
            for pw in range(PW):
                ws = min(max(int(math.floor(pw * bw)) + sw, 0), W)
                we = min(max(int(math.ceil((pw + 1) * bw)) + sw, 0), W)
                if he <= hs or we <= ws:
                    continue
                idx = (torch.arange(hs, he)[:, None] * W + torch.arange(ws, we)[None, :]).reshape(-1)
                vals = fmap[:, idx]
                m, a = vals.max(dim=1)
                out[r, :, ph, pw] = m
                arg[r, :, ph, pw] = idx[a].int()
    return out, arg


def roi_pool_backward(gy, argmax, rois, x_shape):
    gx = torch.zeros(x_shape, dtype=torch.float32, device=gy.device)
    if _on_gpu(gy):
        native.get().roi_pool_bwd(gy.float().contiguous(), argmax.contiguous(), rois.float().contiguous(), gx)
        return gx
    N, C, H, W = x_shape
    R = gy.shape[0]
    b = rois[:, 0].long()
    flat = gx.reshape(N, C, H * W)
    a = argmax.reshape(R, C, -1).long()
    g = gy.reshape(R, C, -1).float()
    valid = a >= 0
    for r in range(R):
        flat[b[r]].scatter_add_(1, a[r].clamp(min=0), g[r] * valid[r])
    return gx


# ------------------------------------------------------------------------------------------- BboxUtil
def bbox_transform_inv(boxes, deltas, normalized=False):
    """Reference BboxUtil.bboxTransformInv: boxes (N, 4), deltas (N, 4a) -> decoded (N, 4a)."""
    if boxes.shape[0] == 0:
        return boxes.clone()
    one = 0.0 if normalized else 1.0
    w = (boxes[:, 2] - boxes[:, 0] + one)[:, None]
    h = (boxes[:, 3] - boxes[:, 1] + one)[:, None]
    x1, y1 = boxes[:, 0:1], boxes[:, 1:2]
    d = deltas.reshape(deltas.shape[0], -1, 4)
    cx = d[..., 0] * w + x1 + w / 2
    cy = d[..., 1] * h + y1 + h / 2
    pw = torch.exp(d[..., 2]) * w / 2
    ph = torch.exp(d[..., 3]) * h / 2
    return torch.stack([cx - pw, cy - ph, cx + pw, cy + ph], dim=-1).reshape(deltas.shape)


def clip_boxes(boxes, height, width, min_h=0.0, min_w=0.0, scores=None):
    """In-place clip of (N, 4a) pixel boxes to the image; zero the scores of boxes smaller than min_h/min_w.
    Returns the number of boxes that pass the size test (reference BboxUtil.clipBoxes)."""
    b = boxes.view(boxes.shape[0], -1, 4)
    b[..., 0::2].clamp_(0, width - 1)
    b[..., 1::2].clamp_(0, height - 1)
    if scores is None:
        return boxes.shape[0]
    ws = b[..., 2] - b[..., 0] + 1
    hs = b[..., 3] - b[..., 1] + 1
    small = ((ws < min_w) | (hs < min_h)).reshape(-1)
    sc = scores.view(-1)
    sc[small] = 0
    return int((~small).sum())


def clip_normalized(boxes):
    return boxes.clamp_(0, 1)


def scale_bbox(boxes, height, width):
    if boxes.numel():
        boxes[:, 0::2] *= width
        boxes[:, 1::2] *= height
    return boxes


def decode_with_weight(encoded, boxes, weight=(10.0, 10.0, 5.0, 5.0), bbox_clip=62.5):
    """Reference BboxUtil.decodeWithWeight (Detectron-style deltas with weights; w/h clamped from above)."""
    wdt = boxes[:, 2] - boxes[:, 0] + 1
    hgt = boxes[:, 3] - boxes[:, 1] + 1
    cx = boxes[:, 0] + wdt / 2
    cy = boxes[:, 1] + hgt / 2
    d = encoded.reshape(encoded.shape[0], -1, 4)
    dx, dy = d[..., 0] / weight[0], d[..., 1] / weight[1]
    dw = torch.clamp(d[..., 2] / weight[2], max=bbox_clip)
    dh = torch.clamp(d[..., 3] / weight[3], max=bbox_clip)
    pcx = dx * wdt[:, None] + cx[:, None]
    pcy = dy * hgt[:, None] + cy[:, None]
    pw = torch.exp(dw) * wdt[:, None] * 0.5
    ph = torch.exp(dh) * hgt[:, None] * 0.5
    return torch.stack([pcx - pw, pcy - ph, pcx + pw - 1, pcy + ph - 1], dim=-1).reshape(encoded.shape)


def decode_boxes(prior_boxes, prior_variances, clip, bboxes, variance_encoded_in_target=False):
    """SSD decode (reference BboxUtil.decodeBoxes / decodeSingleBbox)."""
    pw = prior_boxes[:, 2] - prior_boxes[:, 0]
    ph = prior_boxes[:, 3] - prior_boxes[:, 1]
    pcx = (prior_boxes[:, 0] + prior_boxes[:, 2]) / 2
    pcy = (prior_boxes[:, 1] + prior_boxes[:, 3]) / 2
    v = torch.ones_like(prior_variances) if variance_encoded_in_target else prior_variances
    cx = v[:, 0] * bboxes[:, 0] * pw + pcx
    cy = v[:, 1] * bboxes[:, 1] * ph + pcy
    w = torch.exp(v[:, 2] * bboxes[:, 2]) * pw
    h = torch.exp(v[:, 3] * bboxes[:, 3]) * ph
    out = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], dim=1)
    return out.clamp_(0, 1) if clip else out


def bbox_areas(boxes, normalized=False):
    one = 0.0 if normalized else 1.0
    return (boxes[:, 2] - boxes[:, 0] + one) * (boxes[:, 3] - boxes[:, 1] + one)


def bbox_vote(scores_nms, bbox_nms, scores_all, bbox_all):
    """Reference BboxUtil.bboxVote: replace each kept box by the score-weighted mean of all boxes that overlap
    it with IoU >= 0.5."""
    a_all = bbox_areas(bbox_all)
    out = bbox_nms.clone()
    for i in range(bbox_nms.shape[0]):
        b = bbox_nms[i]
        iw = torch.minimum(b[2], bbox_all[:, 2]) - torch.maximum(b[0], bbox_all[:, 0]) + 1
        ih = torch.minimum(b[3], bbox_all[:, 3]) - torch.maximum(b[1], bbox_all[:, 1]) + 1
        inter = iw * ih
        ua = (b[2] - b[0] + 1) * (b[3] - b[1] + 1) + a_all - inter
        sel = (iw > 0) & (ih > 0) & (inter / ua >= 0.5)
        w = scores_all.reshape(-1) * sel
        out[i] = (w[:, None] * bbox_all).sum(0) / w.sum()
    return scores_nms, out


def decode_rois(output):
    """Reference BboxUtil.decodeRois: flat detection output [num, (label, score, x1, y1, x2, y2)*] -> (num, 6)."""
    if output.numel() < 6 or output.dim() == 2:
        return output
    num = int(output.reshape(-1)[0].item())
    if num == 0:
        return output.new_zeros(0, 6)
    return output.reshape(-1)[1: 1 + num * 6].view(num, 6)
