"""Device-side image preprocessing for variable-size decoded batches (csrc/image.hip ``image_pipeline_kernel``).

Reference: the per-image host chains of S/transform/vision/image/augmentation (RandomAlterAspect / RandomResize /
Resize -> Crop -> HFlip -> ColorJitter (Brightness, Contrast, Saturation, Hue) -> ChannelNormalize ->
MatToTensor) and S/dataset/image/MTLabeledBGRImgToBatch.scala. Here the host only decodes (BGR uint8, any size)
and draws the random parameters; one kernel launch per batch does the resized crop, flip, colour jitter,
normalisation and the conversion to the training layout (fp32 NCHW or bf16 NHWC) on the GPU.

    pipe = DeviceImagePipeline(224, 224, mean=(123.68, 116.78, 103.94), std=(58.4, 57.1, 57.4))
    params = pipe.random_params([img.shape for img in images])
    batch = pipe(images, params)                      # [N, 3, 224, 224] fp32 on the GPU

Every parameter draw uses the framework RNG (utils/random_generator), so a seeded run is reproducible, and
``host_reference`` recomputes one sample with the host transformers for verification.
"""
import math
from dataclasses import dataclass, field

import torch

from ..ops import native
from ..utils.random_generator import RNG

BRIGHTNESS, CONTRAST, SATURATION, HUE = 1, 2, 3, 4
_NP = 16


@dataclass
class ImageParams:
    """Crop box (in source pixels), horizontal flip and up to 4 colour ops ``(code, amount)`` applied in order."""
    y0: int
    x0: int
    ch: int
    cw: int
    flip: bool = False
    ops: list = field(default_factory=list)


def _noop(code, amount):
    """The host transformers skip these amounts (Brightness / Hue 0, Contrast within 1e-3 of 1)."""
    return (code in (BRIGHTNESS, HUE) and amount == 0) or (code == CONTRAST and abs(amount - 1) <= 1e-3)


class DeviceImagePipeline:
    def __init__(self, out_h, out_w, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0), to_rgb=True, out_format="NCHW",
                 device="cuda"):
        if out_format not in ("NCHW", "NHWC_BF16"):
            raise ValueError("out_format is 'NCHW' (fp32) or 'NHWC_BF16'")
        self.out_h, self.out_w = int(out_h), int(out_w)
        self.mean, self.std = [float(v) for v in mean], [float(v) for v in std]
        self.to_rgb, self.out_format, self.device = bool(to_rgb), out_format, device

    # ------------------------------------------------------------------ parameter draws
    def random_params(self, shapes, area=(0.08, 1.0), aspect=(3.0 / 4.0, 4.0 / 3.0), flip_prob=0.5, jitter=None):
        """Inception-style random-resized crops (RandomAlterAspect: area fraction and aspect ratio, falling back to
        a centred square crop after 10 tries), random flips and optional ColorJitter draws. ``jitter`` is a dict of
        ColorJitter arguments (brightnessProb, brightnessDelta, contrastProb, contrastLower, contrastUpper,
        saturationProb, saturationLower, saturationUpper, hueProb, hueDelta) or None."""
        out = []
        for shp in shapes:
            H, W = int(shp[0]), int(shp[1])
            box = None
            for _ in range(10):
                target = RNG.uniform(area[0], area[1]) * H * W
                ratio = math.exp(RNG.uniform(math.log(aspect[0]), math.log(aspect[1])))
                cw = int(round(math.sqrt(target * ratio)))
                ch = int(round(math.sqrt(target / ratio)))
                if 0 < cw <= W and 0 < ch <= H:
                    y0 = int(RNG.uniform(0, H - ch + 1e-9)) if H > ch else 0
                    x0 = int(RNG.uniform(0, W - cw + 1e-9)) if W > cw else 0
                    box = (min(y0, H - ch), min(x0, W - cw), ch, cw)
                    break
            if box is None:
                s = min(H, W)
                box = ((H - s) // 2, (W - s) // 2, s, s)
            flip = RNG.uniform(0, 1) < flip_prob
            out.append(ImageParams(*box, flip=flip, ops=self._jitter_ops(jitter)))
        return out

    @staticmethod
    def _jitter_ops(j):
        if not j:
            return []
        ops = []
        # ColorJitter.scala order1 (brightness, contrast, saturation, hue) or order2 (brightness, saturation, hue,
        # contrast), chosen with probability 1/2
        order1 = RNG.uniform(0, 1) > 0.5
        b = (BRIGHTNESS, RNG.uniform(-j.get("brightnessDelta", 32), j.get("brightnessDelta", 32))) \
            if RNG.uniform(0, 1) < j.get("brightnessProb", 0.5) else None
        c = (CONTRAST, RNG.uniform(j.get("contrastLower", 0.5), j.get("contrastUpper", 1.5))) \
            if RNG.uniform(0, 1) < j.get("contrastProb", 0.5) else None
        s = (SATURATION, RNG.uniform(j.get("saturationLower", 0.5), j.get("saturationUpper", 1.5))) \
            if RNG.uniform(0, 1) < j.get("saturationProb", 0.5) else None
        h = (HUE, RNG.uniform(-j.get("hueDelta", 18), j.get("hueDelta", 18))) \
            if RNG.uniform(0, 1) < j.get("hueProb", 0.5) else None
        seq = [b, c, s, h] if order1 else [b, s, h, c]
        for op in seq:
            if op is not None:
                ops.append(op)
        return ops

    # ------------------------------------------------------------------ launch
    def __call__(self, images, params):
        imgs = [torch.as_tensor(im) for im in images]
        if len(imgs) != len(params):
            raise ValueError("one ImageParams per image")
        for im in imgs:
            if im.dtype != torch.uint8 or im.dim() != 3 or im.shape[2] != 3:
                raise ValueError("images must be uint8 H x W x 3 (BGR)")
        N = len(imgs)
        sizes = [im.numel() for im in imgs]
        offs = torch.zeros(N, dtype=torch.int64)
        if N > 1:
            offs[1:] = torch.cumsum(torch.tensor(sizes[:-1], dtype=torch.int64), 0)
        flat = torch.empty(sum(sizes), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        for im, o, n in zip(imgs, offs.tolist(), sizes):
            flat[o:o + n].copy_(im.contiguous().reshape(-1))
        prm = torch.zeros(N, _NP, dtype=torch.float32)
        for i, (im, p) in enumerate(zip(imgs, params)):
            if len(p.ops) > 4:
                raise ValueError("at most 4 colour ops per image")
            ops = [(c, a) for c, a in p.ops if not _noop(c, a)]
            row = [im.shape[0], im.shape[1], p.y0, p.x0, p.ch, p.cw, 1.0 if p.flip else 0.0, len(ops)]
            for code, amount in ops:
                row += [code, amount]
            prm[i, :len(row)] = torch.tensor(row, dtype=torch.float32)
        dev = torch.device(self.device)
        src = flat.to(dev, non_blocking=True)
        if self.out_format == "NCHW":
            out = torch.empty(N, 3, self.out_h, self.out_w, dtype=torch.float32, device=dev)
        else:
            out = torch.empty(N, self.out_h, self.out_w, 3, dtype=torch.bfloat16, device=dev)
        native.get().image_pipeline(src, offs.to(dev), prm.to(dev), out, self.mean, self.std, self.to_rgb)
        return out

    # ------------------------------------------------------------------ verification
    def host_reference(self, image, p):
        """The same sample through the host transformers (Crop -> Resize -> HFlip -> colour ops ->
        ChannelNormalize -> RGB), fp32, in the layout of the device output (without batch dim, fp32)."""
        from ..transform.vision.image.augmentation import Brightness, Contrast, Hue, Saturation, _resize

        m = torch.as_tensor(image).float()[p.y0:p.y0 + p.ch, p.x0:p.x0 + p.cw]
        m = _resize(m, self.out_w, self.out_h)
        if p.flip:
            m = m.flip(1)
        fns = {BRIGHTNESS: Brightness.transform_mat, CONTRAST: Contrast.transform_mat,
               SATURATION: Saturation.transform_mat, HUE: Hue.transform_mat}
        for code, amount in p.ops:
            m = fns[code](m, amount)
        if self.to_rgb:
            m = m[..., [2, 1, 0]]
        m = (m - torch.tensor(self.mean)) / torch.tensor(self.std)
        return m.permute(2, 0, 1).contiguous() if self.out_format == "NCHW" else m


__all__ = ["DeviceImagePipeline", "ImageParams", "BRIGHTNESS", "CONTRAST", "SATURATION", "HUE"]
