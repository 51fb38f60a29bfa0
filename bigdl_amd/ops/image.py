"""Device-side batch augmentation (csrc/image.hip): crop + flip + BGR->RGB + normalise + layout in one kernel."""
import torch

from . import native


def augment_batch_ref(src, params, oh, ow, mean, std, rgb=True, nhwc_bf16=False):
    """fp32 reference of the kernel: src uint8 [N, H, W, 3] BGR, params int [N, 3] = (y0, x0, flip)."""
    outs = []
    for n in range(src.shape[0]):
        y0, x0, flip = [int(v) for v in params[n]]
        img = src[n, y0:y0 + oh, x0:x0 + ow].float()
        if flip:
            img = img.flip(1)
        if rgb:
            img = img.flip(2)
        img = (img - torch.tensor(mean, dtype=torch.float32)) / torch.tensor(std, dtype=torch.float32)
        outs.append(img)
    out = torch.stack(outs)
    return out.to(torch.bfloat16) if nhwc_bf16 else out.permute(0, 3, 1, 2).contiguous()


def augment_batch(src, params, oh, ow, mean, std, rgb=True, nhwc_bf16=False):
    """src: uint8 [N, H, W, 3] on the GPU; returns fp32 [N, 3, oh, ow] or bf16 [N, oh, ow, 3]."""
    if not src.is_cuda:
        return augment_batch_ref(src, params, oh, ow, mean, std, rgb, nhwc_bf16)
    N = src.shape[0]
    if nhwc_bf16:
        out = torch.empty(N, oh, ow, 3, dtype=torch.bfloat16, device=src.device)
    else:
        out = torch.empty(N, 3, oh, ow, dtype=torch.float32, device=src.device)
    p = params.to(torch.int32).contiguous()
    native.get().image_augment(src.contiguous(), p, out, list(map(float, mean)), list(map(float, std)), bool(rgb))
    return out


def random_crop_params(N, H, W, oh, ow, flip=True, generator=None):
    y = torch.randint(0, H - oh + 1, (N,), generator=generator)
    x = torch.randint(0, W - ow + 1, (N,), generator=generator)
    f = torch.randint(0, 2, (N,), generator=generator) if flip else torch.zeros(N, dtype=torch.long)
    return torch.stack([y, x, f], 1).to(torch.int32)


def center_crop_params(N, H, W, oh, ow):
    return torch.tensor([[(H - oh) // 2, (W - ow) // 2, 0]] * N, dtype=torch.int32)
