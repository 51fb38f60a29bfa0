"""BatchNorm ops (GPU: csrc/batchnorm.hip; CPU: fp32 torch reference).

Reference semantics (S/nn/SpatialBatchNormalization.scala:418-480, S/nn/BatchNormalization.scala:51):
biased batch variance for normalisation, unbiased variance for the running estimate,
``running = momentum * batch + (1 - momentum) * running``.
"""
import os
import torch

from . import native


def _P(x):
    return x.numel() // x.shape[1]


def stat_slots():
    return native.get().STAT_SLOTS


class _StatsArena:
    """One zeroed buffer per training step for every BN statistics / gradient-reduction slot array: a single
    memset replaces ~100 small fills per ResNet-50 step. Slices are handed out in call order, so offsets are the
    same every step (safe inside a captured HIP graph). Outside begin()/end() new_stats falls back to zeros."""

    def __init__(self):
        self.buf, self.off, self.active, self.need = None, 0, False, 0

    def begin(self, device):
        if self.need and (self.buf is None or self.buf.numel() < self.need or self.buf.device != device):
            self.buf = torch.empty(self.need, dtype=torch.float32, device=device)
        if self.buf is not None:
            if self.buf.is_cuda and int(os.environ.get("BIGDL_NATIVE_FILL", "7")) & 2:
                native.get().fill_bytes(self.buf, 0)
            else:
                self.buf.zero_()
        self.off, self.need, self.active = 0, 0, True

    def end(self):
        self.active = False

    def take(self, n, device):
        n_al = (n + 63) // 64 * 64
        self.need += n_al
        if self.active and self.buf is not None and self.buf.device == device and self.off + n_al <= self.buf.numel():
            t = self.buf[self.off:self.off + n]
            self.off += n_al
            return t
        t = torch.empty(n, dtype=torch.float32, device=device)
        if t.is_cuda:
            native.get().fill_bytes(t, 0)
            return t
        return t.zero_()


ARENA = _StatsArena()


def new_stats(C, device):
    """Zeroed [STAT_SLOTS][2][C] fp32 accumulation buffer (see csrc/batchnorm.hip)."""
    return ARENA.take(stat_slots() * 2 * C, torch.device(device))


def _reduce_slots_for_sync(buf, C, P, sync_fn):
    red = torch.empty(2 * C, dtype=torch.float32, device=buf.device)
    native.get().bn_slot_reduce(buf, stat_slots(), C, red)
    P = sync_fn(red, P)
    return red, 1, P


def bn_forward_gpu(x, gamma, beta, rmean, rvar, eps, momentum, training, stats=None, res=None, relu=False,
                   out=None, sync_fn=None, zm=None):
    """Returns (y, save_mean, save_invstd, aff) with aff = [scale | shift] of the apply pass (fp32 [2C]).

    ``zm`` (optional, uint8 [P * C / 8]) receives the sign mask of y (bit e of byte (p, g): y[p][8g + e] > 0), which
    the backward passes read in place of y itself (csrc/batchnorm.hip: 1/16 of the bytes).
    x: (N, C, H, W) bf16 channels_last (or (N, C) bf16 contiguous). ``stats`` may hold the slotted
    (sum, sumsq) already produced by the preceding conv epilogue; otherwise they are computed here.
    ``sync_fn(buf[2C], count) -> total count`` (sync-BN) all-reduces the statistics across replicas.
    """
    C = x.shape[1]
    P = _P(x)
    C_ = native.get()
    dev = x.device
    if out is None:
        out = torch.empty_like(x)
    aff = torch.empty(2 * C, dtype=torch.float32, device=dev)
    scale, shift = aff[:C], aff[C:]
    smean = torch.empty(C, dtype=torch.float32, device=dev)
    sinv = torch.empty(C, dtype=torch.float32, device=dev)
    nslots = stat_slots()
    Ptot = P
    if training:
        if stats is None:
            stats = new_stats(C, dev)
            C_.bn_stats(x, stats, P, C)
        if sync_fn is not None:
            stats, nslots, Ptot = _reduce_slots_for_sync(stats, C, P, sync_fn)
    else:
        stats, nslots = scale, 0  # unused in inference mode
    C_.bn_finalize(stats, nslots, gamma, beta, rmean, rvar, smean, sinv, scale, shift, Ptot, C, float(eps),
                   float(momentum), bool(training))
    C_.bn_apply(x, scale, shift, res, out, P, C, bool(relu), zm)
    return out, smean, sinv, aff


def bn_prepare_gpu(x, gamma, beta, rmean, rvar, eps, momentum, stats=None, sync_fn=None):
    """The statistics / finalize half of a training bn_forward_gpu without the apply pass: returns (save_mean,
    save_invstd, aff). The BN + ReLU output relu(x * aff[:C] + aff[C:]) is then applied on load by its consumer
    (ConvArgs::pre: the streaming 1x1 / halo 3x3 convolutions, the 3x3/2 max pool) or by ``materialize``."""
    C = x.shape[1]
    P = _P(x)
    C_ = native.get()
    dev = x.device
    aff = torch.empty(2 * C, dtype=torch.float32, device=dev)
    smean = torch.empty(C, dtype=torch.float32, device=dev)
    sinv = torch.empty(C, dtype=torch.float32, device=dev)
    nslots, Ptot = stat_slots(), P
    if stats is None:
        stats = new_stats(C, dev)
        C_.bn_stats(x, stats, P, C)
    if sync_fn is not None:
        stats, nslots, Ptot = _reduce_slots_for_sync(stats, C, P, sync_fn)
    C_.bn_finalize(stats, nslots, gamma, beta, rmean, rvar, smean, sinv, aff[:C], aff[C:], Ptot, C, float(eps),
                   float(momentum), True)
    return smean, sinv, aff


def deferred(x, aff):
    """A deferred BN + ReLU output: a new tensor object over x's storage tagged with ``_bn_pre`` = aff. Only a
    consumer that applies it (or ``materialize``) may read it; nn.fusion hands it to such consumers only."""
    y = x.detach()
    y._bn_pre = aff
    return y


def materialize(t):
    """The real values of a deferred BN + ReLU output (bn_apply into a new tensor on the current stream); any
    other tensor is returned as is."""
    aff = getattr(t, "_bn_pre", None)
    if aff is None:
        return t
    C = t.shape[1]
    y = torch.empty_like(t)
    native.get().bn_apply(t, aff[:C], aff[C:], None, y, _P(t), C, True)
    return y


def bn_backward_gpu(dz, z, x, smean, sinv, gamma, dgamma, dbeta, training=True, need_dres=False, need_dx=True,
                    sync_fn=None, aff=None, red=None, zm=None, sec=None):
    """Backward of y = relu?(bn(x) [+ res]).

    dz: gradient w.r.t. the (post-relu) output; z: the forward output (ReLU mask) or None. With z None and
    ``aff`` (the forward's [scale | shift]) the ReLU mask is recomputed from x, so z is never read back.
    Returns (dx, dres) — dres is the gradient flowing into the residual branch (= masked dz).
    ``red``: the slotted backward reduction already accumulated by the producer of dz (a dgrad epilogue).
    ``zm``: the forward's sign mask of the output (bn_forward_gpu), used in place of z.
    ``sec``: (x2, mean2, red2) of a second training BN without ReLU whose output gradient is dres (a projection
    shortcut): its slotted backward reduction is accumulated into red2 by the same pass (requires need_dres).
    """
    C = x.shape[1]
    P = _P(x)
    C_ = native.get()
    nslots, Ptot = 0, P
    if not training:
        red = None
    elif red is None:
        red = new_stats(C, x.device)
        C_.bn_bwd_reduce(dz, z, x, smean, red, P, C, aff, zm)
    if training:
        nslots = stat_slots()
        if sync_fn is not None:
            red, nslots, Ptot = _reduce_slots_for_sync(red, C, P, sync_fn)
    coef = torch.empty(3 * C, dtype=torch.float32, device=x.device)
    dx = torch.empty_like(x) if need_dx else None
    dres = torch.empty_like(x) if need_dres else None
    if sec is not None and dres is not None and training:
        x2, mean2, red2 = sec
        C_.bn_bwd_apply(dz, z, x, smean, sinv, gamma, red, nslots, coef, dx, dres, dgamma, dbeta, Ptot, C, aff, zm,
                        x2=x2, mean2=mean2, red2=red2)
    else:
        C_.bn_bwd_apply(dz, z, x, smean, sinv, gamma, red, nslots, coef, dx, dres, dgamma, dbeta, Ptot, C, aff, zm)
    return dx, dres


# ---------------------------------------------------------------- CPU reference
def bn_forward_cpu(x, gamma, beta, rmean, rvar, eps, momentum, training, sync_fn=None):
    dims = [0] + list(range(2, x.dim()))
    shape = [1, -1] + [1] * (x.dim() - 2)
    if training:
        n = x.numel() // x.shape[1]
        if sync_fn is not None:
            buf = torch.cat([x.sum(dim=dims), (x * x).sum(dim=dims)]).double()
            n = sync_fn(buf, n)
            C = x.shape[1]
            mean = (buf[:C] / n).float()
            var = (buf[C:] / n - (buf[:C] / n) ** 2).clamp_min(0).float()
        else:
            mean = x.mean(dim=dims)
            var = x.var(dim=dims, unbiased=False)
        if rmean is not None:
            unb = var * n / max(n - 1, 1)
            rmean.mul_(1 - momentum).add_(momentum * mean)
            rvar.mul_(1 - momentum).add_(momentum * unb)
    else:
        mean, var = rmean, rvar
    invstd = torch.rsqrt(var + eps)
    xhat = (x - mean.view(shape)) * invstd.view(shape)
    y = xhat
    if gamma is not None:
        y = y * gamma.view(shape) + beta.view(shape)
    return y, mean, invstd


def bn_backward_cpu(x, gy, mean, invstd, gamma, training=True, sync_fn=None):
    dims = [0] + list(range(2, x.dim()))
    shape = [1, -1] + [1] * (x.dim() - 2)
    xhat = (x - mean.view(shape)) * invstd.view(shape)
    g = gamma.view(shape) if gamma is not None else 1.0
    dgamma = (gy * xhat).sum(dim=dims)
    dbeta = gy.sum(dim=dims)
    if training:
        n = x.numel() // x.shape[1]
        sdg, sdb = dgamma, dbeta
        if sync_fn is not None:
            buf = torch.cat([dbeta, dgamma]).double()
            n = sync_fn(buf, n)
            C = x.shape[1]
            sdb, sdg = buf[:C].float(), buf[C:].float()
        gx = g * invstd.view(shape) * (gy - sdb.view(shape) / n - xhat * sdg.view(shape) / n)
    else:
        gx = g * invstd.view(shape) * gy
    return gx, dgamma, dbeta
