"""Convolution / linear ops.

GPU path: bf16 NHWC (torch ``channels_last``) activations and KRSC (channels_last) weights, dispatched to
the implicit-GEMM MFMA kernels of ``csrc/conv_igemm.hip``. CPU path: fp32 torch reference (the analogue of
the reference's MklBlas engine, used for the LeNet local-CPU configuration and as the numerics oracle).

Reference: S/nn/SpatialConvolution.scala:253-520 (fwd / bwd-data / bwd-weight), S/nn/Linear.scala:84-160.
"""
import os
import torch
import torch.nn.functional as F

from . import native

CL = torch.channels_last
BF16 = torch.bfloat16


def out_size(inp, k, s, p, d=1, ceil=False):
    eff = d * (k - 1) + 1
    num = inp + 2 * p - eff
    if ceil:
        o = -(-num // s) + 1
        if (o - 1) * s >= inp + p:
            o -= 1
        return o
    return num // s + 1


def to_nhwc_bf16(x, cpad=8):
    """Convert an activation to the GPU compute layout (bf16 channels_last, C padded to a multiple of 8)."""
    N, C, H, W = x.shape
    Cp = -(-C // cpad) * cpad
    if x.dtype == BF16 and Cp == C and x.is_contiguous(memory_format=CL):
        return x
    if x.dtype == torch.float32 and x.is_contiguous():
        y = torch.empty((N, Cp, H, W), dtype=BF16, device=x.device, memory_format=CL)
        native.get().nchw_to_nhwc(x, y, Cp)
        return y
    y = x.to(dtype=BF16, memory_format=CL)
    if Cp != C:
        y = F.pad(y, (0, 0, 0, 0, 0, Cp - C)).contiguous(memory_format=CL)
    return y


def weight_krsc_bf16(w, cpad=8):
    """(K, C, R, S) weight -> bf16 channels_last with C padded to a multiple of ``cpad``."""
    K, C, R, S = w.shape
    Cp = -(-C // cpad) * cpad
    if w.dtype == BF16 and Cp == C and w.is_contiguous(memory_format=CL):
        return w
    if Cp != C:
        w = F.pad(w, (0, 0, 0, 0, 0, Cp - C))
    return w.to(dtype=BF16, memory_format=CL)


def pad_dim(t, dim, mult=8):
    """Zero-pad dimension ``dim`` of a 4-D bf16 tensor to a multiple of ``mult`` (keeps channels_last)."""
    n = t.shape[dim]
    npad = -(-n // mult) * mult
    if npad == n:
        return t
    shape = list(t.shape)
    shape[dim] = npad
    out = torch.zeros(shape, dtype=t.dtype, device=t.device).contiguous(memory_format=CL)
    out.narrow(dim, 0, n).copy_(t)
    return out


def conv2d_fwd(x, w16, bias, stride, pad, dil=(1, 1), relu=False, stats=None, out=None, addend=None, pre=None):
    """y = conv(x, w) + bias [+ addend] (+ReLU); optionally accumulate per-channel (sum, sumsq) of y into ``stats``.

    ``pre`` ([2C] fp32 scale | shift): x is a deferred BatchNorm + ReLU output (ops/bn.py deferred): the kernel reads
    relu(x * scale + shift). Then returns (y, x_mat) with x_mat the materialised input when no kernel applied it on
    load (csrc/bindings.cpp conv_nt), else None.

    x: (N, C, H, W) bf16 channels_last (C % 8 == 0); w16: (K, C, R, S) bf16 channels_last.
    ``out`` may be a channel slice ``buf[:, c0:c0 + K]`` of a channels_last (N, Ctot, OH, OW) buffer (a concat
    written in place: row stride Ctot); ``addend`` (same shape as y, channels_last) is summed in the epilogue
    before the ReLU (a residual add).
    """
    N, C, H, W = x.shape
    K, Cw, R, S = w16.shape
    assert Cw == C, f"conv2d_fwd: channel mismatch {Cw} vs {C}"
    sh, sw = stride
    ph, pw = pad
    dh, dw = dil
    OH, OW = out_size(H, R, sh, ph, dh), out_size(W, S, sw, pw, dw)
    ldo = K
    if out is None:
        out = torch.empty((N, K, OH, OW), dtype=BF16, device=x.device, memory_format=CL)
    else:
        assert tuple(out.shape) == (N, K, OH, OW) and out.stride(1) == 1, "conv2d_fwd: out must be NHWC (N, K, OH, OW)"
        ldo = out.stride(3) if OW > 1 else out.stride(2) // max(OW, 1)
    if addend is not None:
        assert ldo == K and addend.shape == out.shape and addend.is_contiguous(memory_format=CL), \
            "conv2d_fwd: a residual addend needs a dense NHWC output"
    geo = _fwd_geo(N, H, W, C, OH, OW, sh, sw, R * S * C, K)
    geo[10] = ldo
    if stats is not None and native.deterministic():
        # deterministic mode: statistics in a separate one-writer-per-slot reduction, not the GEMM epilogue
        mat = native.get().conv_nt(x, w16, out, bias, None, geo, _fwd_taps(R, S, ph, pw, dh, dw), relu, addend,
                                   pre=pre)
        dense = out if ldo == K else out.contiguous(memory_format=CL)
        native.get().bn_stats(dense, stats, N * OH * OW, K)
        return (out, mat) if pre is not None else out
    mat = native.get().conv_nt(x, w16, out, bias, stats, geo, _fwd_taps(R, S, ph, pw, dh, dw), relu, addend, pre=pre)
    return (out, mat) if pre is not None else out


_TAP_CACHE = {}


def _fwd_taps(R, S, ph, pw, dh, dw):
    key = ("f", R, S, ph, pw, dh, dw)
    t = _TAP_CACHE.get(key)
    if t is None:
        t = []
        for r in range(R):
            for s in range(S):
                t += [r * dh - ph, s * dw - pw, r * S + s]
        _TAP_CACHE[key] = t
    return t


def _fwd_geo(N, H, W, C, OH, OW, sh, sw, ldw, K):
    return [N, H, W, C, OH, OW, sh, sw, ldw, K, K, OH, OW, 1, 1, 0, 0]


def dgrad_phases(H, W, R, S, stride, pad, dil):
    """Decompose the data gradient of a stride-(sh, sw) conv into sh*sw dense phase GEMMs.

    Output pixel h = a + sh*i receives tap r iff (a + ph - r*dh) % sh == 0, from dY row
    i + (a + ph - r*dh) / sh. Returns [(a, b, nI, nJ, taps)] (taps as flat [th, tw, tap_index] triples);
    phases without taps are omitted (their pixels get zero gradient).
    """
    sh, sw = stride
    ph, pw = pad
    dh, dw = dil
    key = ("d", H, W, R, S, sh, sw, ph, pw, dh, dw)
    res = _TAP_CACHE.get(key)
    if res is not None:
        return res
    res = []
    for a in range(sh):
        for b in range(sw):
            nI, nJ = -(-(H - a) // sh), -(-(W - b) // sw)
            if nI <= 0 or nJ <= 0:
                continue
            taps = []
            for r in range(R):
                if (a + ph - r * dh) % sh:
                    continue
                for s in range(S):
                    if (b + pw - s * dw) % sw:
                        continue
                    taps += [(a + ph - r * dh) // sh, (b + pw - s * dw) // sw, r * S + s]
            if taps:
                res.append((a, b, nI, nJ, taps))
    _TAP_CACHE[key] = res
    return res


def conv2d_dgrad(dy, w16t, x_shape, stride, pad, dil=(1, 1), out=None, addend=None, bn=None, addend_zm=None):
    """dx = conv_transpose(dy, w) [+ addend]. ``w16t`` is the (C, R, S, K)-ordered transposed weight.

    Stride > 1 runs one dense implicit GEMM per stride phase (no zero-insertion, no masked MFMAs).
    ``addend`` (same shape/layout as dx) is summed in the GEMM epilogue — used to fold the residual
    branch gradient of a ResNet block into the block-input gradient.

    ``bn`` = {"x", "z", "mean", "aff", "red"[, "zm"]}: dx is the gradient of a training BatchNorm's (ReLU-fused)
    output (ReLU mask from z, or its sign mask zm, or x * aff), and the epilogue also accumulates that BN's backward reduction into ``red`` (the pass
    bn_bwd_reduce would make over dx and x). ``addend_zm`` (uint8 sign mask, [P][C / 8]): the addend is added only
    where its bit is set (every pixel must be covered by a GEMM phase). Only when every pixel of dx is written by a GEMM phase (or the
    uncovered pixels are zero); ``bn["done"]`` reports whether it ran.
    """
    N, C, H, W = x_shape
    _, K, OH, OW = dy.shape
    R, S = w16t.shape[1], w16t.shape[2]
    phases = dgrad_phases(H, W, R, S, stride, pad, dil)
    covered = sum(nI * nJ for (_, _, nI, nJ, _) in phases)
    if addend is not None and not addend.is_contiguous(memory_format=CL):
        addend = addend.contiguous(memory_format=CL)
    if out is None:
        out = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
    if addend_zm is not None and (addend is None or covered != H * W):
        raise ValueError("conv2d_dgrad: a masked addend needs an addend and a data gradient that covers every pixel")
    if covered != H * W:
        # pixels no phase reaches: zeros, or the folded residual addend (the phase GEMMs add it to theirs)
        mask = 0
        for (a, b, _, _, _) in phases:
            mask |= 1 << (a * stride[1] + b)
        if (out.is_contiguous(memory_format=CL) and C % 8 == 0 and stride[0] * stride[1] <= 32
                and int(os.environ.get("BIGDL_NATIVE_FILL", "7")) & 4):
            native.get().dgrad_fill(out, addend, stride[0], stride[1], mask)
        elif addend is not None:
            out.copy_(addend)
        else:
            out.zero_()
    C_ = native.get()
    ldw = R * S * K
    bnk = {}
    if bn is not None and (covered == H * W or addend is None) and bn["x"].shape == out.shape \
            and bn["x"].stride() == out.stride() and not native.deterministic():
        bnk = dict(bn_x=bn["x"], bn_z=bn["z"], bn_mean=bn["mean"], bn_aff=bn["aff"], bn_red=bn["red"],
                   bn_zm=bn.get("zm"))
        bn["done"] = True
    for (a, b, nI, nJ, taps) in phases:
        geo = [N, OH, OW, K, nI, nJ, 1, 1, ldw, C, C, H, W, stride[0], stride[1], a, b]
        C_.conv_nt(dy, w16t, out, None, None, geo, taps, False, addend, addend_zm=addend_zm, **bnk)
    return out


# Batched weight transposes for the data-gradient GEMMs: TrainStep transposes every eligible conv's bf16 weight in
# one launch right before backward and stamps the modules; a conv whose stamp matches WT_STAMP reuses that buffer.
WT_STAMP = [0]
_DESC_CACHE = {}
DESC_BUILDS = [0]            # descriptor tables built (one per distinct set of weight / buffer addresses)


def prepare_dgrad_weights(convs):
    """Transpose the (K, C, R, S) bf16 weights of ``convs`` (modules with ``_w16_padded``) into their
    ``_wt_cache`` (C, R, S, K) buffers with one kernel launch (csrc/conv_igemm.hip transpose_krsc_batched_kernel).
    Only layers whose bf16 weight is the persistent managed view (C % 8 == 0, K % 8 == 0) take part, so the
    descriptor table is built once (before any HIP-graph capture) and reused."""
    WT_STAMP[0] += 1
    rows, mods, tile = [], [], 0
    for m in convs:
        if not getattr(m, "_w16_managed", False):      # per-call bf16 casts have no stable address
            continue
        wf = getattr(m, "weight", None)
        if wf is None or wf.dim() != 4 or wf.shape[0] % 8 or wf.shape[1] % 8:
            continue                                    # channel-padded weights are rebuilt per call
        w16 = m._w16_padded()
        K, C, R, S = w16.shape
        if K % 8 or C % 8 or not w16.is_cuda or not w16.is_contiguous(memory_format=CL):
            continue
        if mods and w16.device != mods[0]._wt_cache.device:     # one descriptor table per device
            continue
        wt = getattr(m, "_wt_cache", None)
        if wt is None or tuple(wt.shape) != (C, R, S, K) or wt.device != w16.device:
            wt = torch.empty((C, R, S, K), dtype=BF16, device=w16.device)
            m._wt_cache = wt
        rows.append((w16.data_ptr(), wt.data_ptr(), K, R * S, C, tile))
        tile += ((C + 31) // 32) * ((K + 31) // 32) * R * S
        mods.append(m)
    if not rows:
        return 0
    key = tuple(rows)
    desc = _DESC_CACHE.get(key)
    if desc is None:
        if torch.cuda.is_current_stream_capturing():
            return 0                 # no host->device copy inside a graph capture: per-layer transposes instead
        if len(_DESC_CACHE) > 8:
            _DESC_CACHE.clear()
        desc = torch.tensor(rows, dtype=torch.int64).to(mods[0]._wt_cache.device)
        _DESC_CACHE[key] = desc
        DESC_BUILDS[0] += 1
    native.get().transpose_krsc_batched(desc, len(rows), tile)
    for m in mods:
        m._wt_stamp = WT_STAMP[0]
    return len(rows)


def end_dgrad_weights():
    """Invalidate the batched transposes (the optimizer is about to change the weights)."""
    WT_STAMP[0] += 1


def transpose_w(w16, out=None):
    """(K, C, R, S) channels_last bf16 -> contiguous (C, R, S, K) bf16 for the data-gradient GEMM."""
    K, C, R, S = w16.shape
    if out is None:
        out = torch.empty((C, R, S, K), dtype=BF16, device=w16.device)
    native.get().transpose_krsc(w16, out, K, R * S, C)
    return out


def _gemm_shaped(dy, x, dw32, stride, pad, dil):
    """A 1x1 / stride-1 / unpadded weight gradient is a plain GEMM dW[K][C] = sum_p dy[p][K] x[p][C]."""
    K, C = dy.shape[1], x.shape[1]
    return (dw32.shape[2] == 1 and dw32.shape[3] == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0)
            and dy.shape[2:] == x.shape[2:] and dw32.is_contiguous() and C % 8 == 0 and K % 8 == 0
            and dy.is_contiguous(memory_format=CL) and x.is_contiguous(memory_format=CL))


def _rows_T64(t2d):
    """(P, C) bf16 rows -> (C, P64) bf16, P zero-padded to a multiple of 64 (the LDS-DMA GEMM's K step)."""
    P, C = t2d.shape
    P64 = -(-P // 64) * 64
    if P64 != P:
        pad = torch.zeros((P64, C), dtype=BF16, device=t2d.device)
        pad[:P].copy_(t2d)
        t2d = pad
    out = torch.empty((C, P64), dtype=BF16, device=t2d.device)
    native.get().transpose_krsc(t2d, out, P64, 1, C)
    return out


def gemm_wgrad_nt(dy2d, x2d, dw32, dbias32=None):
    """dW (fp32 [K][C]) += dy^T x over P rows on the NT MFMA GEMM kernel: both operands are transposed once (LDS
    tiles) so the reduction runs along contiguous rows, and the epilogue accumulates fp32 straight into dW. For
    large outputs this is ~2-5x the split-K weight-gradient kernel (which exists for small outputs / deep
    reductions, where it fills the chip by splitting P)."""
    P, K = dy2d.shape
    C = x2d.shape[1]
    dyT, xT = _rows_T64(dy2d), _rows_T64(x2d)
    P64 = dyT.shape[1]
    geo = [K, 1, 1, P64, 1, 1, 1, 1, P64, C, C, 1, 1, 1, 1, 0, 0]
    native.get().conv_nt(dyT, xT, dw32.view(K, C), None, None, geo, [0, 0, 0], False, accumulate=True)
    if dbias32 is not None:
        native.get().colsum_bf16(dy2d, dbias32)


# ------------------------------------------------------------------------------------------------
# Pixel-pair packing for <= 4-channel convolutions with width stride 2 (image stems; csrc/stem.hip): the zero-padded
# image is stored NHWC4 and viewed as [N][Hp][Wp/2][8] pixel pairs, so one 16-byte granule carries two width taps.
# ------------------------------------------------------------------------------------------------
def pair_ok(C, stride, dil, groups):
    import os

    return (groups == 1 and C <= 4 and stride[1] == 2 and tuple(dil) == (1, 1)
            and os.environ.get("BIGDL_CONV_PAIR", "1") != "0")


def pair_geometry(H, W, R, S, sh, ph, pw):
    """(OH, OW, S2, Hp, Wp) of the pair view: padded image rows / columns (Wp even) covering every tap."""
    OH, OW = out_size(H, R, sh, ph), out_size(W, S, 2, pw)
    S2 = (S + 1) // 2
    Hp = max(H + 2 * ph, (OH - 1) * sh + R)
    Wp = max(2 * (OW - 1 + S2), W + 2 * pw)
    return OH, OW, S2, Hp, Wp + (Wp & 1)


def to_pairs_bf16(x, R, S, sh, ph, pw):
    N, C, H, W = x.shape
    _, _, _, Hp, Wp = pair_geometry(H, W, R, S, sh, ph, pw)
    y = torch.empty((N, Hp, Wp // 2, 8), dtype=BF16, device=x.device)
    xf = x if (x.dtype == torch.float32 and x.is_contiguous()) else x.float().contiguous()
    native.get().nchw_to_pairs(xf, y, ph, pw)
    return y


def pair_weight(w16):
    """(K, C, R, S) bf16 weight -> (K, R * S2 * 8) pair-packed weight (csrc/stem.hip)."""
    K, C, R, S = w16.shape
    wp = torch.empty((K, R * ((S + 1) // 2) * 8), dtype=BF16, device=w16.device)
    native.get().pair_weight(w16, wp)
    return wp


def _pair_taps(R, S2):
    key = ("p", R, S2)
    t = _TAP_CACHE.get(key)
    if t is None:
        t = []
        for r in range(R):
            for j in range(S2):
                t += [r, j, r * S2 + j]
        _TAP_CACHE[key] = t
    return t


def _window_taps(R):
    key = ("w", R)
    t = _TAP_CACHE.get(key)
    if t is None:
        t = [v for r in range(R) for v in (r, 0, r)]
        _TAP_CACHE[key] = t
    return t


def conv2d_pairs_fwd(xp, wp, bias, K, OH, OW, R, S2, sh, relu=False, stats=None):
    N, Hp, Wq, _ = xp.shape
    out = torch.empty((N, K, OH, OW), dtype=BF16, device=xp.device, memory_format=CL)
    if S2 == 4 and os.environ.get("BIGDL_STEM_WINDOW", "0") != "0":
        # width im2col in place: output column ow reads pairs ow .. ow + 3 = all 7 (8) width taps as ONE 32-element
        # "pixel" of an overlapping-window view (pixel stride 8 elements), so the stem is an R x 1 convolution with a
        # 32-channel fast-K reduction per row tap (csrc/kernels.h ConvArgs::pstride) instead of R x 4 pair taps of 8.
        # Opt-in (BIGDL_STEM_WINDOW=1): bitwise the same result and no faster at batch 256 (369 vs 353 us,
        # profiles/r5_stem_window.txt) — the stem forward is bound by its 411 MB output + statistics epilogue, not
        # by the gather
        geo = [N, Hp, Wq, 32, OH, OW, sh, 1, R * 32, K, K, OH, OW, 1, 1, 0, 0, 8]
        det = stats is not None and native.deterministic()
        native.get().conv_nt(xp, wp, out, bias, None if det else stats, geo, _window_taps(R), relu, None)
        if det:
            native.get().bn_stats(out, stats, N * OH * OW, K)
        return out
    geo = [N, Hp, Wq, 8, OH, OW, sh, 1, R * S2 * 8, K, K, OH, OW, 1, 1, 0, 0]
    if stats is not None and native.deterministic():
        # deterministic mode: the stem kernels commit statistics with float atomics from thousands of workgroups;
        # take them from the one-writer-per-slot reduction instead (as conv2d_fwd does)
        native.get().conv_nt(xp, wp, out, bias, None, geo, _pair_taps(R, S2), relu, None)
        native.get().bn_stats(out, stats, N * OH * OW, K)
        return out
    native.get().conv_nt(xp, wp, out, bias, stats, geo, _pair_taps(R, S2), relu, None)
    return out


def conv2d_pairs_wgrad(dy, xp, R, S2, sh, dwp32, dbias32):
    """dW' (fp32 (K, R * S2 * 8)) += weight gradient of the pair view; dbias += sum(dy)."""
    N, Hp, Wq, _ = xp.shape
    _, K, OH, OW = dy.shape
    geo = [N, Hp, Wq, 8, OH, OW, R, S2, sh, 1, 0, 0, 1, 1, N * OH * OW, K, R * S2 * 8, K]
    native.get().conv_wgrad(dy, xp, dwp32, dbias32, geo)


def conv2d_wgrad(dy, x, dw32, dbias32, stride, pad, dil=(1, 1), pre=None):
    """dW (fp32, (K, C, R, S) channels_last buffer) += conv weight gradient; dbias += sum(dy).

    ``pre`` ([2C] scale | shift): x is a deferred BatchNorm + ReLU output (ops/bn.py deferred): the halo 3x3 weight
    gradient applies it on load; any other kernel gets the materialised input (csrc/bindings.cpp conv_wgrad)."""
    N, C, H, W = x.shape
    _, K, OH, OW = dy.shape
    Kw, Cw, R, S = dw32.shape
    assert Kw == K and Cw == C
    P = N * OH * OW
    sh, sw = stride
    ph, pw = pad
    dh, dw = dil
    geo = [N, H, W, C, OH, OW, R, S, sh, sw, ph, pw, dh, dw, N * OH * OW, K, R * S * C, K]
    if pre is not None and _gemm_shaped(dy, x, dw32, stride, pad, dil):
        from . import bn as bnops

        x, pre = bnops.materialize(bnops.deferred(x, pre)), None
    if (P >= 512 and ((K + 127) // 128) * ((C + 127) // 128) >= 192 and _gemm_shaped(dy, x, dw32, stride, pad, dil)
            and not native.get().conv_wgrad_uses_p8(geo, dbias32 is not None)):
        gemm_wgrad_nt(dy.reshape(P, K) if dy.is_contiguous() else dy.permute(0, 2, 3, 1).reshape(P, K),
                      x.reshape(P, C) if x.is_contiguous() else x.permute(0, 2, 3, 1).reshape(P, C), dw32, dbias32)
        return
    native.get().conv_wgrad(dy, x, dw32, dbias32, geo, pre)


# ------------------------------------------------------------------------------------------------
# CPU reference path (fp32, NCHW): used by the local CPU engine and as the numerics oracle in tests.
# ------------------------------------------------------------------------------------------------
def conv2d_cpu(x, w, b, stride, pad, dil=(1, 1), groups=1):
    return F.conv2d(x, w, b, stride=stride, padding=pad, dilation=dil, groups=groups)


def conv2d_grads_cpu(x, w, gy, stride, pad, dil=(1, 1), groups=1, need_input=True):
    gi = None
    if need_input:
        gi = torch.nn.grad.conv2d_input(x.shape, w, gy, stride=stride, padding=pad, dilation=dil, groups=groups)
    gw = torch.nn.grad.conv2d_weight(x, w.shape, gy, stride=stride, padding=pad, dilation=dil, groups=groups)
    gb = gy.sum(dim=(0, 2, 3))
    return gi, gw, gb
