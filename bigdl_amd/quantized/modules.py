"""Int8 inference modules: quantized Linear / SpatialConvolution / SpatialDilatedConvolution.

Reference: S/nn/quantized/Linear.scala:29-181, SpatialConvolution.scala:33-325,
SpatialDilatedConvolution.scala:27-109, Quantization.scala:27-180 (symmetric max-abs scaling), Desc.scala:179-181.

Numerics (same scheme as the reference's BigQuant path):
  * weights are quantized once, symmetric per output channel: ``q_w = round(w * 127 / max|w_row|)``;
  * activations are quantized per call, symmetric per sample (per sample and group for grouped convs):
    ``q_x = round(x * 127 / max|x_n|)``;
  * the int8 x int8 products accumulate exactly in int32 and are dequantized in the epilogue:
    ``y = acc * (amax_x / 127) * (amax_w / 127) + bias``.

MI355X engine (csrc/quant.hip): the activation is quantized straight from the bf16/fp32 channels-last
tensor into an int8 NHWC buffer (channels padded to 16, one 16-byte granule per MFMA lane), and the
convolution runs as an implicit GEMM on ``v_mfma_i32_16x16x64_i8`` — 4x the K depth per instruction of the
bf16 kernels and half the operand bytes — with the dequantize / bias / ReLU epilogue fused. Linear layers
are the 1x1, H = W = 1 case of the same kernel. On the CPU the identical integer arithmetic is emulated in
float64 (exact for the int32 accumulator range), so CPU and GPU agree to fp32 rounding.

Quantized modules are inference-only (the reference throws on updateGradInput as well).
"""
import math

import torch
import torch.nn.functional as F

from ..nn.abstractnn import TensorModule
from ..ops import native

CL = torch.channels_last
BF16 = torch.bfloat16
QMAX = 127.0


def _ceil(a, m):
    return -(-a // m) * m


def quantize_rows(w2d):
    """Symmetric per-row int8 quantization. Returns (q int8 [rows, cols], scale fp32 [rows])."""
    w2d = w2d.float()
    amax = w2d.abs().amax(dim=1)
    inv = torch.where(amax > 0, QMAX / amax, torch.zeros_like(amax))
    q = torch.round(w2d * inv[:, None]).clamp_(-QMAX, QMAX).to(torch.int8)
    return q, amax / QMAX


def quantize_per_sample_ref(x):
    """CPU reference of the activation quantizer (per leading index): returns (q int8, scale fp32 [N])."""
    xf = x.float()
    amax = xf.reshape(xf.shape[0], -1).abs().amax(dim=1)
    inv = torch.where(amax > 0, QMAX / amax, torch.zeros_like(amax))
    shape = (-1,) + (1,) * (xf.dim() - 1)
    q = torch.round(xf * inv.reshape(shape)).clamp_(-QMAX, QMAX).to(torch.int8)
    return q, amax / QMAX


def quantize_act_gpu(x_nhwc, C, Cp, static_amax=None):
    """x_nhwc: contiguous [N, ..., C] bf16/fp32 device tensor -> (q int8 [N, P, Cp], scale fp32 [N]).
    ``static_amax`` (a calibrated range, MklInt8Convertible-style) replaces the per-sample abs-max pass."""
    N = x_nhwc.shape[0]
    P = x_nhwc.numel() // (N * C)
    q = torch.empty((N, P, Cp), dtype=torch.int8, device=x_nhwc.device)
    scale = torch.empty(N, dtype=torch.float32, device=x_nhwc.device)
    if static_amax is not None:
        amax = torch.full((N,), float(static_amax), dtype=torch.float32, device=x_nhwc.device)
        native.get().quantize_act(x_nhwc, q, amax, scale, N, P, C, Cp, True)
    else:
        amax = torch.empty(N, dtype=torch.float32, device=x_nhwc.device)
        native.get().quantize_act(x_nhwc, q, amax, scale, N, P, C, Cp, False)
    return q, scale


class QuantizedModule(TensorModule):
    """Base of the int8 modules (reference QuantizedModule.scala): inference only, no gradient state."""

    def __init__(self, length):
        super().__init__()
        self.length = length
        self.train = False

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("quantized modules are inference-only (no updateGradInput)")

    def accGradParameters(self, input, gradOutput):
        raise NotImplementedError("quantized modules are inference-only")

    def training(self):
        return self            # stays in evaluation mode

    def parameters(self):
        ws = [getattr(self, b) for b in self._buffers if getattr(self, b, None) is not None]
        return ws, [torch.empty(0) for _ in ws]

    def release(self):
        return self


class QuantizedLinear(QuantizedModule):
    """int8 fully-connected layer (reference quantized/Linear.scala:29)."""

    def __init__(self, inputSize, outputSize, withBias=True, initWeight=None, initBias=None):
        super().__init__(outputSize)
        self.inputSize, self.outputSize, self.withBias = inputSize, outputSize, withBias
        self.Kp = _ceil(inputSize, 16)
        self.weight = torch.zeros(outputSize, self.Kp, dtype=torch.int8)
        self.weightScale = torch.zeros(outputSize)
        self.bias = torch.zeros(outputSize)
        self._buffers = ["weight", "weightScale", "bias"]
        if initWeight is not None:
            self.set_float_weights(initWeight, initBias)

    def set_float_weights(self, w, b=None):
        w = torch.as_tensor(w).reshape(self.outputSize, self.inputSize).float().cpu()
        q, s = quantize_rows(w)
        dev = self.weight.device
        qp = torch.zeros(self.outputSize, self.Kp, dtype=torch.int8)
        qp[:, : self.inputSize] = q
        self.weight, self.weightScale = qp.to(dev), s.to(dev)
        self.bias = (torch.as_tensor(b).float().reshape(-1) if b is not None else torch.zeros(self.outputSize)).to(dev)
        return self

    def dequantized_weight(self):
        return self.weight[:, : self.inputSize].float() * self.weightScale[:, None]

    def quantized_weight(self):
        """The int8 weight as a QuantizedTensor (reference ``weight: QuantizedTensor``), sharing the kernel's bytes."""
        from ..tensor.quantized import QuantizedTensor

        return QuantizedTensor.from_scaled(self.weight[:, : self.inputSize], self.weightScale,
                                           {"kind": "LinearWeight", "outputSize": self.outputSize,
                                            "inputSize": self.inputSize})

    def updateOutput(self, input):
        assert input.dim() in (1, 2), "quantized.Linear: input must be a vector or a batch of vectors"
        x = input.unsqueeze(0) if input.dim() == 1 else input
        assert x.shape[1] == self.inputSize, f"quantized.Linear: expected {self.inputSize} inputs, got {x.shape[1]}"
        if x.is_cuda:
            y = self._fwd_gpu(x)
        else:
            q, sx = quantize_per_sample_ref(x)
            acc = q.double() @ self.weight[:, : self.inputSize].double().t()
            y = (acc * sx.double()[:, None] * self.weightScale.double()[None, :]).float() + self.bias
        self.output = y.squeeze(0) if input.dim() == 1 else y
        return self.output

    def _fwd_gpu(self, x):
        B = x.shape[0]
        if x.dtype not in (BF16, torch.float32):
            x = x.float()
        q, sx = quantize_act_gpu(x.contiguous(), self.inputSize, self.Kp, getattr(self, "inputAmax", None))
        out = torch.empty(B, self.outputSize, dtype=torch.float32, device=x.device)
        geo = [B, 1, 1, self.Kp, 1, 1, 1, 1, self.Kp, self.outputSize, self.outputSize, 1, 1, 1, 1, 0, 0]
        native.get().conv_i8(q, self.weight, out, self.bias, sx, self.weightScale, geo, [0, 0, 0], False)
        return out

    def __repr__(self):
        return f"quantized.Linear({self.inputSize} -> {self.outputSize})"


class QuantizedSpatialConvolution(QuantizedModule):
    """int8 2-D convolution (reference quantized/SpatialConvolution.scala:33). Accepts NCHW input (or NHWC
    with ``format='NHWC'``); on the GPU the output is bf16 channels-last like the float engine's convs."""

    def __init__(self, nInputPlane, nOutputPlane, kernelW, kernelH, strideW=1, strideH=1, padW=0, padH=0,
                 nGroup=1, initWeight=None, initBias=None, format="NCHW", dilationW=1, dilationH=1, withBias=True):
        super().__init__(nOutputPlane)
        assert nInputPlane % nGroup == 0, "Number of input channels should be multiples of group."
        assert nOutputPlane % nGroup == 0, "Number of output channels should be multiples of group."
        self.nInputPlane, self.nOutputPlane = nInputPlane, nOutputPlane
        self.kernelW, self.kernelH, self.strideW, self.strideH = kernelW, kernelH, strideW, strideH
        self.padW, self.padH, self.nGroup, self.format = padW, padH, nGroup, format
        self.dilationW, self.dilationH = dilationW, dilationH
        self.withBias = withBias
        cin = nInputPlane // nGroup
        self.Cp = _ceil(cin, 16)
        # int8 weight, KRSC with C padded to 16: [nOut][kH][kW][Cp] (group g owns rows g*cout:(g+1)*cout)
        self.weight = torch.zeros(nOutputPlane, kernelH, kernelW, self.Cp, dtype=torch.int8)
        self.weightScale = torch.zeros(nOutputPlane)
        self.bias = torch.zeros(nOutputPlane)
        self._buffers = ["weight", "weightScale", "bias"]
        self.fuse_relu = False
        if initWeight is not None:
            self.set_float_weights(initWeight, initBias)

    def set_float_weights(self, w, b=None):
        cin = self.nInputPlane // self.nGroup
        w = torch.as_tensor(w).float().cpu().reshape(self.nOutputPlane, cin, self.kernelH, self.kernelW)
        q, s = quantize_rows(w.reshape(self.nOutputPlane, -1))
        q = q.reshape(self.nOutputPlane, cin, self.kernelH, self.kernelW).permute(0, 2, 3, 1)
        qp = torch.zeros(self.nOutputPlane, self.kernelH, self.kernelW, self.Cp, dtype=torch.int8)
        qp[..., :cin] = q
        dev = self.weight.device
        self.weight, self.weightScale = qp.to(dev), s.to(dev)
        self.bias = (torch.as_tensor(b).float().reshape(-1) if b is not None
                     else torch.zeros(self.nOutputPlane)).to(dev)
        return self

    def quantized_weight(self):
        """The int8 weight [nOutputPlane, kH, kW, nInputPlane / nGroup] (NHWC order, as the i8 kernels read it) as a
        QuantizedTensor sharing the kernel's bytes."""
        from ..tensor.quantized import QuantizedTensor

        cin = self.nInputPlane // self.nGroup
        return QuantizedTensor.from_scaled(self.weight[..., :cin], self.weightScale, {"kind": "ConvWeight"})

    def dequantized_weight(self):
        cin = self.nInputPlane // self.nGroup
        return self.weight[..., :cin].permute(0, 3, 1, 2).float() * self.weightScale[:, None, None, None]

    def _pads(self, H, W):
        if self.padW == -1 and self.padH == -1:
            def same(inp, k, s, d):
                out = -(-inp // s)
                return max((out - 1) * s + (k - 1) * d + 1 - inp, 0) // 2
            return same(H, self.kernelH, self.strideH, self.dilationH), same(W, self.kernelW, self.strideW,
                                                                              self.dilationW)
        return self.padH, self.padW

    def updateOutput(self, input):
        x = input.permute(0, 3, 1, 2) if self.format == "NHWC" else input
        squeeze = x.dim() == 3
        if squeeze:
            x = x.unsqueeze(0)
        assert x.shape[1] == self.nInputPlane, f"input channel size {x.shape[1]} != {self.nInputPlane}"
        ph, pw = self._pads(x.shape[2], x.shape[3])
        y = self._fwd_gpu(x, ph, pw) if x.is_cuda else self._fwd_cpu(x, ph, pw)
        if squeeze:
            y = y.squeeze(0)
        self.output = y.permute(0, 2, 3, 1) if self.format == "NHWC" else y
        return self.output

    def _fwd_cpu(self, x, ph, pw):
        G = self.nGroup
        cin, cout = self.nInputPlane // G, self.nOutputPlane // G
        wq = self.weight[..., :cin].permute(0, 3, 1, 2).double()
        ys = []
        for g in range(G):
            q, sx = quantize_per_sample_ref(x[:, g * cin:(g + 1) * cin])
            acc = F.conv2d(q.double(), wq[g * cout:(g + 1) * cout], None, (self.strideH, self.strideW), (ph, pw),
                           (self.dilationH, self.dilationW))
            ys.append(acc * sx.double()[:, None, None, None]
                      * self.weightScale[g * cout:(g + 1) * cout].double()[None, :, None, None])
        y = (torch.cat(ys, 1) if G > 1 else ys[0]).float() + self.bias[None, :, None, None]
        if self.fuse_relu:
            y = torch.relu(y)
        return y

    def _fwd_gpu(self, x, ph, pw):
        from ..ops.conv import _fwd_taps, out_size

        N, C, H, W = x.shape
        G = self.nGroup
        cin, cout = C // G, self.nOutputPlane // G
        R, S = self.kernelH, self.kernelW
        OH = out_size(H, R, self.strideH, ph, self.dilationH)
        OW = out_size(W, S, self.strideW, pw, self.dilationW)
        if x.dtype not in (BF16, torch.float32):
            x = x.float()
        xn = x.permute(0, 2, 3, 1)            # NHWC view; contiguous when x is channels-last
        taps = _fwd_taps(R, S, ph, pw, self.dilationH, self.dilationW)
        ys = []
        for g in range(G):
            xg = xn if G == 1 else xn[..., g * cin:(g + 1) * cin]
            q, sx = quantize_act_gpu(xg.contiguous(), cin, self.Cp, getattr(self, "inputAmax", None))
            y = torch.empty((N, cout, OH, OW), dtype=BF16, device=x.device, memory_format=CL)
            geo = [N, H, W, self.Cp, OH, OW, self.strideH, self.strideW, R * S * self.Cp, cout, cout,
                   OH, OW, 1, 1, 0, 0]
            wg = self.weight if G == 1 else self.weight[g * cout:(g + 1) * cout].contiguous()
            bg = self.bias if G == 1 else self.bias[g * cout:(g + 1) * cout].contiguous()
            sg = self.weightScale if G == 1 else self.weightScale[g * cout:(g + 1) * cout].contiguous()
            native.get().conv_i8(q, wg, y, bg, sx, sg, geo, taps, self.fuse_relu)
            ys.append(y)
        return ys[0] if G == 1 else torch.cat(ys, 1).contiguous(memory_format=CL)

    def __repr__(self):
        return (f"quantized.SpatialConvolution({self.nInputPlane} -> {self.nOutputPlane}, {self.kernelW} x "
                f"{self.kernelH}, {self.strideW}, {self.strideH}, {self.padW}, {self.padH})")


class QuantizedSpatialDilatedConvolution(QuantizedSpatialConvolution):
    """int8 dilated convolution (reference quantized/SpatialDilatedConvolution.scala:27)."""

    def __init__(self, nInputPlane, nOutputPlane, kW, kH, dW=1, dH=1, padW=0, padH=0, dilationW=1, dilationH=1,
                 initWeight=None, initBias=None, format="NCHW"):
        super().__init__(nInputPlane, nOutputPlane, kW, kH, dW, dH, padW, padH, 1, initWeight, initBias, format,
                         dilationW, dilationH)

    def __repr__(self):
        return (f"quantized.SpatialDilatedConvolution({self.nInputPlane} -> {self.nOutputPlane}, {self.kernelW} x "
                f"{self.kernelH}, dilation {self.dilationW} x {self.dilationH})")


def quantization_loss(before, after):
    """Relative L1 error of a quantized tensor (reference Quantization.scala:148-166)."""
    return float((before.float() - after.float()).abs().sum() / before.float().sum())
