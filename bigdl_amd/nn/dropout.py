"""Dropout / noise layers (reference S/nn/Dropout.scala:44, SpatialDropout1D/2D/3D, GaussianDropout,
GaussianNoise, GaussianSampler). In training mode the mask is regenerated from the device RNG and kept
only for the backward of the same step."""
import torch

from .abstractnn import AutogradModule, TensorModule


class Dropout(TensorModule):
    def __init__(self, initP=0.5, inplace=False, scale=True):
        super().__init__()
        self.p, self.inplace, self.scale = initP, inplace, scale

    def setP(self, p):
        self.p = p
        return self

    def getP(self):
        return self.p

    def updateOutput(self, input):
        self._seed = None
        if not self.train or self.p == 0:
            self._mask = None
            return input
        if input.is_cuda and input.dtype in (torch.float32, torch.bfloat16):
            from ..ops import nnk      # Philox keep-mask, regenerated in backward (csrc/nn_misc.hip)

            self._mask = None
            self._seed = nnk.next_seed()
            return nnk.dropout_gpu(input, self.p, self.scale, self._seed)
        keep = 1.0 - self.p
        mask = (torch.rand(input.shape, device=input.device) < keep).to(input.dtype)
        if self.scale:
            mask = mask / keep
        self._mask = mask
        return input * mask

    def updateGradInput(self, input, gradOutput):
        if getattr(self, "_seed", None) is not None:
            from ..ops import nnk

            return nnk.dropout_gpu(gradOutput.to(input.dtype), self.p, self.scale, self._seed)
        if self._mask is None:
            return gradOutput
        return gradOutput * self._mask


class _ChannelDropout(TensorModule):
    spatial_dims = 2

    def __init__(self, initP=0.5, format="NCHW"):
        super().__init__()
        self.p, self.format = initP, format

    def updateOutput(self, input):
        if not self.train or self.p == 0:
            self._mask = None
            return input
        shape = list(input.shape)
        if self.format == "NCHW":
            for i in range(input.dim() - self.spatial_dims, input.dim()):
                shape[i] = 1
        else:
            for i in range(1, 1 + self.spatial_dims):
                shape[i] = 1
        self._mask = (torch.rand(shape, device=input.device) >= self.p).to(input.dtype)
        return input * self._mask

    def updateGradInput(self, input, gradOutput):
        return gradOutput if self._mask is None else gradOutput * self._mask


class SpatialDropout1D(_ChannelDropout):
    spatial_dims = 1

    def __init__(self, initP=0.5):
        super().__init__(initP, "NHWC")


class SpatialDropout2D(_ChannelDropout):
    spatial_dims = 2


class SpatialDropout3D(_ChannelDropout):
    spatial_dims = 3


class GaussianDropout(TensorModule):
    def __init__(self, rate):
        super().__init__()
        self.rate = rate

    def updateOutput(self, input):
        if not self.train:
            self._mask = None
            return input
        std = (self.rate / (1.0 - self.rate)) ** 0.5
        self._mask = 1.0 + std * torch.randn_like(input)
        return input * self._mask

    def updateGradInput(self, input, gradOutput):
        return gradOutput if self._mask is None else gradOutput * self._mask


class GaussianNoise(TensorModule):
    def __init__(self, stddev):
        super().__init__()
        self.stddev = stddev

    def updateOutput(self, input):
        if not self.train:
            return input
        return input + self.stddev * torch.randn_like(input)

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class GaussianSampler(AutogradModule):
    """Table(mean, logVar) -> mean + exp(logVar/2) * eps (VAE reparameterisation)."""

    def fn(self, x):
        mean, logvar = x[1], x[2]
        eps = torch.randn_like(mean)
        return mean + torch.exp(0.5 * logvar) * eps


__all__ = ["Dropout", "SpatialDropout1D", "SpatialDropout2D", "SpatialDropout3D", "GaussianDropout",
           "GaussianNoise", "GaussianSampler"]
