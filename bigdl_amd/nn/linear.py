"""Dense layers. Reference: S/nn/Linear.scala:84-160 (fwd addmm, bwd-data :128, bwd-weight :154),
SparseLinear.scala, Bilinear.scala, LookupTable.scala:47, LookupTableSparse.scala, MM.scala, MV.scala,
Cosine.scala, CosineDistance.scala, Euclidean.scala, PairwiseDistance.scala, DotProduct.scala,
CrossProduct.scala, Maxout.scala, Highway.scala.

GPU engine: Linear runs on the MFMA GEMM kernels of csrc/conv_igemm.hip (a Linear layer IS a 1x1
convolution over a 1x1 image: fwd = NT GEMM with fused bias/ReLU, dgrad = NT GEMM against the transposed
weight, wgrad = split-K TN GEMM accumulated in fp32 into the flat gradient buffer). Feature sizes that are
not multiples of 8 are zero-padded on the fly.

Large plain GEMMs (a language model's vocabulary projection, an RNN's input projection: M >= 8192 rows, K >= 512,
N >= 2048) go to hipBLASLt instead (torch.addmm / torch.mm with fp32 accumulation; the weight gradient in fp32
straight from the GEMM, the bias gradient as one extra ones-column of the input): on the PTB LM's shapes it runs
15-40 % faster than the in-tree tiles (tools/lm_gemm_vs_blas.py, profiles/r6_lm_gemm_vs_hipblaslt.log), while the
convolution-shaped and fused GEMMs stay on the in-tree kernels, which beat it there (tools/gemm_vs_blas.py).
BIGDL_LINEAR_BLAS=0 keeps every Linear on the in-tree kernels.
"""
import math
import os

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import conv as cv
from ..ops import conv_fn
from ..ops import native
from .abstractnn import AutogradModule, TensorModule
from .init_methods import RandomUniform

BF16 = torch.bfloat16
CL = torch.channels_last


def _pad8(n):
    return -(-n // 8) * 8


_BLAS = [os.environ.get("BIGDL_LINEAR_BLAS", "1") != "0"]


def _blas_shape(M, K, N):
    return M >= 8192 and K >= 512 and N >= 2048


class Linear(TensorModule):
    def __init__(self, inputSize, outputSize, withBias=True, wRegularizer=None, bRegularizer=None,
                 initWeight=None, initBias=None, initGradWeight=None, initGradBias=None):
        super().__init__()
        self.inputSize, self.outputSize, self.withBias = inputSize, outputSize, withBias
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.fuse_relu = False
        self.register_parameter("weight", "gradWeight", torch.empty(outputSize, inputSize))
        if withBias:
            self.register_parameter("bias", "gradBias", torch.empty(outputSize))
        else:
            self.bias = self.gradBias = None
        stdv = 1.0 / math.sqrt(inputSize)
        self.weightInitMethod = RandomUniform(-stdv, stdv)
        self.biasInitMethod = RandomUniform(-stdv, stdv)
        self.reset()
        if initWeight is not None:
            self.weight.copy_(torch.as_tensor(initWeight).reshape(self.weight.shape))
        if initBias is not None and withBias:
            self.bias.copy_(torch.as_tensor(initBias).reshape(self.bias.shape))
        if initGradWeight is not None:
            self.gradWeight.copy_(torch.as_tensor(initGradWeight).reshape(self.weight.shape))
        if initGradBias is not None and withBias:
            self.gradBias.copy_(torch.as_tensor(initGradBias).reshape(self.bias.shape))

    def reset(self):
        with torch.no_grad():
            self.weightInitMethod.init(self.weight, "out_in")
            if self.bias is not None:
                self.biasInitMethod.init(self.bias)

    # ------------------------------------------------------------------ GPU helpers
    def _padded(self):
        return _pad8(self.inputSize) != self.inputSize or _pad8(self.outputSize) != self.outputSize

    def _w16_4d(self):
        """(Op, Ip, 1, 1) bf16 weight (zero padded to multiples of 8)."""
        w16 = self.w16("weight")
        Ip, Op = _pad8(self.inputSize), _pad8(self.outputSize)
        if Ip != self.inputSize or Op != self.outputSize:
            w16 = F.pad(w16, (0, Ip - self.inputSize, 0, Op - self.outputSize))
        return w16.contiguous().view(Op, Ip, 1, 1)

    def _x4d(self, x):
        B = x.shape[0]
        Ip = _pad8(self.inputSize)
        if x.dtype != BF16:
            x = ops.to_bf16(x.contiguous()) if x.dtype == torch.float32 else x.to(BF16)
        x = x.contiguous()
        if Ip != self.inputSize:
            x = F.pad(x, (0, Ip - self.inputSize))
        return x.view(B, Ip, 1, 1)

    def _use_blas(self, M):
        if not _BLAS[0] or self._padded() or self.fuse_relu or not _blas_shape(M, self.inputSize, self.outputSize):
            return False
        from ..ops import native

        return not native.deterministic()

    def _blas_fwd(self, x):
        """hipBLASLt forward; keeps [x | 1 | 0...] (bf16, one extra 8-column block) for the weight gradient, whose
        GEMM then yields the bias gradient as its last column."""
        M, K = x.shape
        x16 = x if x.dtype == BF16 else (ops.to_bf16(x.contiguous()) if x.dtype == torch.float32 else x.to(BF16))
        w16 = self.w16("weight")
        if self.bias is not None:
            xe = torch.empty(M, K + 8, dtype=BF16, device=x.device)
            native.get().ones_col_pack(x16.contiguous(), xe)      # [x | 1 | 0...] in one pass (no aten fills)
            self._xe = xe
            y = torch.addmm(self.w16("bias"), xe[:, :K], w16.t())
        else:
            self._xe = x16.contiguous()
            y = torch.mm(self._xe, w16.t())
        self._x4 = None
        return y

    def updateOutput(self, input):
        x = input
        lead = None
        if x.dim() == 1:
            x = x.unsqueeze(0)
        elif x.dim() > 2:
            lead = x.shape[:-1]
            x = x.reshape(-1, x.shape[-1])
        self._xe = None
        if x.is_cuda and self._use_blas(x.shape[0]):
            y = self._blas_fwd(x)
        elif x.is_cuda:
            x4 = self._x4d(x)
            self._x4 = x4
            bias = self.bias
            Op = _pad8(self.outputSize)
            if bias is not None and Op != self.outputSize:
                bias = F.pad(bias, (0, Op - self.outputSize))
            y = cv.conv2d_fwd(x4, self._w16_4d(), bias, (1, 1), (0, 0), relu=self.fuse_relu)
            y = y.view(x.shape[0], Op)
            if Op != self.outputSize:
                y = y[:, : self.outputSize].contiguous()
        else:
            y = F.linear(x.float(), self.weight, self.bias)
            if self.fuse_relu:
                y = torch.relu(y)
        if input.dim() == 1:
            y = y.squeeze(0)
        elif lead is not None:
            y = y.reshape(tuple(lead) + (self.outputSize,))
        return y

    def _gy2d(self, gradOutput):
        g = gradOutput
        if g.dim() == 1:
            g = g.unsqueeze(0)
        elif g.dim() > 2:
            g = g.reshape(-1, g.shape[-1])
        if self.fuse_relu:
            out = self.output.reshape(g.shape)
            g = g * (out > 0).to(g.dtype)
        return g

    def updateGradInput(self, input, gradOutput):
        g = self._gy2d(gradOutput)
        if g.is_cuda and getattr(self, "_xe", None) is not None:
            g16 = ops.to_bf16(g) if g.dtype == torch.float32 else g.to(BF16).contiguous()
            self._g16 = g16
            gi = torch.mm(g16, self.w16("weight"))
        elif g.is_cuda:
            B = g.shape[0]
            Op, Ip = _pad8(self.outputSize), _pad8(self.inputSize)
            g16 = ops.to_bf16(g) if g.dtype == torch.float32 else g.to(BF16).contiguous()
            if Op != self.outputSize:
                g16 = F.pad(g16, (0, Op - self.outputSize))
            g4 = g16.view(B, Op, 1, 1)
            wt = cv.transpose_w(self._w16_4d())           # (Ip, 1, 1, Op)
            gi = cv.conv2d_dgrad(g4, wt, (B, Ip, 1, 1), (1, 1), (0, 0)).view(B, Ip)
            if Ip != self.inputSize:
                gi = gi[:, : self.inputSize].contiguous()
            self._g16 = g4
        else:
            gi = g.float() @ self.weight
        return gi.reshape(input.shape)

    def accGradParameters(self, input, gradOutput):
        g = self._gy2d(gradOutput)
        if g.is_cuda and getattr(self, "_xe", None) is not None:
            g16 = getattr(self, "_g16", None)
            if g16 is None or g16.dim() != 2 or g16.shape[0] != g.shape[0]:
                g16 = ops.to_bf16(g) if g.dtype == torch.float32 else g.to(BF16).contiguous()
            K = self.inputSize
            gw = torch.mm(g16.t(), self._xe, out_dtype=torch.float32)     # [N, K (+8)] fp32 from the GEMM
            if self.bias is not None and self.gradWeight.is_contiguous():
                native.get().ones_col_acc(gw, self.gradWeight, self.gradBias, self.scaleW, self.scaleB)
            elif self.bias is not None:
                self.gradWeight.add_(gw[:, :K], alpha=self.scaleW)
                self.gradBias.add_(gw[:, K], alpha=self.scaleB)
            else:
                self.gradWeight.add_(gw, alpha=self.scaleW)
            self._g16 = None
            return
        if g.is_cuda:
            g4 = getattr(self, "_g16", None)
            if g4 is None or g4.shape[0] != g.shape[0]:
                Op = _pad8(self.outputSize)
                g16 = ops.to_bf16(g) if g.dtype == torch.float32 else g.to(BF16).contiguous()
                if Op != self.outputSize:
                    g16 = F.pad(g16, (0, Op - self.outputSize))
                g4 = g16.view(g.shape[0], Op, 1, 1)
            x4 = self._x4
            direct = (not self._padded()) and self.scaleW == 1.0 and self.scaleB == 1.0
            if direct:
                cv.conv2d_wgrad(g4, x4, self.gradWeight.view(self.outputSize, self.inputSize, 1, 1),
                                self.gradBias, (1, 1), (0, 0))
            else:
                Op, Ip = g4.shape[1], x4.shape[1]
                dw = torch.zeros(Op, Ip, 1, 1, device=g.device)
                db = torch.zeros(Op, device=g.device) if self.bias is not None else None
                cv.conv2d_wgrad(g4, x4, dw, db, (1, 1), (0, 0))
                self.gradWeight.add_(dw.view(Op, Ip)[: self.outputSize, : self.inputSize], alpha=self.scaleW)
                if db is not None:
                    self.gradBias.add_(db[: self.outputSize], alpha=self.scaleB)
            self._g16 = None
            return
        x = input
        if x.dim() == 1:
            x = x.unsqueeze(0)
        elif x.dim() > 2:
            x = x.reshape(-1, x.shape[-1])
        gf = g.float()
        self.gradWeight.add_(gf.t() @ x.float(), alpha=self.scaleW)
        if self.bias is not None:
            self.gradBias.add_(gf.sum(0), alpha=self.scaleB)

    def __repr__(self):
        return f"Linear({self.inputSize} -> {self.outputSize})"


class SparseLinear(AutogradModule):
    """Linear over a sparse (COO) input (reference SparseLinear.scala; wide & deep models)."""

    def __init__(self, inputSize, outputSize, withBias=True, backwardStart=-1, backwardLength=-1,
                 wRegularizer=None, bRegularizer=None, initWeight=None, initBias=None):
        super().__init__()
        self.inputSize, self.outputSize = inputSize, outputSize
        self.register_parameter("weight", "gradWeight", torch.empty(outputSize, inputSize))
        if withBias:
            self.register_parameter("bias", "gradBias", torch.empty(outputSize))
        else:
            self.bias = None
        stdv = 1.0 / math.sqrt(inputSize)
        RandomUniform(-stdv, stdv).init(self.weight)
        if self.bias is not None:
            RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        if x.is_sparse:
            y = torch.sparse.mm(x.float(), self.weight.t())
        else:
            y = x.float() @ self.weight.t()
        return y + self.bias if self.bias is not None else y


class Bilinear(AutogradModule):
    def __init__(self, inputSize1, inputSize2, outputSize, biasRes=True, wRegularizer=None, bRegularizer=None):
        super().__init__()
        self.register_parameter("weight", "gradWeight", torch.empty(outputSize, inputSize1, inputSize2))
        if biasRes:
            self.register_parameter("bias", "gradBias", torch.empty(outputSize))
        else:
            self.bias = None
        stdv = 1.0 / math.sqrt(inputSize1)
        RandomUniform(-stdv, stdv).init(self.weight)
        if self.bias is not None:
            RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        return F.bilinear(x[1].float(), x[2].float(), self.weight, self.bias)


class LookupTable(TensorModule):
    """Embedding lookup with 1-based indices (reference LookupTable.scala:47, incl. maxNorm renorm)."""

    def __init__(self, nIndex, nOutput, paddingValue=0.0, maxNorm=float("inf"), normType=2.0,
                 shouldScaleGradByFreq=False, wRegularizer=None, maskZero=False):
        super().__init__()
        self.nIndex, self.nOutput = nIndex, nOutput
        self.paddingValue, self.maxNorm, self.normType = paddingValue, maxNorm, normType
        self.shouldScaleGradByFreq, self.maskZero = shouldScaleGradByFreq, maskZero
        self.wRegularizer = wRegularizer
        self.register_parameter("weight", "gradWeight", torch.empty(nIndex, nOutput))
        self.reset()

    def reset(self):
        with torch.no_grad():
            self.weight.normal_(0, 1)

    def _idx(self, input):
        idx = input.long() - 1
        if self.maskZero:
            idx = idx.clamp_min(-1)
        return idx

    def _native_ids(self, input):
        """GPU fast path: the kernels read the raw 1-based ids (no index tensor, no aten index arithmetic)."""
        return (input.is_cuda and self.weight.is_cuda and self.weight.dtype == torch.float32
                and input.dtype in (torch.float32, torch.int64) and self.maxNorm == float("inf"))

    def updateOutput(self, input):
        if self._native_ids(input):
            from ..ops import native

            ids = input.contiguous()
            out = torch.empty(tuple(ids.shape) + (self.nOutput,), device=ids.device, dtype=torch.float32)
            native.get().embedding_fwd_ids(self.weight, ids, out, bool(self.maskZero))
            return out
        idx = self._idx(input)
        if self.maxNorm != float("inf"):
            with torch.no_grad():
                rows = idx[idx >= 0].unique()
                w = self.weight[rows]
                n = w.norm(p=self.normType, dim=1, keepdim=True)
                scale = torch.where(n > self.maxNorm, self.maxNorm / (n + 1e-7), torch.ones_like(n))
                self.weight[rows] = w * scale
        safe = idx.clamp_min(0)
        if self.weight.is_cuda and self.weight.dtype == torch.float32:
            from ..ops import nnk      # wave-per-row gather (csrc/nn_misc.hip); negative ids -> zero rows

            return nnk.embedding_fwd_gpu(self.weight, idx if self.maskZero else safe)
        out = self.weight[safe]
        if self.maskZero:
            out = out * (idx >= 0).unsqueeze(-1).to(out.dtype)
        return out

    def updateGradInput(self, input, gradOutput):
        gi = torch.empty_like(input, dtype=torch.float32)
        if gi.is_cuda:
            from ..ops import native

            native.get().fill_bytes(gi, 0)
            return gi
        return gi.zero_()

    def accGradParameters(self, input, gradOutput):
        if (self._native_ids(input) and self.gradWeight.is_cuda and not self.shouldScaleGradByFreq
                and gradOutput.dtype in (torch.float32, torch.bfloat16)):
            from ..ops import native

            pad = int(self.paddingValue) - 1 if self.paddingValue != 0 else -1
            native.get().embedding_bwd_ids(gradOutput.contiguous(), input.contiguous(), self.gradWeight, pad,
                                           float(self.scaleW))
            return
        idx = self._idx(input).reshape(-1)
        g = gradOutput.reshape(-1, self.nOutput).float()
        keep = idx >= 0
        if self.paddingValue != 0:
            keep = keep & (idx != int(self.paddingValue) - 1)
        if self.gradWeight.is_cuda and not self.shouldScaleGradByFreq:
            from ..ops import nnk      # fp32 atomic scatter-add straight into gradWeight

            nnk.embedding_bwd_gpu(self.gradWeight, torch.where(keep, idx, torch.full_like(idx, -1)), g, self.scaleW)
            return
        idx, g = idx[keep], g[keep]
        if self.shouldScaleGradByFreq:
            cnt = torch.bincount(idx, minlength=self.nIndex).float()
            g = g / cnt[idx].unsqueeze(1)
        self.gradWeight.index_add_(0, idx.to(self.gradWeight.device), g.to(self.gradWeight.device), alpha=self.scaleW)


class LookupTableSparse(AutogradModule):
    """Sparse-id embedding with ``combiner`` in {sum, mean, sqrtn} (reference LookupTableSparse.scala:47)."""

    def __init__(self, nIndex, nOutput, combiner="sum", maxNorm=-1.0, wRegularizer=None):
        super().__init__()
        self.combiner = combiner
        self.register_parameter("weight", "gradWeight", torch.empty(nIndex, nOutput).normal_(0, 1))

    def fn(self, x):
        ids, weights = (x[1], x[2]) if not isinstance(x, torch.Tensor) else (x, None)
        dense = ids.to_dense() if ids.is_sparse else ids
        idx = dense.long() - 1
        mask = (idx >= 0).float()
        w = mask if weights is None else (weights.to_dense() if weights.is_sparse else weights).float() * mask
        emb = self.weight[idx.clamp_min(0)] * w.unsqueeze(-1)
        s = emb.sum(1)
        if self.combiner == "mean":
            s = s / w.sum(1, keepdim=True).clamp_min(1e-12)
        elif self.combiner == "sqrtn":
            s = s / (w * w).sum(1, keepdim=True).sqrt().clamp_min(1e-12)
        return s


class MM(AutogradModule):
    def __init__(self, transA=False, transB=False):
        super().__init__()
        self.transA, self.transB = transA, transB

    def fn(self, x):
        a, b = x[1], x[2]
        if self.transA:
            a = a.transpose(-1, -2)
        if self.transB:
            b = b.transpose(-1, -2)
        if a.is_cuda:       # native batched bf16 MFMA GEMM (ops/bmm.py, csrc/bmm.hip), gradients on the same kernel
            from ..ops.bmm import matmul

            return matmul(a, b)
        return a @ b


class Gemm(AutogradModule):
    """y = alpha * op(A) * op(B) + beta * C (ONNX Gemm; reference S/nn/onnx/Gemm.scala:25-80, P/nn/layer.py Gemm).

    Input is A with B and C given at construction (``matrixB`` / ``matrixC``, as the ONNX importer builds it), or a
    Table(A, B, C). 2-D operands on the GPU engine run on the native MFMA GEMM (``ops/conv_fn.linear``)."""

    def __init__(self, alpha=1.0, beta=1.0, transA=False, transB=False, matrixB=None, matrixC=None):
        super().__init__()
        self.alpha, self.beta, self.transA, self.transB = float(alpha), float(beta), bool(transA), bool(transB)
        self.matrixB = None if matrixB is None else torch.as_tensor(matrixB, dtype=torch.float32)
        self.matrixC = None if matrixC is None else torch.as_tensor(matrixC, dtype=torch.float32)

    def fn(self, x):
        if isinstance(x, torch.Tensor):
            a, b, c = x, self.matrixB.to(x.device), self.matrixC.to(x.device)
        else:
            a, b, c = x[1], x[2], x[3]
        a = a.transpose(-1, -2) if self.transA else a
        b = b.transpose(-1, -2) if self.transB else b
        if a.dim() == 2 and b.dim() == 2:
            ab = conv_fn.linear(a.float(), b.float().t().contiguous())     # a @ b
        else:
            ab = a.float() @ b.float()
        return self.alpha * ab + self.beta * c.float()


class MV(AutogradModule):
    def __init__(self, trans=False):
        super().__init__()
        self.trans = trans

    def fn(self, x):
        m, v = x[1], x[2]
        if self.trans:
            m = m.transpose(-1, -2)
        if m.is_cuda:
            from ..ops.bmm import matmul

            return matmul(m, v.unsqueeze(-1)).squeeze(-1)
        return (m @ v.unsqueeze(-1)).squeeze(-1)


class DotProduct(AutogradModule):
    def fn(self, x):
        return (x[1] * x[2]).sum(-1)


class CosineDistance(AutogradModule):
    def fn(self, x):
        return F.cosine_similarity(x[1].float(), x[2].float(), dim=-1, eps=1e-12)


class PairwiseDistance(AutogradModule):
    def __init__(self, norm=2):
        super().__init__()
        self.norm = norm

    def fn(self, x):
        return (x[1] - x[2]).abs().pow(self.norm).sum(-1).pow(1.0 / self.norm)


class Cosine(AutogradModule):
    """Cosine similarity of the input to each of outputSize learnable vectors."""

    def __init__(self, inputSize, outputSize):
        super().__init__()
        self.register_parameter("weight", "gradWeight", torch.empty(outputSize, inputSize))
        stdv = 1.0 / math.sqrt(inputSize)
        RandomUniform(-stdv, stdv).init(self.weight)

    def fn(self, x):
        xs = x if x.dim() > 1 else x.unsqueeze(0)
        y = conv_fn.linear(F.normalize(xs.float(), dim=1, eps=1e-12), F.normalize(self.weight, dim=1, eps=1e-12))
        return y if x.dim() > 1 else y.squeeze(0)


class Euclidean(AutogradModule):
    def __init__(self, inputSize, outputSize, fastBackward=True):
        super().__init__()
        self.register_parameter("weight", "gradWeight", torch.empty(inputSize, outputSize))
        stdv = 1.0 / math.sqrt(inputSize)
        RandomUniform(-stdv, stdv).init(self.weight)

    def fn(self, x):
        xs = x if x.dim() > 1 else x.unsqueeze(0)
        d = (xs.float().unsqueeze(2) - self.weight.unsqueeze(0)).pow(2).sum(1).sqrt()
        return d if x.dim() > 1 else d.squeeze(0)


class CrossProduct(AutogradModule):
    """Pairwise dot products between all tensors of the input table."""

    def __init__(self, numTensor=0, embeddingSize=0):
        super().__init__()

    def fn(self, x):
        ts = x.toSeq()
        outs = []
        for i in range(len(ts)):
            for j in range(i + 1, len(ts)):
                outs.append((ts[i] * ts[j]).sum(-1, keepdim=True))
        return torch.cat(outs, dim=-1)


class Maxout(AutogradModule):
    def __init__(self, inputSize, outputSize, maxoutNumber, withBias=True, wRegularizer=None, bRegularizer=None,
                 initWeight=None, initBias=None):
        super().__init__()
        self.outputSize, self.k = outputSize, maxoutNumber
        self.register_parameter("weight", "gradWeight", torch.empty(outputSize * maxoutNumber, inputSize))
        self.register_parameter("bias", "gradBias", torch.empty(outputSize * maxoutNumber))
        stdv = 1.0 / math.sqrt(inputSize)
        RandomUniform(-stdv, stdv).init(self.weight)
        RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        y = conv_fn.linear(x.float(), self.weight, self.bias)          # GPU: MFMA GEMM
        return y.view(y.shape[0], self.outputSize, self.k).max(dim=2).values


class Highway(AutogradModule):
    def __init__(self, size, withBias=True, activation=None, wRegularizer=None, bRegularizer=None):
        super().__init__()
        self.size = size
        self.register_parameter("weight", "gradWeight", torch.empty(2 * size, size))
        self.register_parameter("bias", "gradBias", torch.zeros(2 * size))
        self.activation = activation
        stdv = 1.0 / math.sqrt(size)
        RandomUniform(-stdv, stdv).init(self.weight)

    def fn(self, x):
        y = conv_fn.linear(x.float(), self.weight, self.bias)
        t = torch.sigmoid(y[:, : self.size])
        h = y[:, self.size:]
        h = torch.tanh(h) if self.activation is None else _act_fn(self.activation, h)
        return t * h + (1 - t) * x.float()


__all__ = ["Linear", "SparseLinear", "Bilinear", "LookupTable", "LookupTableSparse", "MM", "Gemm", "MV", "DotProduct",
           "CosineDistance", "PairwiseDistance", "Cosine", "Euclidean", "CrossProduct", "Maxout", "Highway"]


def _act_fn(m, x):
    """Differentiable application of an activation module inside an autograd-derived layer."""
    if hasattr(m, "fn"):
        return m.fn(x)
    name = type(m).__name__
    fns = {"ReLU": torch.relu, "Tanh": torch.tanh, "Sigmoid": torch.sigmoid, "Identity": lambda t: t}
    if name in fns:
        return fns[name](x)
    return m.updateOutput(x)
