"""The compiled engine's fused multi-layer RNN primitive (reference S/nn/mkldnn/RNN.scala:36-483): ``RNN(mode,
inputSize, hiddenSize, f, direction, layers)`` runs a stack of LSTM or GRU layers, in one or both directions, over a
whole sequence.

Parameters keep the reference's layouts and order (``parameters()`` = weight, bias, weight_i, RNN.scala:475-478):
  weight   [layers, dirs, inputSize, gates, hidden]   (ldigo)
  weight_i [layers, dirs, hidden, gates, hidden]      (ldigo)
  bias     [layers, dirs, gates, hidden]              (ldgo)
with the primitive's gate order: LSTM (i, f, g, o), GRU (u = z, r, n); nn/LSTM is (i, g, f, o) and nn/GRU (r, z, n)
(the mapping of RNN.scala:110-121). Input and output are TNC (default) or NTC ([T, N, C] / [N, T, C]); the output has
``hidden`` channels, ``2 * hidden`` for BidirectionalConcat (RNN.scala:100-109: concat only for one layer; with
BidirectionalSum each layer's two directions are summed before the next layer). Initial states are zero
(RNN.scala:245-248).

On the GPU every (layer, direction) is one input-projection GEMM over all T * N rows plus the whole-sequence
persistent recurrence (csrc/lstm_seq.hip: the recurrent weight resident in VGPRs for the sequence, one launch per
layer and direction, no per-step kernel boundary) where its shape applies, else the fused per-step kernels
(csrc/lstm.hip, csrc/gru.hip); the backward runs the matching persistent backward launches. On the CPU the same
recurrences run as torch loops. Layer l + 1 consumes layer l's output directly (inputSize == hidden for layers > 1,
RNN.scala:87-92).
"""
import math

import torch

from .abstractnn import AutogradModule
from .recurrent import _GRUSeq, _LSTMSeq


class AlgKind:
    """Cell kinds and activations of the reference's MKL-DNN enum (only the RNN-relevant members)."""
    VanillaLstm = "vanilla_lstm"
    VanillaGru = "vanilla_gru"
    EltwiseTanh = "eltwise_tanh"
    EltwiseRelu = "eltwise_relu"


class Direction:
    UnidirectionalLeft2Right = "unidirectional_left2right"
    UnidirectionalRight2Left = "unidirectional_right2left"
    BidirectionalConcat = "bidirectional_concat"
    BidirectionalSum = "bidirectional_sum"


class RNNCellFlags:
    RNNCellWithRelu = 0
    RNNCellWithClipping = 1


# nn-layer gate k <- primitive gate _ORDER[mode][k]
_ORDER = {AlgKind.VanillaLstm: (0, 2, 1, 3), AlgKind.VanillaGru: (1, 0, 2)}


class RNN(AutogradModule):
    def __init__(self, mode, inputSize, hiddenSize, f=AlgKind.EltwiseTanh, direction=Direction.UnidirectionalLeft2Right,
                 layers=1, flags=RNNCellFlags.RNNCellWithRelu, alpha=0.0, clipping=0.0, initWeight=None,
                 initWeightIter=None, initBias=None, inputFormat="tnc"):
        super().__init__()
        if mode not in _ORDER:
            raise ValueError(f"RNN: unsupported cell {mode!r} (VanillaLstm or VanillaGru)")
        if layers > 1 and inputSize != hiddenSize:
            raise ValueError(f"RNN: with {layers} layers the input size ({inputSize}) must equal the hidden size "
                             f"({hiddenSize})")
        if direction == Direction.BidirectionalConcat and layers != 1:
            raise ValueError("RNN: BidirectionalConcat supports one layer only")
        if direction not in (Direction.UnidirectionalLeft2Right, Direction.UnidirectionalRight2Left,
                             Direction.BidirectionalConcat, Direction.BidirectionalSum):
            raise ValueError(f"RNN: unsupported direction {direction!r}")
        if inputFormat not in ("tnc", "ntc"):
            raise ValueError("RNN: inputFormat is 'tnc' or 'ntc'")
        self.mode, self.inputSize, self.hiddenSize, self.f = mode, inputSize, hiddenSize, f
        self.direction, self.layers, self.flags, self.alpha, self.clipping = direction, layers, flags, alpha, clipping
        self.inputFormat = inputFormat
        self.ngates = 4 if mode == AlgKind.VanillaLstm else 3
        self.ndirs = 2 if direction in (Direction.BidirectionalConcat, Direction.BidirectionalSum) else 1
        L, D, G, H = layers, self.ndirs, self.ngates, hiddenSize
        self.register_parameter("weight", "gradWeight", torch.empty(L, D, inputSize, G, H))
        self.register_parameter("bias", "gradBias", torch.empty(L, D, G, H))
        self.register_parameter("weight_i", "gradWeight_i", torch.empty(L, D, H, G, H))
        self._init = (initWeight, initWeightIter, initBias)
        self.reset()

    def reset(self):
        stdv = 1.0 / math.sqrt(self.hiddenSize)
        iw, iwi, ib = self._init
        with torch.no_grad():
            for t, init in ((self.weight, iw), (self.weight_i, iwi)):
                if init is None:
                    t.uniform_(-stdv, stdv)
                else:
                    t.copy_(torch.as_tensor(init).reshape(t.shape))
            if ib is None:
                self.bias.zero_()
            else:
                self.bias.copy_(torch.as_tensor(ib).reshape(self.bias.shape))
        return self

    def outputSize(self):
        return self.hiddenSize * (2 if self.direction == Direction.BidirectionalConcat else 1)

    # -- one (layer, direction) ---------------------------------------------------------------------------------------
    def _nn_params(self, l, d):
        """(W [G H, in], U [G H, H], b [G H]) in the nn layer's gate order, differentiable w.r.t. the ldigo tensors."""
        order = list(_ORDER[self.mode])
        W = self.weight[l, d].permute(1, 2, 0)[order]          # [G, H, in]
        U = self.weight_i[l, d].permute(1, 2, 0)[order]        # [G, H, H]
        b = self.bias[l, d][order]                              # [G, H]
        G, H = self.ngates, self.hiddenSize
        return W.reshape(G * H, -1), U.reshape(G * H, H), b.reshape(G * H)

    def _run(self, x, l, d):
        """x [N, T, C] (already in this direction's time order) -> [N, T, H]."""
        N, T, C = x.shape
        H = self.hiddenSize
        W, U, b = self._nn_params(l, d)
        xf = x.float()
        xg = torch.addmm(b, xf.reshape(N * T, C), W.t()).view(N, T, -1)
        h0 = xf.new_zeros(N, H)
        if self.mode == AlgKind.VanillaLstm:
            out, _, _ = _LSTMSeq.apply(xg, h0, h0.clone(), U)
            return out.float()
        if _GRUSeq.usable(xg, H):
            out, _ = _GRUSeq.apply(xg, h0, U[:2 * H], U[2 * H:])
            return out
        Urz, Un = U[:2 * H], U[2 * H:]
        h, outs = h0, []
        for t in range(T):
            g = xg[:, t]
            rz = torch.sigmoid(g[:, :2 * H] + h @ Urz.t())
            r, z = rz[:, :H], rz[:, H:]
            n = torch.tanh(g[:, 2 * H:] + (r * h) @ Un.t())
            h = (1 - z) * n + z * h
            outs.append(h)
        return torch.stack(outs, 1)

    def fn(self, x):
        if x.dim() != 3 or x.shape[-1] != self.inputSize:
            raise ValueError(f"RNN: expected a 3-D {self.inputFormat.upper()} input with {self.inputSize} channels, "
                             f"got {tuple(x.shape)}")
        seq = x.transpose(0, 1) if self.inputFormat == "tnc" else x        # [N, T, C]
        for l in range(self.layers):
            outs = []
            for d in range(self.ndirs):
                rev = d == 1 or self.direction == Direction.UnidirectionalRight2Left
                o = self._run(seq.flip(1) if rev else seq, l, d)
                outs.append(o.flip(1) if rev else o)
            if self.direction == Direction.BidirectionalConcat:
                seq = torch.cat(outs, -1)
            elif self.direction == Direction.BidirectionalSum:
                seq = outs[0] + outs[1]
            else:
                seq = outs[0]
        seq = seq.to(x.dtype) if x.is_floating_point() else seq
        return (seq.transpose(0, 1) if self.inputFormat == "tnc" else seq).contiguous()

    def __repr__(self):
        return (f"mkldnn.RNN({self.mode}, {self.inputSize} -> {self.hiddenSize}, {self.direction}, "
                f"layers={self.layers})")


__all__ = ["RNN", "AlgKind", "Direction", "RNNCellFlags"]
