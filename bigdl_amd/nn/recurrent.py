"""Recurrent layers: Cell, RnnCell, LSTM, LSTMPeephole, GRU, ConvLSTMPeephole(3D), MultiRNNCell, Recurrent,
BiRecurrent, RecurrentDecoder, TimeDistributed.

Reference: S/nn/Cell.scala:46 (hiddensShape, preTopology, T(input, hidden) protocol), S/nn/Recurrent.scala:47-330
(preTopology hoisted out of the time loop and run once over [batch*time] rows, hidden state threaded through
per-step cell clones, maskZero, get/setHiddenState), S/nn/LSTM.scala:46-176 (gate order i, g, f, o),
S/nn/GRU.scala (r, z, n; h' = (1-z)*n + z*h), S/nn/RNN.scala:49 (RnnCell), S/nn/LSTMPeephole.scala (gate order
i, f, g, o; peepholes on c_{t-1} for i/f and on c_t for o), S/nn/ConvLSTMPeephole.scala:53 and
ConvLSTMPeephole3D.scala (conv gates, SAME padding for padding=-1), S/nn/MultiRNNCell.scala:36,
S/nn/BiRecurrent.scala:41 (reverse-time twin + merge, default CAddTable), S/nn/RecurrentDecoder.scala:79 (output of
step t is the input of step t+1), S/nn/TimeDistributed.scala.

Execution model (MI355X): the reference clones the cell graph once per time step and runs every tiny op
through the module machinery. Here the input projection (``preTopology``) is ONE large GEMM over all B*T rows
(the MFMA Linear kernels on the GPU engine); the time loop is recorded once with torch autograd on fp32 leaves
of the cell weights, so backward is a single reverse sweep. LSTM (tanh/sigmoid, p == 0) bypasses the generic
loop entirely: a sequence-level autograd Function runs ``h @ U^T`` (library GEMM) + the fused HIP cell kernel
(csrc/elementwise.hip lstm_fwd_kernel / lstm_bwd_kernel: all four gate nonlinearities, the cell update and
the gradient of both in one pass) per step, and computes dU with ONE [4H, T*B] x [T*B, H] GEMM after the
reverse sweep instead of T small ones.
"""
import os

import torch
import torch.nn.functional as F

from ..ops.conv_fn import linear as _linear

__all__ = ["Cell", "RnnCell", "RNN", "LSTM", "LSTMPeephole", "GRU", "ConvLSTMPeephole", "ConvLSTMPeephole3D", "MultiRNNCell",
           "Recurrent", "RecurrentDecoder", "BiRecurrent", "TimeDistributed"]

from .. import ops
from ..utils.table import Table
from .abstractnn import AbstractModule
from .activation import CMul, Sigmoid, Tanh
from .containers import Container
from .conv import SpatialConvolution, VolumetricConvolution, _same_pad
from .linear import Linear


# ---------------------------------------------------------------------------------------------- helpers
def _param_modules(mods):
    """Leaf modules that own parameters, in traversal order, without duplicates."""
    out, seen = [], set()

    def walk(m):
        if id(m) in seen:
            return
        seen.add(id(m))
        if m._params:
            out.append(m)
        for c in m.modules_list():
            walk(c)

    for m in mods:
        if m is not None:
            walk(m)
    return out


class _Leaves:
    """Temporarily replace module weights by fp32 autograd leaves (the reference shares one weight set across
    all time-step clones, Recurrent.scala:198 ``share``; autograd sums the per-step contributions)."""

    def __init__(self, mods, requires_grad=True):
        self.entries = [(m, w, g) for m in _param_modules(mods) for (w, g) in m._params
                        if getattr(m, w, None) is not None]
        self.requires_grad = requires_grad
        self.leaves = []

    def __enter__(self):
        self.saved = [getattr(m, w) for m, w, _ in self.entries]
        self.leaves = [t.detach().float().requires_grad_(self.requires_grad) for t in self.saved]
        for (m, w, _), leaf in zip(self.entries, self.leaves):
            object.__setattr__(m, w, leaf)
        return self

    def __exit__(self, *exc):
        for (m, w, _), t in zip(self.entries, self.saved):
            object.__setattr__(m, w, t)
        return False

    def accumulate(self, grads):
        for (m, w, g), gr in zip(self.entries, grads):
            if gr is None or m._frozen:
                continue
            gt = getattr(m, g)
            gt.add_(gr.to(gt.dtype).reshape(gt.shape), alpha=m.scaleB if w == "bias" else m.scaleW)
        for m in {id(m): m for m, _, _ in self.entries}.values():
            if not m._frozen:
                m._apply_regularizers()


def _act(m):
    """Differentiable functional form of an activation module."""
    if m is None:
        return None
    if hasattr(m, "fn"):
        return m.fn
    name = type(m).__name__
    if name == "ReLU":
        return torch.relu
    raise ValueError(f"unsupported cell activation {name}")


def _is(m, cls):
    return type(m) is cls


def _hidden_to_activity(hid):
    return hid[0] if len(hid) == 1 else Table(*hid)


def _activity_to_hidden(a):
    if isinstance(a, torch.Tensor):
        return [a]
    if isinstance(a, Table):
        out = []
        for i in range(1, len(a) + 1):
            out.extend(_activity_to_hidden(a[i]))
        return out
    return list(a)


def _copy_module_state(dst, src):
    """Copy parameters and buffers positionally (used when deserializing a cell whose sub-structure is
    rebuilt by its constructor)."""
    for a, b in zip(_param_modules([dst]), _param_modules([src])):
        for (w, _), (w2, _) in zip(a._params, b._params):
            ta, tb = getattr(a, w, None), getattr(b, w2, None)
            if ta is not None and tb is not None:
                ta.data.copy_(tb.reshape(ta.shape))


# ---------------------------------------------------------------------------------------------- cells
class Cell(Container):
    """Abstract recurrent cell: ``step(x_t, hidden) -> (output_t, new_hidden)``.

    ``x_t`` is this step's slice of the preTopology output (or of the raw input when the cell has none).
    Standalone use follows the reference protocol: ``forward(T(input, hidden)) -> T(output, hidden)`` where
    ``hidden`` is a Tensor for one-state cells and a Table for LSTM-like cells.
    """

    def __init__(self, hiddensShape, regularizers=None):
        super().__init__()
        self.hiddensShape = list(hiddensShape)
        self.preTopology = None
        self.regularizers = regularizers

    def _set_pre(self, m):
        self.preTopology = m
        if m is not None:
            self.modules.insert(0, m)

    def hiddenSizeOfPreTopo(self):
        return self.hiddensShape[0]

    def step_modules(self):
        return [m for m in self.modules if m is not self.preTopology]

    def init_hidden(self, B, x_t):
        return [ops.zeros(B, h, device=x_t.device, dtype=torch.float32) for h in self.hiddensShape]

    def pre_fn(self, x):
        """Differentiable preTopology (used when the projection cannot be hoisted out of the time loop)."""
        p = self.preTopology
        if p is None:
            return x
        if isinstance(p, Linear):
            return _linear(x, p.weight, p.bias)
        raise ValueError(f"unsupported preTopology {type(p).__name__}")

    def step(self, x, hid):
        raise NotImplementedError

    def bf16_sequence_ok(self, x2, mask=None):
        """True when ``sequence`` takes the bf16 gate inputs as they come from the projection GEMM (GPU)."""
        return False

    def sequence(self, x2, hid, mask=None):
        """Run ``step`` over the time dimension of x2 [B, T, ...]; returns (out [B, T, ...], last hidden)."""
        outs = []
        for t in range(x2.shape[1]):
            o, nh = self.step(x2[:, t], hid)
            if mask is not None:
                m = mask[:, t]
                nh = [torch.where(m.view((-1,) + (1,) * (a.dim() - 1)), a, b) for a, b in zip(nh, hid)]
                o = o * m.view((-1,) + (1,) * (o.dim() - 1)).to(o.dtype)
            outs.append(o)
            hid = nh
        return torch.stack(outs, 1), hid

    # standalone cell (T(input, hidden) -> T(output, hidden))
    def updateOutput(self, input):
        x, h = input[1], input[2]
        xl = _f32(x.detach()).requires_grad_(True)
        hl = [t.detach().float().requires_grad_(True) for t in _activity_to_hidden(h)]
        with _Leaves(self.modules) as L, torch.enable_grad():
            o, nh = self.step(self.pre_fn(xl), hl)
        self._ag = (xl, hl, L, o, nh)
        return Table(o.detach(), _hidden_to_activity([t.detach() for t in nh]))

    def updateGradInput(self, input, gradOutput):
        xl, hl, L, o, nh = self._ag
        outs, gouts = [o], [_f32(gradOutput[1])]
        gh = gradOutput[2] if len(gradOutput) >= 2 else None
        if gh is not None:
            for t, g in zip(nh, _activity_to_hidden(gh)):
                outs.append(t)
                gouts.append(_f32(g))
        grads = torch.autograd.grad(outs, [xl] + hl + L.leaves, gouts, allow_unused=True, retain_graph=True)
        gx = grads[0] if grads[0] is not None else torch.zeros_like(xl)
        ghs = [g if g is not None else torch.zeros_like(t) for g, t in zip(grads[1:1 + len(hl)], hl)]
        self._pending = grads[1 + len(hl):]
        return Table(gx.to(input[1].dtype), _hidden_to_activity(ghs))

    def accGradParameters(self, input, gradOutput):
        pending = getattr(self, "_pending", None)
        if pending is not None:
            self._ag[2].accumulate(pending)
            self._pending = None

    def _set_children(self, children):
        src = Container(*children)
        _copy_module_state(self, src)


class RnnCell(Cell):
    """h_t = activation(W x_t + b + U h_{t-1} + b_U) (S/nn/RNN.scala:49)."""

    def __init__(self, inputSize=4, hiddenSize=3, activation=None, isInputWithBias=True, isHiddenWithBias=True,
                 wRegularizer=None, uRegularizer=None, bRegularizer=None):
        super().__init__([hiddenSize], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.hiddenSize = inputSize, hiddenSize
        self.activation = activation if activation is not None else Tanh()
        self._set_pre(Linear(inputSize, hiddenSize, withBias=isInputWithBias, wRegularizer=wRegularizer,
                             bRegularizer=bRegularizer))
        self.h2h = Linear(hiddenSize, hiddenSize, withBias=isHiddenWithBias, wRegularizer=uRegularizer)
        self.modules.append(self.h2h)

    def step(self, x, hid):
        h = _act(self.activation)(x + _linear(hid[0], self.h2h.weight, self.h2h.bias))
        return h, [h]


def _f32(t):
    """fp32 view of an activation / gradient: bf16 GPU tensors go through the native cast kernel."""
    if t.is_cuda and t.dtype == torch.bfloat16:
        return ops.to_f32(t)
    return t.float()


def _rnn_param_grads(dg16, h16, U, WT16):
    """Native MFMA GEMMs closing a fused recurrent backward sweep (no library GEMM):
    dU = sum_t dg_t^T h_{t-1} over all T*B rows (the conv weight-gradient kernel on a 1x1 'image' of T*B pixels:
    split-K over rows, fp32 accumulation) and dh0 = dg_0 . U (the conv forward kernel, 1x1)."""
    from ..ops import conv as cv

    T, B, G = dg16.shape
    H = U.shape[1]
    dU = torch.zeros(G, H, 1, 1, device=dg16.device)
    cv.conv2d_wgrad(dg16.view(T * B, G, 1, 1), h16[:T].view(T * B, H, 1, 1), dU, None, (1, 1), (0, 0))
    dh0 = cv.conv2d_fwd(dg16[0].view(B, G, 1, 1), WT16.view(H, G, 1, 1), None, (1, 1), (0, 0))
    return _f32(dh0.view(B, H)), dU.view(G, H)


# The whole-sequence backward may add dU straight into the recurrent Linear's gradWeight (no dU buffer, no extra
# add). That is only the updateGradInput + accGradParameters pair that Recurrent.backward runs back to back: a bare
# updateGradInput (input gradients only, or called twice) must leave gradWeight alone, so the sink is armed only
# inside Recurrent.backward, and the buffer is looked up when the backward runs (not the one seen at forward time).
_SINK_ARMED = [0]


def _live_sink(m):
    if m is None or not _SINK_ARMED[0]:
        return None
    g = getattr(m, "gradWeight", None)
    if (m._frozen or getattr(m, "scaleW", 1.0) != 1.0 or g is None or not g.is_cuda or g.dtype != torch.float32
            or not g.is_contiguous()):
        return None
    return g


# BIGDL_RNN_WGRAD_BLAS=0 keeps the whole-sequence LSTM's recurrent weight gradient on the in-tree kernel (A/B)
_RWG_BLAS = [os.environ.get("BIGDL_RNN_WGRAD_BLAS", "1") != "0"]


def _recurrent_wgrad_blas(rows, H, n=None):
    """The recurrent weight gradients of the whole-sequence LSTM / GRU (dU = dg^T h, [n x H] over all T * B rows;
    n = 4H for the LSTM) on hipBLASLt: the Linear route's shape rule (nn/linear.py _blas_shape), not in
    deterministic mode. LSTM LM 11.81 -> 11.46 ms/iteration."""
    from . import linear

    n = 4 * H if n is None else n
    return _RWG_BLAS[0] and linear._blas_shape(rows, H, n) and not ops.native.deterministic()


class _LSTMSeq(torch.autograd.Function):
    """Whole-sequence LSTM (gate order i, g, f, o) with the fused HIP cell kernels on the GPU engine."""

    @staticmethod
    def _cell_fwd(g, c_prev, c, h, act):
        if g.is_cuda:
            ops.native.get().lstm_cell_fwd(g, c_prev, c, h, act)
            return
        H = c.shape[1]
        i, gg, f, o = (torch.sigmoid(g[:, :H]), torch.tanh(g[:, H:2 * H]), torch.sigmoid(g[:, 2 * H:3 * H]),
                       torch.sigmoid(g[:, 3 * H:]))
        c.copy_(f * c_prev + i * gg)
        h.copy_(o * torch.tanh(c))
        act.copy_(torch.cat([i, gg, f, o], 1))

    @staticmethod
    def _cell_bwd(act, c_prev, c, dh, dc_next, dg, dc_prev):
        if act.is_cuda:
            ops.native.get().lstm_cell_bwd(act, c_prev, c, dh, dc_next, dg, dc_prev)
            return
        H = c.shape[1]
        i, gg, f, o = act[:, :H], act[:, H:2 * H], act[:, 2 * H:3 * H], act[:, 3 * H:]
        tc = torch.tanh(c)
        dc = dh * o * (1 - tc * tc) + dc_next
        dg.copy_(torch.cat([dc * gg * i * (1 - i), dc * i * (1 - gg * gg), dc * c_prev * f * (1 - f),
                            dh * tc * o * (1 - o)], 1))
        dc_prev.copy_(dc * f)

    @staticmethod
    def _fused_gpu(xg, U):
        if not (xg.is_cuda and U.shape[1] % 32 == 0):
            return False
        if xg.dtype == torch.bfloat16:     # bf16 gate inputs: whole-sequence kernels only (Recurrent checks first)
            return bool(ops.native.get().lstm_seq_supported(xg.shape[0], U.shape[1]))
        return xg.dtype == torch.float32

    @staticmethod
    def forward(ctx, xg, h0, c0, U, gsink=None):
        ctx.set_materialize_grads(False)   # unused outputs (final h / c) get None, not a zero-filled aten tensor
        # gsink: the module's fp32 gradWeight buffer (Recurrent training, scale 1): the whole-sequence backward then
        # accumulates dU straight into it with the weight-gradient kernel (+=) and returns no U gradient — no zeroed
        # temporary and no separate add into gradWeight afterwards
        ctx.gmod = gsink
        B, T, G = xg.shape
        H = G // 4
        if xg.dtype != torch.float32 and not _LSTMSeq._fused_gpu(xg, U):
            xg = _f32(xg)                   # bf16 inputs outside the whole-sequence kernels' shapes
        if _LSTMSeq._fused_gpu(xg, U):
            # one fused launch per step (csrc/lstm.hip): bf16 MFMA recurrent GEMM + cell in its epilogue
            C = ops.native.get()
            W16 = ops.to_bf16(U.detach())
            out = xg.new_empty(B, T, H)
            cs = xg.new_empty(T, B, H, dtype=torch.float32)
            acts = xg.new_empty(T, B, G, dtype=torch.float32)
            # time-major bf16 states h_{-1..T-1}: step t's GEMM operand, and (rows t*B + b) the B operand of the
            # weight-gradient GEMM after the backward sweep
            h16 = xg.new_empty(T + 1, B, H, dtype=torch.bfloat16)
            C.cast_f32_bf16(h0.contiguous(), h16[0])
            ctx.seq = bool(C.lstm_seq_supported(B, H))
            if ctx.seq:
                ops.native.check_persistent()      # an earlier launch's timeout surfaces before more work is queued
                # whole sequence in ONE persistent launch (csrc/lstm_seq.hip): W resident in VGPRs, per-step
                # state exchange inside each XCD's batch group; bf16 xg -> bf16 out (the projections' dtype)
                sync = torch.empty(C.lstm_seq_sync_words(), dtype=torch.int32, device=xg.device)
                out = xg.new_empty(B, T, H)
                hT = xg.new_empty(B, H, dtype=torch.float32)
                C.lstm_seq_fwd(W16, xg, c0.contiguous(), h16, out, hT, cs, acts, sync)
                ctx.save_for_backward(h0, c0, U, out, cs, acts, h16, W16)
                ctx.fused = True
                return out, hT, cs[T - 1]          # a view of the saved states: no device copy
            else:
                c_prev = c0.contiguous()
                for t in range(T):
                    C.lstm_fwd_step(W16, h16[t], xg[:, t], c_prev, cs[t], out[:, t], h16[t + 1], acts[t])
                    c_prev = cs[t]
            ctx.save_for_backward(h0, c0, U, out, cs, acts, h16, W16)
            ctx.fused = True
            return out, out[:, -1].clone(), cs[-1].clone()
        hs = xg.new_empty(T, B, H)
        cs = xg.new_empty(T, B, H)
        acts = xg.new_empty(T, B, G)
        Ut = U.t()
        h, c = h0.contiguous(), c0.contiguous()
        for t in range(T):
            g = torch.addmm(xg[:, t], h, Ut)
            _LSTMSeq._cell_fwd(g, c, cs[t], hs[t], acts[t])
            h, c = hs[t], cs[t]
        ctx.save_for_backward(h0, c0, U, hs, cs, acts)
        ctx.fused = False
        return hs.transpose(0, 1).contiguous(), hs[-1].clone(), cs[-1].clone()

    @staticmethod
    def _backward_fused(ctx, dout, dhT, dcT):
        from ..ops import conv as cv

        h0, c0, U, out, cs, acts, h16, W16 = ctx.saved_tensors
        B, T, H = out.shape
        C = ops.native.get()
        dout = dout.contiguous() if dout is not None else None
        if ctx.seq:
            ops.native.check_persistent()
            # one persistent launch for the whole backward sweep, dh0 = dg_0 U included (no transposed copy of U)
            dxg = out.new_empty(B, T, 4 * H)        # out's dtype: bf16 in, bf16 gradient out
            if dout is not None and dout.dtype != out.dtype:
                dout = dout.to(out.dtype)
            dg16 = out.new_empty(T, B, 4 * H, dtype=torch.bfloat16)
            dc0 = out.new_empty(B, H, dtype=torch.float32)
            dh0 = out.new_empty(B, H, dtype=torch.float32)
            sync = torch.empty(C.lstm_seq_sync_words(), dtype=torch.int32, device=out.device)
            C.lstm_seq_bwd(W16, dout, dhT.contiguous() if dhT is not None else None,
                           dcT.contiguous() if dcT is not None else None, acts, cs, c0.contiguous(), dg16, dxg, dc0,
                           dh0, sync)
            sink = _live_sink(ctx.gmod)
            if _recurrent_wgrad_blas(T * B, H):
                # dU (+)= dg^T h over all T * B rows on hipBLASLt, accumulated in place (beta = 1) into the fp32
                # gradient: the [4H x H x T*B] GEMM is the shape the Linear route measured fastest there
                # (profiles/r6_lm_gemm_vs_hipblaslt.log: 532 -> 355 us)
                a, b = dg16.view(T * B, 4 * H).t(), h16[:T].view(T * B, H)
                if sink is not None and sink.is_contiguous():
                    torch.addmm(sink, a, b, out_dtype=torch.float32, out=sink)
                    return dxg, dh0, dc0, None, None
                return dxg, dh0, dc0, torch.mm(a, b, out_dtype=torch.float32), None
            if sink is not None:
                dU = sink.view(4 * H, H, 1, 1)
            else:
                dU = out.new_empty(4 * H, H, 1, 1, dtype=torch.float32)
                C.fill_bytes(dU, 0)
            cv.conv2d_wgrad(dg16.view(T * B, 4 * H, 1, 1), h16[:T].view(T * B, H, 1, 1), dU, None, (1, 1), (0, 0))
            return dxg, dh0, dc0, (None if sink is not None else dU.view(4 * H, H)), None
        WT16 = cv.transpose_w(W16.view(4 * H, H, 1, 1)).view(H, 4 * H)
        dxg = out.new_empty(B, T, 4 * H)
        dg16 = out.new_empty(T, B, 4 * H, dtype=torch.bfloat16)      # time-major: rows t*B + b
        dc = dcT.contiguous().clone() if dcT is not None else out.new_zeros(B, H)
        dhT = dhT.contiguous() if dhT is not None else None
        c0 = c0.contiguous()
        for t in range(T - 1, -1, -1):
            C.lstm_bwd_step(WT16, dg16[t + 1] if t < T - 1 else None,
                            dout[:, t] if dout is not None else None, dhT if t == T - 1 else None, acts[t],
                            cs[t - 1] if t > 0 else c0, cs[t], dc, dxg[:, t], dg16[t])
        dh0, dU = _rnn_param_grads(dg16, h16, U, WT16)
        sink = _live_sink(ctx.gmod)
        if sink is not None:
            sink.add_(dU)
            dU = None
        return dxg, dh0, dc, dU, None

    @staticmethod
    def backward(ctx, dout, dhT, dcT):
        if ctx.fused:
            return _LSTMSeq._backward_fused(ctx, dout, dhT, dcT)
        h0, c0, U, hs, cs, acts = ctx.saved_tensors
        T, B, H = hs.shape
        dgs = acts.new_empty(T, B, 4 * H)
        dh_next = dhT.contiguous() if dhT is not None else hs.new_zeros(B, H)
        dc_next = dcT.contiguous() if dcT is not None else hs.new_zeros(B, H)
        dc_prev = hs.new_empty(B, H)
        c0 = c0.contiguous()
        for t in range(T - 1, -1, -1):
            dh = dh_next + dout[:, t] if dout is not None else dh_next
            c_prev = cs[t - 1] if t > 0 else c0
            _LSTMSeq._cell_bwd(acts[t], c_prev, cs[t], dh.contiguous(), dc_next, dgs[t], dc_prev)
            dh_next = dgs[t] @ U
            dc_next, dc_prev = dc_prev, dc_next
        hprev = torch.cat([h0.unsqueeze(0), hs[:-1]], 0).reshape(T * B, H)
        dU = dgs.reshape(T * B, 4 * H).t() @ hprev
        sink = _live_sink(ctx.gmod)
        if sink is not None:
            sink.add_(dU)
            dU = None
        return dgs.transpose(0, 1), dh_next, dc_next, dU, None


class _GRUSeq(torch.autograd.Function):
    """Whole-sequence GRU (preTopology order r, z, n). Where the persistent kernels apply (B <= 128 per GPU,
    H in {256, 512, 1024}: csrc/lstm_seq.hip gru_seq_*_kernel) the whole sequence is ONE launch per direction (the
    reference's fused VanillaGru RNN primitive, S/nn/mkldnn/RNN.scala:213-219); otherwise the fused HIP step kernels
    (csrc/gru.hip: two MFMA launches per step and direction). Then the recurrent weight gradients as two native
    GEMMs over all T*B rows."""

    @staticmethod
    def usable(x, H):
        return x.is_cuda and H % 32 == 0 and x.dtype == torch.float32

    @staticmethod
    def forward(ctx, xg, h0, Urz, Un):
        ctx.set_materialize_grads(False)
        B, T, G = xg.shape
        H = G // 3
        C = ops.native.get()
        bf = torch.bfloat16
        Wrz, Wn = Urz.detach().to(bf).contiguous(), Un.detach().to(bf).contiguous()
        ctx.seq = bool(C.gru_seq_supported(B, H))
        if ctx.seq:
            # whole sequence in ONE persistent launch (csrc/lstm_seq.hip gru_seq_fwd_kernel): both recurrent weight
            # blocks resident in VGPRs, two group hand-offs per step (r * h, then h)
            ops.native.check_persistent()
            out = xg.new_empty(B, T, H)
            gates = xg.new_empty(3, T, B, H)
            h16 = xg.new_empty(T + 1, B, H, dtype=bf)
            rh16 = xg.new_empty(T, B, H, dtype=bf)
            h0 = h0.contiguous()
            C.cast_f32_bf16(h0, h16[0])
            sync = torch.empty(C.lstm_seq_sync_words(), dtype=torch.int32, device=xg.device)
            C.gru_seq_fwd(Wrz, Wn, xg, h0, h16, rh16, gates, out, sync)
            ctx.save_for_backward(h0, Urz, Un, out, gates, h16, rh16)
            ctx.w16 = (Wrz, Wn)
            return out, out[:, -1].clone()
        out = xg.new_empty(B, T, H)
        gates = xg.new_empty(3, T, B, H)                 # r, z, n per step
        h16 = xg.new_empty(T + 1, B, H, dtype=bf)         # h_{t-1} operands, time-major
        rh16 = xg.new_empty(T, B, H, dtype=bf)            # (r * h_{t-1}) operands, time-major
        h16[0].copy_(h0)
        h0 = h0.contiguous()
        for t in range(T):
            hp = h0 if t == 0 else out[:, t - 1]
            C.gru_step(0, h16[t], Wrz, B, H, xg=xg[:, t], hprev=hp, r=gates[0, t], z=gates[1, t], rh16=rh16[t])
            C.gru_step(1, rh16[t], Wn, B, H, xg=xg[:, t], hprev=hp, z=gates[1, t], n=gates[2, t], hout=out[:, t],
                       h16out=h16[t + 1])
        ctx.save_for_backward(h0, Urz, Un, out, gates, h16, rh16)
        return out, out[:, -1].clone()

    @staticmethod
    def backward(ctx, dout, dhT):
        from ..ops import conv as cv

        h0, Urz, Un, out, gates, h16, rh16 = ctx.saved_tensors
        B, T, H = out.shape
        C = ops.native.get()
        bf = torch.bfloat16
        if ctx.seq:
            ops.native.check_persistent()
            Wrz, Wn = ctx.w16
            dx = out.new_empty(B, T, 3 * H)
            dn16 = out.new_empty(T, B, H, dtype=bf)
            drz16 = out.new_empty(T, B, 2 * H, dtype=bf)
            dh0 = out.new_empty(B, H)
            sync = torch.empty(C.lstm_seq_sync_words(), dtype=torch.int32, device=out.device)
            C.gru_seq_bwd(Wrz, Wn, h0, gates, out, dout.contiguous() if dout is not None else None,
                          dhT.contiguous() if dhT is not None else None, dx, dn16, drz16, dh0, sync)
            def wgrad(g16, x16, n):        # [n, H] = g^T x over all T * B rows (hipBLASLt where the LSTM's rule says)
                if _recurrent_wgrad_blas(T * B, H, n):
                    return torch.mm(g16.view(T * B, n).t(), x16.view(T * B, H), out_dtype=torch.float32)
                d = out.new_empty(n, H, 1, 1)
                C.fill_bytes(d, 0)
                cv.conv2d_wgrad(g16.view(T * B, n, 1, 1), x16.view(T * B, H, 1, 1), d, None, (1, 1), (0, 0))
                return d.view(n, H)

            return dx, dh0, wgrad(drz16, h16[:T], 2 * H), wgrad(dn16, rh16, H)
        UrzT = Urz.detach().t().contiguous().to(bf)       # [H, 2H]: D = drz . U_rz
        UnT = Un.detach().t().contiguous().to(bf)         # [H, H]:  D = dn . U_n
        dout = dout.contiguous() if dout is not None else None
        dx = out.new_empty(B, T, 3 * H)
        dn16 = out.new_empty(T, B, H, dtype=bf)
        drz16 = out.new_empty(T, B, 2 * H, dtype=bf)
        dhp = dhT.contiguous().clone() if dhT is not None else out.new_zeros(B, H)
        for t in range(T - 1, -1, -1):
            hp = h0 if t == 0 else out[:, t - 1]
            C.gru_step(2, drz16[t + 1] if t < T - 1 else None, UrzT, B, H, hprev=hp, z=gates[1, t], n=gates[2, t],
                       dout=dout[:, t] if dout is not None else None, dhp=dhp, dx=dx[:, t], dn16=dn16[t],
                       drz16=drz16[t])
            C.gru_step(3, dn16[t], UnT, B, H, hprev=hp, r=gates[0, t], dhp=dhp, dx=dx[:, t], drz16=drz16[t])
        dh0 = out.new_empty(B, H)
        C.gru_step(4, drz16[0], UrzT, B, H, dhp=dhp, dh0=dh0)
        dUrz = torch.zeros(2 * H, H, 1, 1, device=out.device)
        cv.conv2d_wgrad(drz16.view(T * B, 2 * H, 1, 1), h16[:T].view(T * B, H, 1, 1), dUrz, None, (1, 1), (0, 0))
        dUn = torch.zeros(H, H, 1, 1, device=out.device)
        cv.conv2d_wgrad(dn16.view(T * B, H, 1, 1), rh16.view(T * B, H, 1, 1), dUn, None, (1, 1), (0, 0))
        return dx, dh0, dUrz.view(2 * H, H), dUn.view(H, H)


def _ceil(v, m):
    return (v + m - 1) // m * m


class _LSTMDropSeq(torch.autograd.Function):
    """LSTM with dropout p != 0 on the GPU, the reference's per-gate Dropout + Linear branches
    (S/nn/LSTM.scala:68-96) as native kernels (csrc/lstm_drop.hip): gate g of step t reads x_t and h_{t-1} through
    their own Philox masks (regenerated, never stored). The input side is ONE batched gate GEMM over all T * B rows
    (four masked copies of x, biases folded in as a ones column); per step: mask h_{t-1} (one launch), the four
    recurrent GEMMs accumulating into that step's gate pre-activations (bmm_nt on a [4][B][H] view of [B][4H]), the
    fused cell. Backward mirrors it; weight gradients are one NT GEMM per gate over the whole sequence."""

    @staticmethod
    def usable(x, H, I):
        return x.is_cuda and x.dim() == 3 and H % 32 == 0 and I % 4 == 0 and x.dtype == torch.float32

    @staticmethod
    def forward(ctx, x, h0, c0, Wi, bi, U, bu, p):
        from ..ops import nnk

        C = ops.native.get()
        B, T, I = x.shape
        H = U.shape[1]
        R, Ip = T * B, _ceil(I + 1, 32)
        keep = 1.0 - p
        mul = 1.0 / keep
        sx, sh = nnk.next_seed(), nnk.next_seed()
        dev = x.device
        x = x.contiguous()
        Wi4 = torch.empty(4, H, Ip, dtype=torch.bfloat16, device=dev)
        C.lstm_pack_gate_w(Wi.detach().contiguous(), bi, bu, H, I, Ip, Wi4, None)
        U4 = torch.empty(4, H, H, dtype=torch.bfloat16, device=dev)
        C.lstm_pack_gate_w(U.detach().contiguous(), None, None, H, H, H, U4, None)
        xm = torch.empty(4, R, Ip, dtype=torch.bfloat16, device=dev)
        C.lstm_drop_rep(x, T * I, I, xm, R * Ip, B, T, I, Ip, True, p, mul, sx, 0)
        G = torch.empty(T, B, 4 * H, dtype=torch.float32, device=dev)      # gate pre-activations, time-major
        C.bmm_nt(xm, Wi4, G.view(R, 4, H).permute(1, 0, 2), 1.0, False)
        hm = torch.empty(4, T, B, H, dtype=torch.bfloat16, device=dev)    # masked h_{t-1} per gate (dU operand)
        cs = torch.empty(T, B, H, dtype=torch.float32, device=dev)
        hs = torch.empty(T, B, H, dtype=torch.float32, device=dev)
        acts = torch.empty(T, B, 4 * H, dtype=torch.float32, device=dev)
        h_prev, c_prev = h0.detach().contiguous(), c0.detach().contiguous()
        for t in range(T):
            C.lstm_drop_rep(h_prev, H, 0, hm[:, t], T * B * H, B, 1, H, H, False, p, mul, sh, t * 4 * B * H)
            C.bmm_nt(hm[:, t], U4, G[t].view(B, 4, H).permute(1, 0, 2), 1.0, True)
            C.lstm_cell_fwd(G[t], c_prev, cs[t], hs[t], acts[t])
            h_prev, c_prev = hs[t], cs[t]
        ctx.save_for_backward(c0, Wi, U, xm, hm, cs, acts)
        ctx.cfg = (p, mul, sx, sh, B, T, I, H)
        ctx.set_materialize_grads(False)
        return hs.transpose(0, 1).contiguous(), hs[T - 1], cs[T - 1]

    @staticmethod
    def backward(ctx, dout, dhT, dcT):
        C = ops.native.get()
        c0, Wi, U, xm, hm, cs, acts = ctx.saved_tensors
        p, mul, sx, sh, B, T, I, H = ctx.cfg
        R, Ip = T * B, xm.shape[2]
        dev = xm.device
        dout = dout.float().contiguous() if dout is not None else None
        UT4 = torch.empty(4, H, H, dtype=torch.bfloat16, device=dev)
        C.lstm_pack_gate_w(U.detach().contiguous(), None, None, H, H, H, None, UT4)
        dG = torch.empty(T, B, 4 * H, dtype=torch.float32, device=dev)
        dG16 = torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev)
        dhm = torch.empty(4, B, H, dtype=torch.float32, device=dev)
        dc = dcT.float().contiguous().clone() if dcT is not None else ops.zeros(B, H, device=dev)
        if dout is not None and dhT is not None:
            dh = dout[:, T - 1] + dhT.float()
        elif dout is not None:
            dh = dout[:, T - 1].contiguous()
        elif dhT is not None:
            dh = dhT.float().contiguous().clone()
        else:
            dh = ops.zeros(B, H, device=dev)
        dh0 = torch.empty(B, H, dtype=torch.float32, device=dev)
        dhb = torch.empty(B, H, dtype=torch.float32, device=dev)     # dh of steps T-2 .. 0 (stream-ordered reuse)
        c0 = c0.detach().contiguous()
        for t in range(T - 1, -1, -1):
            C.lstm_cell_bwd(acts[t], cs[t - 1] if t > 0 else c0, cs[t], dh, dc, dG[t], dc)
            C.cast_f32_bf16(dG[t], dG16[t])
            C.bmm_nt(dG16[t].view(B, 4, H).permute(1, 0, 2), UT4, dhm, 1.0, False)
            if t > 0:     # dh_{t-1} = dout_{t-1} + sum_g (dG_g U_g) * mask_h(g, t)
                C.lstm_drop_rep_bwd(dhm, B * H, H, dhb, H, 0, dout[:, t - 1] if dout is not None else None, T * H, 0,
                                    B, 1, H, p, mul, sh, t * 4 * B * H)
                dh = dhb
            else:
                C.lstm_drop_rep_bwd(dhm, B * H, H, dh0, H, 0, None, 0, 0, B, 1, H, p, mul, sh, 0)
        # weight / bias gradients: one NT GEMM per gate over all T * B rows (dbu = column sums of dG_g)
        dU = ops.zeros(4 * H, H, device=dev)
        dbu = ops.zeros(4 * H, device=dev)
        dWi4 = ops.zeros(4, H, Ip, device=dev)
        flat = dG16.view(-1)
        for g in range(4):
            C.conv_wgrad(flat[g * H:], hm[g], dU[g * H:(g + 1) * H], dbu[g * H:(g + 1) * H],
                         [R, 1, 1, H, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, R, H, H, 4 * H])
            C.conv_wgrad(flat[g * H:], xm[g], dWi4[g], None, [R, 1, 1, Ip, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, R, H, Ip, 4 * H])
        dWi = dWi4[:, :, :I].reshape(4 * H, I)
        dbi = dWi4[:, :, I].reshape(4 * H)
        # input gradient: dxm_g = dG_g Wi_g, summed back through the input masks into [B][T][I]
        WiT4 = torch.empty(4, I, H, dtype=torch.bfloat16, device=dev)
        C.lstm_pack_gate_w(Wi.detach().contiguous(), None, None, H, I, I, None, WiT4)
        dxm = torch.empty(4, R, I, dtype=torch.float32, device=dev)
        C.bmm_nt(dG16.view(R, 4, H).permute(1, 0, 2), WiT4, dxm, 1.0, False)
        dx = torch.empty(B, T, I, dtype=torch.float32, device=dev)
        C.lstm_drop_rep_bwd(dxm, R * I, I, dx, T * I, I, None, 0, 0, B, T, I, p, mul, sx, 0)
        return dx, dh0, dc, dWi, dbi, dU, dbu, None


class LSTM(Cell):
    """Long short-term memory cell (S/nn/LSTM.scala:46). Hidden = T(h, c); gate order (i, g, f, o)."""

    def __init__(self, inputSize, hiddenSize, p=0.0, activation=None, innerActivation=None, wRegularizer=None,
                 uRegularizer=None, bRegularizer=None):
        super().__init__([hiddenSize, hiddenSize], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.hiddenSize, self.p = inputSize, hiddenSize, p
        self.activation = activation if activation is not None else Tanh()
        self.innerActivation = innerActivation if innerActivation is not None else Sigmoid()
        if p != 0:
            # the reference's dropout topology (LSTM.scala:76-129): no preTopology; every step, gate g reads
            # Dropout(p)(x_t) through its own input Linear and Dropout(p)(h_{t-1}) through its own hidden Linear
            # (with bias, wRegularizer / bRegularizer). The four per-gate Linears of each side are stored stacked
            # as one [4H, .] Linear (gate order i, g, f, o)
            self.i2g = Linear(inputSize, 4 * hiddenSize, wRegularizer=wRegularizer, bRegularizer=bRegularizer)
            self.modules.append(self.i2g)
            self.h2g = Linear(hiddenSize, 4 * hiddenSize, wRegularizer=wRegularizer, bRegularizer=bRegularizer)
        else:
            self._set_pre(Linear(inputSize, 4 * hiddenSize, wRegularizer=wRegularizer, bRegularizer=bRegularizer))
            self.h2g = Linear(hiddenSize, 4 * hiddenSize, withBias=False, wRegularizer=uRegularizer)
        self.modules.append(self.h2g)

    def hiddenSizeOfPreTopo(self):
        return 4 * self.hiddenSize

    def _fused_ok(self):
        return self.p == 0 and _is(self.activation, Tanh) and _is(self.innerActivation, Sigmoid)

    def _gate_inputs(self, x, h):
        """Gate pre-activations [B, 4H]. p != 0 (x is the raw input then): four independent dropout masks per side,
        one per gate block, in training (LSTM.scala:68-96); the plain affine maps otherwise."""
        H = self.hiddenSize
        if self.p == 0:
            return x + _linear(h, self.h2g.weight, self.h2g.bias)
        Wi, U = self.i2g.weight, self.h2g.weight
        if not self.train:
            return _linear(x, Wi, self.i2g.bias) + _linear(h, U, self.h2g.bias)
        keep = 1.0 - self.p

        def gated(v, W):
            m = torch.stack([torch.bernoulli(torch.full_like(v, keep)) / keep for _ in range(4)])
            out = torch.bmm(v.unsqueeze(0) * m, W.view(4, H, -1).transpose(1, 2))      # [4, B, H]
            return out.permute(1, 0, 2).reshape(v.shape[0], 4 * H)

        return gated(x, Wi) + self.i2g.bias + gated(h, U) + self.h2g.bias

    def step(self, x, hid):
        h, c = hid
        H = self.hiddenSize
        g = self._gate_inputs(x, h)
        sig, tanh = _act(self.innerActivation), _act(self.activation)
        i, gg, f, o = sig(g[:, :H]), tanh(g[:, H:2 * H]), sig(g[:, 2 * H:3 * H]), sig(g[:, 3 * H:])
        c2 = f * c + i * gg
        h2 = o * tanh(c2)
        return h2, [h2, c2]

    def bf16_sequence_ok(self, x2, mask=None):
        return (mask is None and self._fused_ok() and x2.is_cuda and x2.dim() == 3
                and bool(ops.native.get().lstm_seq_supported(x2.shape[0], self.hiddenSize)))

    def _grad_sink(self, m):
        """m when a fused backward may accumulate into m.gradWeight directly (see _LSTMSeq.forward and _live_sink)."""
        return m if self.train else None

    def sequence(self, x2, hid, mask=None):
        if mask is None and self._fused_ok():
            out, h, c = _LSTMSeq.apply(x2.contiguous(), hid[0], hid[1], self.h2g.weight, self._grad_sink(self.h2g))
            return out, [h, c]
        default_act = _is(self.activation, Tanh) and _is(self.innerActivation, Sigmoid)
        if self.p != 0 and mask is None and default_act:
            if self.train and _LSTMDropSeq.usable(x2, self.hiddenSize, self.inputSize):
                out, h, c = _LSTMDropSeq.apply(x2, hid[0], hid[1], self.i2g.weight, self.i2g.bias, self.h2g.weight,
                                               self.h2g.bias, float(self.p))
                return out, [h, c]
            if not self.train and x2.is_cuda:
                # evaluation: dropout is the identity -> one input GEMM with both biases, then the fused recurrence
                B, T = x2.shape[:2]
                xg = _linear(x2.reshape(B * T, -1), self.i2g.weight, self.i2g.bias + self.h2g.bias)
                out, h, c = _LSTMSeq.apply(xg.reshape(B, T, -1).contiguous(), hid[0], hid[1], self.h2g.weight)
                return out, [h, c]
        return super().sequence(x2, hid, mask)


class LSTMPeephole(Cell):
    """LSTM with peephole connections (S/nn/LSTMPeephole.scala). preTopology order (i, f, g, o)."""

    def __init__(self, inputSize, hiddenSize, p=0.0, wRegularizer=None, uRegularizer=None, bRegularizer=None):
        super().__init__([hiddenSize, hiddenSize], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.hiddenSize, self.p = inputSize, hiddenSize, p
        self._set_pre(Linear(inputSize, 4 * hiddenSize, wRegularizer=wRegularizer, bRegularizer=bRegularizer))
        self.h2g = Linear(hiddenSize, 4 * hiddenSize, withBias=False, wRegularizer=uRegularizer)
        self.peepI, self.peepF, self.peepO = CMul([hiddenSize]), CMul([hiddenSize]), CMul([hiddenSize])
        self.modules += [self.h2g, self.peepI, self.peepF, self.peepO]

    def hiddenSizeOfPreTopo(self):
        return 4 * self.hiddenSize

    def step(self, x, hid):
        h, c = hid
        H = self.hiddenSize
        g = x + _linear(h, self.h2g.weight)
        i = torch.sigmoid(g[:, :H] + self.peepI.weight * c)
        f = torch.sigmoid(g[:, H:2 * H] + self.peepF.weight * c)
        gg = torch.tanh(g[:, 2 * H:3 * H])
        c2 = f * c + i * gg
        o = torch.sigmoid(g[:, 3 * H:] + self.peepO.weight * c2)
        h2 = o * torch.tanh(c2)
        return h2, [h2, c2]


class GRU(Cell):
    """Gated recurrent unit (S/nn/GRU.scala). preTopology order (r, z, n); h' = (1 - z) * n + z * h."""

    def __init__(self, inputSize, outputSize, p=0.0, activation=None, innerActivation=None, wRegularizer=None,
                 uRegularizer=None, bRegularizer=None):
        super().__init__([outputSize], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.outputSize, self.p = inputSize, outputSize, p
        self.activation = activation if activation is not None else Tanh()
        self.innerActivation = innerActivation if innerActivation is not None else Sigmoid()
        self._set_pre(Linear(inputSize, 3 * outputSize, wRegularizer=wRegularizer, bRegularizer=bRegularizer))
        self.h2g = Linear(outputSize, 2 * outputSize, withBias=False, wRegularizer=uRegularizer)
        self.h2n = Linear(outputSize, outputSize, withBias=False, wRegularizer=uRegularizer)
        self.modules += [self.h2g, self.h2n]

    def hiddenSizeOfPreTopo(self):
        return 3 * self.outputSize

    def _drop(self, t):
        if self.p != 0 and self.train:
            return F.dropout(t, self.p, True)
        return t

    def step(self, x, hid):
        h = hid[0]
        H = self.outputSize
        sig, act = _act(self.innerActivation), _act(self.activation)
        rz = sig(x[:, :2 * H] + _linear(self._drop(h), self.h2g.weight))
        r, z = rz[:, :H], rz[:, H:]
        n = act(x[:, 2 * H:] + _linear(self._drop(r * h), self.h2n.weight))
        h2 = (1 - z) * n + z * h
        return h2, [h2]

    def _fused_ok(self):
        return self.p == 0 and _is(self.activation, Tanh) and _is(self.innerActivation, Sigmoid)

    def sequence(self, x2, hid, mask=None):
        if mask is None and self._fused_ok() and _GRUSeq.usable(x2, self.outputSize):
            out, h = _GRUSeq.apply(x2.contiguous(), hid[0], self.h2g.weight, self.h2n.weight)
            return out, [h]
        return super().sequence(x2, hid, mask)


class _ConvLSTMBase(Cell):
    _nd = 2

    def __init__(self, inputSize, outputSize, kernelI, kernelC, stride=1, padding=-1, activation=None,
                 innerActivation=None, wRegularizer=None, uRegularizer=None, bRegularizer=None, cRegularizer=None,
                 withPeephole=True):
        super().__init__([outputSize, outputSize], [wRegularizer, uRegularizer, bRegularizer, cRegularizer])
        self.inputSize, self.outputSize = inputSize, outputSize
        self.kernelI, self.kernelC, self.stride, self.padding = kernelI, kernelC, stride, padding
        self.withPeephole = withPeephole
        self.activation = activation if activation is not None else Tanh()
        self.innerActivation = innerActivation if innerActivation is not None else Sigmoid()
        if self._nd == 2:
            self.i2g = SpatialConvolution(inputSize, 4 * outputSize, kernelI, kernelI, stride, stride, padding,
                                          padding, wRegularizer=wRegularizer, bRegularizer=bRegularizer)
            self.h2g = SpatialConvolution(outputSize, 4 * outputSize, kernelC, kernelC, stride, stride, padding,
                                          padding, withBias=False, wRegularizer=uRegularizer)
        else:
            self.i2g = VolumetricConvolution(inputSize, 4 * outputSize, kernelI, kernelI, kernelI, stride, stride,
                                             stride, padding, padding, padding, wRegularizer=wRegularizer,
                                             bRegularizer=bRegularizer)
            self.h2g = VolumetricConvolution(outputSize, 4 * outputSize, kernelC, kernelC, kernelC, stride, stride,
                                             stride, padding, padding, padding, withBias=False,
                                             wRegularizer=uRegularizer)
        self.modules += [self.i2g, self.h2g]
        if withPeephole:
            shape = [1, outputSize] + [1] * self._nd
            self.peepI, self.peepF, self.peepO = (CMul(shape, cRegularizer), CMul(shape, cRegularizer),
                                                  CMul(shape, cRegularizer))
            self.modules += [self.peepI, self.peepF, self.peepO]

    def _conv(self, x, conv, k):
        from ..ops import conv_fn

        fn = conv_fn.conv2d if self._nd == 2 else conv_fn.conv3d      # native implicit GEMM on the GPU
        w = conv.weight
        if self.padding == -1:
            pads = []
            for d in range(self._nd - 1, -1, -1):
                pads.extend(_same_pad(x.shape[2 + d], k, self.stride))
            x = F.pad(x, pads)
            pad = 0
        else:
            pad = self.padding
        st = (self.stride,) * self._nd
        return fn(x, w, conv.bias, st, (pad,) * self._nd)

    def init_hidden(self, B, x_t):
        spatial = []
        for d in range(self._nd):
            n = x_t.shape[2 + d]
            if self.padding == -1:
                spatial.append(-(-n // self.stride))
            else:
                spatial.append((n + 2 * self.padding - self.kernelI) // self.stride + 1)
        return [torch.zeros(B, self.outputSize, *spatial, device=x_t.device, dtype=torch.float32)
                for _ in range(2)]

    def step(self, x, hid):
        h, c = hid
        C = self.outputSize
        g = self._conv(x, self.i2g, self.kernelI) + self._conv(h, self.h2g, self.kernelC)
        sig, act = _act(self.innerActivation), _act(self.activation)
        gi, gf, gh, go = g[:, :C], g[:, C:2 * C], g[:, 2 * C:3 * C], g[:, 3 * C:]
        if self.withPeephole:
            gi = gi + self.peepI.weight * c
            gf = gf + self.peepF.weight * c
        c2 = sig(gf) * c + sig(gi) * act(gh)
        if self.withPeephole:
            go = go + self.peepO.weight * c2
        h2 = sig(go) * act(c2)
        return h2, [h2, c2]


class ConvLSTMPeephole(_ConvLSTMBase):
    """Convolutional LSTM with peepholes over [B, T, C, H, W] (S/nn/ConvLSTMPeephole.scala:53)."""
    _nd = 2


class ConvLSTMPeephole3D(_ConvLSTMBase):
    """Volumetric convolutional LSTM over [B, T, C, D, H, W] (S/nn/ConvLSTMPeephole3D.scala)."""
    _nd = 3


class MultiRNNCell(Cell):
    """Stack of cells applied within one time step (S/nn/MultiRNNCell.scala:36). Hidden = concatenation of
    the cells' hidden states (a Table of Tables through get/setHiddenState)."""

    def __init__(self, cells):
        cells = list(cells)
        super().__init__(sum((c.hiddensShape for c in cells), []))
        self.cells = cells
        self.modules = list(cells)

    def hiddenSizeOfPreTopo(self):
        return self.cells[0].inputSize if hasattr(self.cells[0], "inputSize") else None

    def init_hidden(self, B, x_t):
        out = []
        x = x_t
        for c in self.cells:
            hs = c.init_hidden(B, x)
            out.extend(hs)
            x = hs[0]
        return out

    def step(self, x, hid):
        new, off = [], 0
        for c in self.cells:
            n = len(c.hiddensShape)
            o, nh = c.step(c.pre_fn(x), hid[off:off + n])
            new.extend(nh)
            off += n
            x = o
        return x, new

    def _set_children(self, children):
        _copy_module_state(self, Container(*children))


# ---------------------------------------------------------------------------------------------- drivers
class Recurrent(Container):
    """Runs a Cell over [batch, time, ...] input (S/nn/Recurrent.scala:47). Output [batch, time, hidden...]."""

    def __init__(self, batchNormParams=None, maskZero=False, bf16IO=False):
        super().__init__()
        self.batchNormParams = batchNormParams
        self.maskZero = maskZero
        # bf16IO (opt-in, GPU engine): when the whole-sequence kernels apply, take the projection GEMM's bf16 output
        # as is and return bf16 (no f32 round trip of [B, T, 4H] / [B, T, H]). Off by default: the output is fp32 on
        # every path, whatever the batch size or GPU (the reference's LSTM output dtype)
        self.bf16IO = bf16IO
        self.cell = None
        self.bn = None
        self._init_hidden = None
        self._last_hidden = None

    def setBf16IO(self, on=True):
        """Opt in (or out) of bf16 sequence I/O on the GPU whole-sequence path (see __init__)."""
        self.bf16IO = bool(on)
        return self

    def add(self, cell):
        assert isinstance(cell, Cell), "Recurrent.add expects a Cell"
        self.cell = cell
        self.modules = [cell]
        if self.batchNormParams is not None:
            if cell.preTopology is None:
                raise ValueError("batchNormParams need a cell with a preTopology")
            from .normalization import BatchNormalization

            bp = self.batchNormParams
            self.bn = BatchNormalization(cell.hiddenSizeOfPreTopo(), **(bp if isinstance(bp, dict) else {}))
            self.modules.append(self.bn)
        return self

    def getCell(self):
        return self.cell

    def _set_children(self, children):
        self.add(children[0])
        if self.bn is not None and len(children) > 1:
            self.bn = children[1]
            self.modules[1] = children[1]

    def getHiddenState(self):
        if self._last_hidden is None:
            raise RuntimeError("getHiddenState need to be called after updateOutput")
        return _hidden_to_activity(self._last_hidden)

    def setHiddenState(self, hiddenState):
        self._init_hidden = None if hiddenState is None else _activity_to_hidden(hiddenState)

    def _project(self, input):
        cell = self.cell
        B, T = input.shape[:2]
        if cell.preTopology is None:
            return input, None
        flat = input.reshape((B * T,) + tuple(input.shape[2:]))
        x2 = cell.preTopology.forward(flat)
        if self.bn is not None:
            x2 = self.bn.forward(x2)
        return x2.reshape((B, T) + tuple(x2.shape[1:])), flat

    def updateOutput(self, input):
        assert input.dim() in (3, 5, 6), "Recurrent: input should be [batch, times, ...]"
        B = input.shape[0]
        x2, self._flat = self._project(input)
        need_grad = self.train
        mask0 = None if not self.maskZero else True
        if (getattr(self, "bf16IO", False) and self.bn is None and mask0 is None and x2.is_cuda
                and x2.dtype == torch.bfloat16 and self.cell.bf16_sequence_ok(x2)):
            x2l = x2.detach().requires_grad_(need_grad)     # bf16 straight from the projection GEMM
        else:
            x2l = _f32(x2.detach()).requires_grad_(need_grad)
        h0 = self._init_hidden if self._init_hidden is not None else self.cell.init_hidden(B, x2l[:, 0])
        h0l = [h.detach().float().to(x2l.device).requires_grad_(need_grad) for h in h0]
        mask = None
        if self.maskZero:
            mask = input.reshape(B, input.shape[1], -1).abs().amax(-1) != 0
        with _Leaves(self.cell.step_modules(), need_grad) as L, torch.set_grad_enabled(need_grad):
            out, hid = self.cell.sequence(x2l, h0l, mask)
        self._ag = (x2l, h0l, L, out, hid) if need_grad else None
        self._last_hidden = [t.detach() for t in hid]
        return out.detach()

    def updateGradInput(self, input, gradOutput):
        if self._ag is None:
            raise RuntimeError("Recurrent: backward called without a training forward")
        x2l, h0l, L, out, hid = self._ag
        targets = [x2l] + L.leaves + h0l
        go = gradOutput.to(out.dtype) if out.dtype == torch.bfloat16 else _f32(gradOutput)
        grads = torch.autograd.grad([out], targets, [go], allow_unused=True, retain_graph=True)
        gx2 = grads[0] if grads[0] is not None else torch.zeros_like(x2l)
        n = len(L.leaves)
        self._pending = grads[1:1 + n]
        self.gradHiddenState = [g for g in grads[1 + n:]]
        pre = self.cell.preTopology
        if pre is None:
            return gx2.to(input.dtype)
        B, T = input.shape[:2]
        g = gx2.reshape((B * T,) + tuple(gx2.shape[2:]))
        if self.bn is not None:
            self._gbn = g
            g = self.bn.updateGradInput(pre.output, g)
        self._gpre = g
        gi = pre.updateGradInput(self._flat, g).reshape(input.shape)
        if gi.dtype == torch.bfloat16 and input.dtype == torch.float32 and gi.is_cuda:
            return ops.to_f32(gi)           # native cast (bf16 projection gradient -> fp32 embedding gradient)
        return gi.to(input.dtype)

    def accGradParameters(self, input, gradOutput):
        if getattr(self, "_pending", None) is not None:
            self._ag[2].accumulate(self._pending)
            self._pending = None
        pre = self.cell.preTopology
        if pre is not None and not pre._frozen:
            if self.bn is not None and not self.bn._frozen:
                self.bn.accGradParameters(pre.output, self._gbn)
                self.bn._apply_regularizers()
            pre.accGradParameters(self._flat, self._gpre)
            pre._apply_regularizers()

    def backward(self, input, gradOutput):
        _SINK_ARMED[0] += 0 if self._frozen else 1
        try:
            self.gradInput = self.updateGradInput(input, gradOutput)
        finally:
            _SINK_ARMED[0] -= 0 if self._frozen else 1
        if not self._frozen:
            self.accGradParameters(input, gradOutput)
        return self.gradInput

    def clearState(self):
        super().clearState()
        self._ag = None
        return self


class RecurrentDecoder(Recurrent):
    """Feeds the output of step t as the input of step t+1 for ``outputLength`` steps
    (S/nn/RecurrentDecoder.scala:79). Input [batch, hidden...]; output [batch, outputLength, hidden...]."""

    def __init__(self, outputLength):
        super().__init__()
        self.outputLength = outputLength

    def updateOutput(self, input):
        B = input.shape[0]
        cell = self.cell
        need_grad = self.train
        xl = _f32(input.detach()).requires_grad_(need_grad)
        with _Leaves(cell.modules, need_grad) as L, torch.set_grad_enabled(need_grad):
            x = xl
            hid = self._init_hidden if self._init_hidden is not None else cell.init_hidden(B, cell.pre_fn(x))
            hid = [h.detach().float().to(xl.device).requires_grad_(need_grad) for h in hid]
            h0l = hid
            outs = []
            for _ in range(self.outputLength):
                o, hid = cell.step(cell.pre_fn(x), hid)
                outs.append(o)
                x = o
            out = torch.stack(outs, 1)
        self._ag = (xl, h0l, L, out, hid) if need_grad else None
        self._last_hidden = [t.detach() for t in hid]
        return out.detach()

    def updateGradInput(self, input, gradOutput):
        xl, h0l, L, out, hid = self._ag
        grads = torch.autograd.grad([out], [xl] + L.leaves + h0l, [_f32(gradOutput)], allow_unused=True,
                                    retain_graph=True)
        n = len(L.leaves)
        self._pending = grads[1:1 + n]
        self.gradHiddenState = list(grads[1 + n:])
        gx = grads[0] if grads[0] is not None else torch.zeros_like(xl)
        return gx.to(input.dtype)

    def accGradParameters(self, input, gradOutput):
        if getattr(self, "_pending", None) is not None:
            self._ag[2].accumulate(self._pending)
            self._pending = None


class BiRecurrent(Container):
    """Forward and time-reversed Recurrent over the same (or split) input, merged (S/nn/BiRecurrent.scala:41)."""

    def __init__(self, merge=None, batchNormParams=None, isSplitInput=False):
        super().__init__()
        from .table_ops import CAddTable

        self.isSplitInput = isSplitInput
        self.batchNormParams = batchNormParams
        self.layer = Recurrent(batchNormParams)
        self.revLayer = Recurrent(batchNormParams)
        self.merge = merge if merge is not None else CAddTable(True)
        self.modules = [self.layer, self.revLayer, self.merge]

    def add(self, cell):
        self.layer.add(cell)
        self.revLayer.add(cell.cloneModule())
        return self

    def getMerge(self):
        return self.merge

    def _set_children(self, children):
        self.layer, self.revLayer, self.merge = children
        self.modules = list(children)

    def _split(self, x):
        if not self.isSplitInput:
            return x, x
        d = x.shape[2] // 2
        return x[:, :, :d], x[:, :, d:]

    def updateOutput(self, input):
        a, b = self._split(input)
        self._ins = (a, b.flip(1))
        o1 = self.layer.forward(self._ins[0])
        o2 = self.revLayer.forward(self._ins[1]).flip(1)
        return self.merge.forward(Table(o1, o2))

    def updateGradInput(self, input, gradOutput):
        o1 = self.layer.output
        o2 = self.revLayer.output.flip(1)
        gm = self.merge.backward(Table(o1, o2), gradOutput)
        g1 = self.layer.backward(self._ins[0], gm[1])
        g2 = self.revLayer.backward(self._ins[1], gm[2].flip(1).contiguous()).flip(1)
        if self.isSplitInput:
            return torch.cat([g1, g2], 2)
        return g1 + g2

    def backward(self, input, gradOutput):
        self.gradInput = self.updateGradInput(input, gradOutput)
        return self.gradInput

    def accGradParameters(self, input, gradOutput):
        pass


class TimeDistributed(Container):
    """Applies ``layer`` to every time step by folding time into batch (S/nn/TimeDistributed.scala)."""

    def __init__(self, layer, maskZero=False):
        super().__init__(layer)
        self.layer = layer
        self.maskZero = maskZero

    def _fold(self, x):
        return x.reshape((x.shape[0] * x.shape[1],) + tuple(x.shape[2:]))

    def updateOutput(self, input):
        B, T = input.shape[:2]
        y = self.layer.forward(self._fold(input))
        y = y.reshape((B, T) + tuple(y.shape[1:]))
        if self.maskZero:
            m = input.reshape(B, T, -1).abs().amax(-1) != 0
            y = y * m.view(B, T, *([1] * (y.dim() - 2))).to(y.dtype)
        return y

    def _gfold(self, input, gradOutput):
        g = gradOutput
        if self.maskZero:
            B, T = input.shape[:2]
            m = input.reshape(B, T, -1).abs().amax(-1) != 0
            g = g * m.view(B, T, *([1] * (g.dim() - 2))).to(g.dtype)
        return self._fold(g)

    def updateGradInput(self, input, gradOutput):
        gi = self.layer.updateGradInput(self._fold(input), self._gfold(input, gradOutput))
        return gi.reshape(input.shape)

    def accGradParameters(self, input, gradOutput):
        self.layer.accGradParameters(self._fold(input), self._gfold(input, gradOutput))

    def backward(self, input, gradOutput):
        gi = self.layer.backward(self._fold(input), self._gfold(input, gradOutput))
        self.gradInput = gi.reshape(input.shape)
        return self.gradInput


RNN = RnnCell   # reference file S/nn/RNN.scala defines RnnCell
