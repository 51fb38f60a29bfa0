"""Transformer family: Attention, FeedForwardNetwork, Transformer (LanguageModel / Translation), the helper
layers of TransformerOperation, and SequenceBeamSearch.

Reference: S/nn/Attention.scala:35-115 (Q/K/V dense without bias, SplitHeads with q scaled by depth^-0.5,
MM(transB) + additive bias, softmax, dropout, MM, CombineHeads, output dense; incremental-decoding cache
``<name>_k``/``<name>_v`` :117-160), S/nn/FeedForwardNetwork.scala (dense+ReLU, dropout, dense),
S/nn/TransformerOperation.scala (dense = TimeDistributed Linear with Xavier/zeros init, getPositionEncode,
attentionBiasLowerTriangle, getPaddingBias), S/nn/Transformer.scala:53-560 (pre-norm blocks, LN at the end,
PositionEncode / PositionEncodeWithShift / SelfAttentionMask / PaddingMask / SplitTensor, shared embedding and
output projection, beam-search prediction), S/nn/SequenceBeamSearch.scala:39-631 (length-normalised beam
search with alive/finished sets, 1-based ids, ``layer_<i>_k/v`` caches).

Dropout arguments follow the reference convention: they are KEEP probabilities (``Dropout(1 - x)``), so 1.0
disables dropout.

MI355X execution: projections are GEMMs over all B*L rows; the attention core (ops.attention) dispatches to the
fused flash-attention HIP kernel on the GPU engine (online softmax in registers, no [L, L] score tensor in
HBM, causal block skipping) and to the explicit math path elsewhere.
"""
import math

import torch
import torch.nn.functional as F

from ..ops.conv_fn import linear as _linear

from ..ops.attention import attention as attention_core
from ..utils.table import Table
from .abstractnn import AbstractModule, TensorModule
from .activation import MulConstant, ReLU
from .containers import Container, Sequential
from .dropout import Dropout
from .graph import Graph, Input
from .init_methods import Xavier, Zeros
from .linear import Linear, LookupTable
from .normalization import LayerNormalization
from .recurrent import TimeDistributed, _Leaves
from .table_ops import CAddTable, JoinTable, SelectTable

__all__ = ["Attention", "FeedForwardNetwork", "Transformer", "SequenceBeamSearch", "PositionEncode",
           "PositionEncodeWithShift", "SelfAttentionMask", "PaddingMask", "SplitTensor", "TransformerOperation",
           "LanguageModel", "Translation"]

LanguageModel = "LanguageModel"
Translation = "Translation"
MASK_VALUE = -1e9


# ---------------------------------------------------------------------------------------------- operations
class TransformerOperation:
    """Static helpers (S/nn/TransformerOperation.scala)."""

    @staticmethod
    def dense(inputSize, outputSize, bias=True, activation=None, wRegularizer=None, bRegularizer=None, name=""):
        lin = Linear(inputSize, outputSize, withBias=bias, wRegularizer=wRegularizer, bRegularizer=bRegularizer)
        lin.setInitMethod(Xavier(), Zeros())
        if name:
            lin.setName(name)
        seq = Sequential().add(TimeDistributed(lin))
        if activation is not None:
            seq.add(activation)
        return seq

    @staticmethod
    def getPositionEncode(length, channels, minTimescale=1.0, maxTimescale=1.0e4, device=None):
        """Sinusoid timing signal [length, channels]: sin in the first half, cos in the second."""
        n = channels // 2
        log_inc = math.log(maxTimescale / minTimescale) / max(n - 1, 1)
        inv = minTimescale * torch.exp(torch.arange(n, dtype=torch.float32, device=device) * -log_inc)
        scaled = torch.arange(length, dtype=torch.float32, device=device).unsqueeze(1) * inv.unsqueeze(0)
        out = torch.zeros(length, channels, device=device)
        out[:, :n] = torch.sin(scaled)
        out[:, n:2 * n] = torch.cos(scaled)
        return out

    @staticmethod
    def attentionBiasLowerTriangle(length, device=None):
        b = torch.triu(torch.full((length, length), MASK_VALUE, device=device), diagonal=1)
        return b.view(1, 1, length, length)

    @staticmethod
    def getPadding(input, paddingValue=0.0):
        return (input == paddingValue).float()

    @staticmethod
    def getPaddingBias(input):
        return (TransformerOperation.getPadding(input) * MASK_VALUE).unsqueeze(1).unsqueeze(1)

    @staticmethod
    def shiftRight3D(input):
        out = torch.zeros_like(input)
        out[:, 1:] = input[:, :-1]
        return out


class _ConstGrad(TensorModule):
    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input, dtype=torch.float32 if not input.is_floating_point() else input.dtype)


class PositionEncode(_ConstGrad):
    """Timing signal [length, channels] for a [batch, length, channels] input (Transformer.scala:600)."""

    def updateOutput(self, input):
        return TransformerOperation.getPositionEncode(input.shape[1], input.shape[2], device=input.device)


class PositionEncodeWithShift(TensorModule):
    """Shift the sequence right by one and add the timing signal (Transformer.scala:627)."""

    def updateOutput(self, input):
        sig = TransformerOperation.getPositionEncode(input.shape[1], input.shape[2], device=input.device)
        return TransformerOperation.shiftRight3D(input.float()) + sig

    def updateGradInput(self, input, gradOutput):
        g = torch.zeros_like(gradOutput)
        g[:, :-1] = gradOutput[:, 1:]
        return g


class SelfAttentionMask(_ConstGrad):
    """Lower-triangular -1e9 bias [1, 1, L, L] hiding future positions (Transformer.scala:695)."""

    def updateOutput(self, input):
        b = TransformerOperation.attentionBiasLowerTriangle(input.shape[1], device=input.device)
        b._bigdl_causal = True
        return b


class PaddingMask(_ConstGrad):
    """-1e9 bias [B, 1, 1, L] on padding positions (Transformer.scala:680)."""

    def updateOutput(self, input):
        return TransformerOperation.getPaddingBias(input)


class SplitTensor(AbstractModule):
    """Split a tensor into ``num`` equal chunks along 1-based ``dimension`` (Transformer.scala:735)."""

    def __init__(self, dimension, num):
        super().__init__()
        self.dimension, self.num = dimension, num

    def updateOutput(self, input):
        d = self.dimension - 1
        return Table(*torch.chunk(input, self.num, d))

    def updateGradInput(self, input, gradOutput):
        return torch.cat(gradOutput.toSeq(), self.dimension - 1)


# ---------------------------------------------------------------------------------------------- attention
class Attention(Container):
    """Multi-head attention over T(x, y, bias) (or T(x, y, T(bias, cache)) for incremental decoding)."""

    def __init__(self, hiddenSize, numHeads, attentionDropout):
        super().__init__()
        assert hiddenSize % numHeads == 0
        self.hiddenSize, self.numHeads, self.attentionDropout = hiddenSize, numHeads, attentionDropout
        name = self.getName()
        self.queryLayer = self._dense(f"{name}_q")
        self.keyLayer = self._dense(f"{name}_k")
        self.valueLayer = self._dense(f"{name}_v")
        self.outputLayer = self._dense(f"{name}_output_transform")
        self.modules = [self.queryLayer, self.keyLayer, self.valueLayer, self.outputLayer]
        self._ag = None

    def _dense(self, name):
        lin = Linear(self.hiddenSize, self.hiddenSize, withBias=False)
        lin.setInitMethod(Xavier(), Zeros())
        return lin.setName(name)

    def _split(self, t):
        B, L, _ = t.shape
        return t.view(B, L, self.numHeads, self.hiddenSize // self.numHeads).transpose(1, 2)

    def _forward(self, x, y, bias, cache, causal):
        q = _linear(x, self.queryLayer.weight)
        k = _linear(y, self.keyLayer.weight)
        v = _linear(y, self.valueLayer.weight)
        if cache is not None:
            kn, vn = self.getName() + "_k", self.getName() + "_v"
            ck, cv = cache.get(kn), cache.get(vn)
            if ck is not None and ck.numel() > 0:
                k = torch.cat([k, ck.to(k.dtype)], 1)
                v = torch.cat([v, cv.to(v.dtype)], 1)
            if kn in cache.keys() or cache.length() > 0:
                cache[kn], cache[vn] = k.detach(), v.detach()
        depth = self.hiddenSize // self.numHeads
        qh = self._split(q) * depth ** -0.5
        kh, vh = self._split(k), self._split(v)
        o = attention_core(qh.contiguous(), kh.contiguous(), vh.contiguous(), bias,
                           dropout_p=1.0 - self.attentionDropout, training=self.train, causal=causal)
        B, _, L, _ = o.shape
        o = o.transpose(1, 2).reshape(B, L, self.hiddenSize)
        return _linear(o, self.outputLayer.weight)

    def updateOutput(self, input):
        x, y, b = input[1], input[2], input[3]
        cache = None
        if isinstance(b, Table):
            bias, cache = b[1], b[2]
        else:
            bias = b
        causal = bool(getattr(bias, "_bigdl_causal", False))
        need_grad = self.train and cache is None
        xl = x.detach().float().requires_grad_(need_grad)
        yl = y.detach().float().requires_grad_(need_grad)
        bl = None
        if bias is not None:
            bl = bias.detach().float().requires_grad_(need_grad)
        with _Leaves(self.modules, need_grad) as L, torch.set_grad_enabled(need_grad):
            out = self._forward(xl, yl, bl, cache, causal)
        self._ag = (xl, yl, bl, L, out) if need_grad else None
        return out.detach()

    def updateGradInput(self, input, gradOutput):
        if self._ag is None:
            raise RuntimeError("Attention: backward called without a training forward")
        xl, yl, bl, L, out = self._ag
        targets = [xl, yl] + ([bl] if bl is not None else []) + L.leaves
        grads = torch.autograd.grad([out], targets, [gradOutput.float()], allow_unused=True, retain_graph=True)
        z = lambda g, t: g if g is not None else torch.zeros_like(t)  # noqa: E731
        gi = Table(z(grads[0], xl), z(grads[1], yl))
        off = 2
        if bl is not None:
            gb = z(grads[2], bl)
            b3 = input[3]
            gi[3] = gb if not isinstance(b3, Table) else Table(gb, Table())
            off = 3
        self._pending = grads[off:]
        return gi

    def accGradParameters(self, input, gradOutput):
        if getattr(self, "_pending", None) is not None:
            self._ag[3].accumulate(self._pending)
            self._pending = None

    def backward(self, input, gradOutput):
        self.gradInput = self.updateGradInput(input, gradOutput)
        if not self._frozen:
            self.accGradParameters(input, gradOutput)
        return self.gradInput


class FeedForwardNetwork(Container):
    """dense(hidden -> filter, ReLU) -> Dropout(1 - reluDropout) -> dense(filter -> hidden)
    (S/nn/FeedForwardNetwork.scala). The first dense runs the MFMA Linear kernel with the ReLU fused into its
    epilogue on the GPU engine."""

    def __init__(self, hiddenSize, filterSize, reluDropout):
        super().__init__()
        self.hiddenSize, self.filterSize, self.reluDropout = hiddenSize, filterSize, reluDropout
        name = self.getName()
        self.filterLayer = Linear(hiddenSize, filterSize)
        self.filterLayer.setInitMethod(Xavier(), Zeros())
        self.filterLayer.setName(f"{name}_filter_layer")
        self.outputLayer = Linear(filterSize, hiddenSize)
        self.outputLayer.setInitMethod(Xavier(), Zeros())
        self.outputLayer.setName(f"{name}_output_layer")
        self.seq = Sequential().add(self.filterLayer).add(ReLU()).add(Dropout(1.0 - reluDropout)) \
            .add(self.outputLayer)
        self.modules = [self.seq]

    def _set_children(self, children):
        self.seq = children[0]
        self.modules = [self.seq]
        self.filterLayer, self.outputLayer = self.seq.modules[0], self.seq.modules[3]

    def updateOutput(self, input):
        return self.seq.forward(input)

    def updateGradInput(self, input, gradOutput):
        return self.seq.updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        self.seq.accGradParameters(input, gradOutput)

    def backward(self, input, gradOutput):
        self.gradInput = self.seq.backward(input, gradOutput)
        return self.gradInput


# ---------------------------------------------------------------------------------------------- transformer
class Transformer(Container):
    def __init__(self, vocabSize, hiddenSize, numHeads, filterSize, numHiddenlayers, embeddingDropout,
                 attentionDropout, ffnDropout, paddingValue=0.0, withShareWeightsLinear=False,
                 transformerType=LanguageModel, beamSearch=None):
        super().__init__()
        self.vocabSize, self.hiddenSize, self.numHeads = vocabSize, hiddenSize, numHeads
        self.filterSize, self.numHiddenlayers = filterSize, numHiddenlayers
        self.embeddingDropout, self.attentionDropout, self.ffnDropout = embeddingDropout, attentionDropout, \
            ffnDropout
        self.paddingValue = paddingValue
        self.withShareWeightsLinear = withShareWeightsLinear
        self.transformerType = transformerType
        self.beamSearch = beamSearch
        self.embedding = LookupTable(vocabSize, hiddenSize, paddingValue=paddingValue, maskZero=True) \
            .setName("embedding")
        self.embeddingLayer = Sequential().add(self.embedding).add(MulConstant(math.sqrt(hiddenSize)))
        self.linearSharedWeigths = TimeDistributed(Linear(hiddenSize, vocabSize, withBias=False))
        self.decoderStack = self.encoderStack = self.predictModel = None
        self.model = self._buildTranslation() if transformerType == Translation else self._buildLM()
        self.modules = [self.model] + ([self.linearSharedWeigths] if withShareWeightsLinear else [])

    def _set_children(self, children):
        _copy_state(self, Container(*children))

    # -- builders -----------------------------------------------------------------------------------
    def _drop(self, keep, name=None):
        d = Dropout(1.0 - keep)
        return d.setName(name) if name else d

    def block(self, numLayers, decoderInput, decoderSelfAttentionBias, encoderOutput=None,
              encoderAttentionBias=None, blockType="decode"):
        x = decoderInput
        for i in range(numLayers):
            pre = f"{blockType}_self_attention_{i}"
            norm = LayerNormalization(self.hiddenSize).setName(pre + "/norm").inputs(x)
            att = Attention(self.hiddenSize, self.numHeads, self.attentionDropout).setName(pre + "/self_attention")
            drop = self._drop(self.embeddingDropout, pre + "/dropout").inputs(
                att.inputs(norm, norm, decoderSelfAttentionBias))
            x = CAddTable().inputs(x, drop)
            if encoderOutput is not None and encoderAttentionBias is not None:
                pre = f"{blockType}_encdec_attention_{i}"
                norm = LayerNormalization(self.hiddenSize).setName(pre + "/norm").inputs(x)
                att = Attention(self.hiddenSize, self.numHeads, self.attentionDropout) \
                    .setName(pre + "/encdec_attention")
                drop = self._drop(self.embeddingDropout, pre + "/dropout").inputs(
                    att.inputs(norm, encoderOutput, encoderAttentionBias))
                x = CAddTable().inputs(x, drop)
            pre = f"{blockType}_ffn_{i}"
            norm = LayerNormalization(self.hiddenSize).setName(pre + "/norm").inputs(x)
            ffn = FeedForwardNetwork(self.hiddenSize, self.filterSize, self.ffnDropout).setName(pre + "/ffn")
            drop = self._drop(self.embeddingDropout, pre + "/dropout").inputs(ffn.inputs(norm))
            x = CAddTable().inputs(x, drop)
        return LayerNormalization(self.hiddenSize).inputs(x)

    def _buildLM(self):
        inp = Input()
        emb = MulConstant(math.sqrt(self.hiddenSize)).inputs(self.embedding.inputs(inp))
        dec_in = PositionEncodeWithShift().inputs(emb)
        bias = SelfAttentionMask().inputs(emb)
        drop = self._drop(self.embeddingDropout).inputs(dec_in)
        out = self.block(self.numHiddenlayers, drop, bias, blockType="decode")
        return Graph(inp, out)

    def _createDecoder(self):
        a, b, c, d = Input(), Input(), Input(), Input()
        return Graph([a, b, c, d], self.block(self.numHiddenlayers, a, b, c, d, blockType="decoder"))

    def _createEncoder(self):
        a, b = Input(), Input()
        return Graph([a, b], self.block(self.numHiddenlayers, a, b, blockType="encoder"))

    def _encode(self, inputs, bias):
        pos = PositionEncode().inputs(inputs)
        x = CAddTable().inputs(inputs, pos)
        x = self._drop(self.embeddingDropout).inputs(x)
        return self.encoderStack.inputs(x, bias)

    def _decode(self, targets, encoderOutput, bias):
        dec_in = PositionEncodeWithShift().inputs(targets)
        self_bias = SelfAttentionMask().inputs(targets)
        x = self._drop(self.embeddingDropout).inputs(dec_in)
        return self.decoderStack.inputs(x, self_bias, encoderOutput, bias)

    def _buildTranslation(self):
        self.decoderStack = self._createDecoder()
        self.encoderStack = self._createEncoder()
        inp, tgt = Input(), Input()
        bias = PaddingMask().inputs(inp)
        join = JoinTable(1, -1).inputs(inp, tgt)
        emb = self.embeddingLayer.inputs(join)
        split = SplitTensor(1, 2).inputs(emb)
        emb_in, emb_out = SelectTable(1).inputs(split), SelectTable(2).inputs(split)
        en, pn = Input(), Input()
        self.encoderGraph = Graph([en, pn], self._encode(en, pn))
        out = self._decode(emb_out, self.encoderGraph.inputs(emb_in, bias), bias)
        pi = Input()
        pmask = PaddingMask().inputs(pi)
        pemb = self.embeddingLayer.inputs(pi)
        self.predictModel = Graph(pi, [self.encoderGraph.inputs(pemb, pmask), pmask])
        if self.beamSearch is not None:
            self.beamSearch.setLogitFn(self.symbols)
        return Graph([inp, tgt], out)

    # -- execution ----------------------------------------------------------------------------------
    def _share(self):
        self.linearSharedWeigths.layer.weight.data.copy_(self.embedding.weight.data)

    def updateOutput(self, input):
        if self.transformerType == Translation and isinstance(input, torch.Tensor):
            assert not self.train, "tensor input for a Translation transformer means beam-search prediction"
            res = self.predictModel.forward(input)
            bs = self.beamSearch.forward(Table(res[1], res[2]))
            ids, scores = bs[1][:, 0], bs[2][:, 0]
            return Table(ids[:, 1:], scores)
        out = self.model.forward(input)
        if self.withShareWeightsLinear:
            self._share()
            out = self.linearSharedWeigths.forward(out)
        return out

    def updateGradInput(self, input, gradOutput):
        g = gradOutput
        if self.withShareWeightsLinear:
            g = self.linearSharedWeigths.updateGradInput(self.model.output, gradOutput)
        return self.model.updateGradInput(input, g)

    def accGradParameters(self, input, gradOutput):
        g = gradOutput
        if self.withShareWeightsLinear:
            g = self.linearSharedWeigths.gradInput
        self.model.accGradParameters(input, g)

    def backward(self, input, gradOutput):
        g = gradOutput
        if self.withShareWeightsLinear:
            g = self.linearSharedWeigths.updateGradInput(self.model.output, gradOutput)
        self.gradInput = self.model.backward(input, g)
        return self.gradInput

    def symbols(self, ids, i, maxDecodeLength, encoder_outputs, encoder_decoder_attention_bias, cacheValue):
        """One incremental decoding step for beam search (Transformer.scala:162-212)."""
        cache = Table()
        for m in range(1, self.hiddenSize + 1):
            if f"layer_{m}_k" in cacheValue.keys():
                cache[f"decoder_self_attention_{m - 1}/self_attention_k"] = cacheValue[f"layer_{m}_k"]
                cache[f"decoder_self_attention_{m - 1}/self_attention_v"] = cacheValue[f"layer_{m}_v"]
        length = maxDecodeLength + 1
        timing = TransformerOperation.getPositionEncode(length, self.hiddenSize, device=ids.device)
        bias_full = TransformerOperation.attentionBiasLowerTriangle(maxDecodeLength, device=ids.device)
        dec_in = ids[:, i:i + 1]
        emb = self.embeddingLayer.forward(dec_in).float() + timing[i]
        self_bias = bias_full[:, :, i:i + 1, :i + 1]
        out = self.decoderStack.forward(Table(emb, Table(self_bias, cache), encoder_outputs,
                                              encoder_decoder_attention_bias))
        self._share()
        logits = self.linearSharedWeigths.forward(out)
        for m in range(1, self.hiddenSize + 1):
            if f"layer_{m}_k" in cacheValue.keys():
                cacheValue[f"layer_{m}_k"] = cache[f"decoder_self_attention_{m - 1}/self_attention_k"]
                cacheValue[f"layer_{m}_v"] = cache[f"decoder_self_attention_{m - 1}/self_attention_v"]
        return logits.squeeze(1), cacheValue


def _copy_state(dst, src):
    from .recurrent import _copy_module_state

    _copy_module_state(dst, src)


# ---------------------------------------------------------------------------------------------- beam search
class SequenceBeamSearch(AbstractModule):
    """Beam search over ``symbolToLogits`` (S/nn/SequenceBeamSearch.scala:39). Input T(encoder_outputs,
    encoder_decoder_attention_bias); output T(sequences [B, beam, len] (1-based ids), scores [B, beam])."""

    INF = -1e7

    def __init__(self, vocabSize, beamSize, alpha, maxDecodeLength, eosID, paddingValue, numHiddenLayers,
                 hiddenSize):
        super().__init__()
        self.vocabSize, self.beamSize, self.alpha = vocabSize, beamSize, alpha
        self.maxDecodeLength, self.eosID, self.paddingValue = maxDecodeLength, eosID, paddingValue
        self.numHiddenLayers, self.hiddenSize = numHiddenLayers, hiddenSize
        self.symbolToLogits = None

    def setLogitFn(self, fn):
        self.symbolToLogits = fn
        return self

    def _lnorm(self, length):
        return (5.0 + length / 6.0) ** self.alpha

    @staticmethod
    def _gather(t, idx):
        """t [B, K, ...], idx [B, K'] -> [B, K', ...]."""
        B, K2 = idx.shape
        view = idx.view(B, K2, *([1] * (t.dim() - 2))).expand(B, K2, *t.shape[2:])
        return torch.gather(t, 1, view)

    def _topk_gather(self, ts, scores, k):
        _, ix = torch.topk(scores, k, dim=-1)
        return [self._gather(t, ix) if t is not None and t.numel() else t for t in ts]

    def updateOutput(self, input):
        enc, att_bias = input[1], input[2]
        assert self.symbolToLogits is not None, "symbolToLogits function is null, please set this function"
        B, K, V = enc.shape[0], self.beamSize, self.vocabSize
        dev = enc.device
        alive_seq = torch.full((B, K, 1), float(self.paddingValue), device=dev)
        alive_lp = torch.full((B, K), self.INF, device=dev)
        alive_lp[:, 0] = 0.0
        alive_enc = enc.unsqueeze(1).expand(B, K, *enc.shape[1:]).contiguous()
        alive_bias = att_bias.unsqueeze(1).expand(B, K, *att_bias.shape[1:]).contiguous()
        layers = {f"layer_{j}_{c}": None for j in range(1, self.numHiddenLayers + 1) for c in "kv"}
        fin_seq = torch.zeros_like(alive_seq)
        fin_scores = torch.full((B, K), self.INF, device=dev)
        fin_flags = torch.zeros(B, K, dtype=torch.bool, device=dev)
        i = 0
        while self._continue(i, alive_lp, fin_scores, fin_flags):
            flat = lambda t: t.reshape(B * K, *t.shape[2:])  # noqa: E731
            cache = Table()
            for name, t in layers.items():
                cache[name] = flat(t) if t is not None else torch.zeros(0, device=dev)
            logits, new_cache = self.symbolToLogits(flat(alive_seq), i, self.maxDecodeLength, flat(alive_enc),
                                                    flat(alive_bias), cache)
            logits = logits.reshape(B, K, V).float()
            lp = torch.log_softmax(logits, -1) + alive_lp.unsqueeze(2)
            top_lp, top_ix = torch.topk(lp.reshape(B, K * V), 2 * K, dim=-1)
            beam_ix = top_ix // V
            top_seq = self._gather(alive_seq, beam_ix)
            top_enc = self._gather(alive_enc, beam_ix)
            top_bias = self._gather(alive_bias, beam_ix)
            top_layers = {}
            for name in layers:
                t = new_cache[name]
                top_layers[name] = self._gather(t.reshape(B, K, *t.shape[1:]), beam_ix) if t is not None and \
                    t.numel() else None
            ids = (top_ix % V + 1).float().unsqueeze(2)
            new_seq = torch.cat([top_seq, ids], 2)
            new_fin = new_seq[:, :, -1] == self.eosID
            # alive set: best K not-finished
            lp_alive = top_lp + new_fin.float() * self.INF
            _, ix = torch.topk(lp_alive, K, dim=-1)
            alive_seq = self._gather(new_seq, ix)
            alive_lp = torch.gather(lp_alive, 1, ix)
            alive_enc = self._gather(top_enc, ix)
            alive_bias = self._gather(top_bias, ix)
            layers = {n: (self._gather(t, ix) if t is not None else None) for n, t in top_layers.items()}
            # finished set
            fin_seq = torch.cat([fin_seq, torch.full((B, K, 1), float(self.paddingValue), device=dev)], 2)
            new_scores = top_lp / self._lnorm(i + 1) + (~new_fin).float() * self.INF
            all_seq = torch.cat([fin_seq, new_seq], 1)
            all_scores = torch.cat([fin_scores, new_scores], 1)
            all_flags = torch.cat([fin_flags, new_fin], 1)
            _, ix = torch.topk(all_scores, K, dim=-1)
            fin_seq = self._gather(all_seq, ix)
            fin_scores = torch.gather(all_scores, 1, ix)
            fin_flags = torch.gather(all_flags, 1, ix)
            i += 1
        any_fin = fin_flags.any(1)
        seq = torch.where(any_fin.view(B, 1, 1), fin_seq, alive_seq)
        scores = torch.where(any_fin.view(B, 1), fin_scores, alive_lp)
        return Table(seq, scores)

    def _continue(self, i, alive_lp, fin_scores, fin_flags):
        if i >= self.maxDecodeLength:
            return False
        best_alive = alive_lp[:, 0] / self._lnorm(self.maxDecodeLength)
        lowest_fin = (fin_scores * fin_flags.float()).min(1).values
        lowest_fin = lowest_fin + (1.0 - fin_flags.any(1).float()) * self.INF
        return not bool(torch.all(lowest_fin > best_alive))

    def updateGradInput(self, input, gradOutput):
        return gradOutput
