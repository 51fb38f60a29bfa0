"""Transformer family on the CPU engine. The encode-block and beam-search tests pin the reference's own
numeric fixtures (T/nn/TransformerSpec.scala:27-197 "tranformer decode stack", extracted to
tests/fixtures/transformer_encode_block.json by tools/extract_scala_fixture.py; SequenceBeamSearchSpec.scala:24)."""
import json
import os

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.utils.gradient_checker import GradientChecker
from bigdl_amd.utils.random_generator import RNG
from bigdl_amd.utils.table import T

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def test_encode_block_matches_reference_fixture():
    q, k, v, o, filt, outl, inp, bias, expect, gi1, gi2, gw = json.load(
        open(os.path.join(FIX, "transformer_encode_block.json")))
    tr = nn.Transformer(10, 4, 2, 3, 1, 1.0, 1.0, 1.0)
    i1, i2 = nn.Input(), nn.Input()
    block = nn.Graph([i1, i2], tr.block(1, i1, i2, blockType="encode"))
    table = block.getParametersTable()
    for key in table.keys():
        w = table[key].get("weight")
        if w is None:
            continue
        for tag, val in (("_q", q), ("_k", k), ("_v", v), ("_output_transform", o), ("_filter_layer", filt),
                         ("_output_layer", outl)):
            if str(key).endswith(tag):
                w.copy_(torch.tensor(val).t())
    x, b = torch.tensor(inp), torch.tensor(bias)
    y = block.forward(T(x, b))
    assert torch.allclose(y, torch.tensor(expect), atol=1e-5)
    g = block.backward(T(x, b), y)
    # The reference back-propagates gradOutput = output through the final LayerNorm (unit gamma, zero beta):
    # ||LN(x)||^2 is constant, so the exact input gradient is 0 and the fixture holds fp32 rounding noise of
    # magnitude ~1e-5. Pin the noise level, and the meaningful parts exactly: the final LN's parameter
    # gradients and the total parameter count/order.
    assert g[1].abs().max() < 1e-4 and torch.tensor(gi1).abs().max() < 1e-4
    assert torch.allclose(g[2], torch.tensor(gi2), atol=1e-6)
    gws = torch.cat([t.reshape(-1) for t in block.parameters()[1]])
    assert gws.numel() == len(gw)
    assert torch.allclose(gws[-8:], torch.tensor(gw[-8:]), rtol=1e-5)


def test_beam_search_matches_reference_fixture():
    logits = torch.tensor([0.14, 0.62, 0.02, 0.93, 0.59, 0.48, 0.27, 0.70, 0.11, 0.30, 0.35, 0.15,
                           0.67, 0.39, 0.33, 0.01, 0.44, 0.52, 0.45, 0.23, 0.75, 0.79, 0.26, 0.47]).view(6, 4)

    def fn(ids, i, maxlen, enc, bias, layer):
        out = T()
        for j in range(1, 3):
            out[f"layer_{j}_k"] = torch.rand(6, i + 1, 5)
            out[f"layer_{j}_v"] = torch.rand(6, i + 1, 5)
        return logits, out

    bs = nn.SequenceBeamSearch(4, 3, 0.0, 10, 2.0, 1.0, 2, 5).setLogitFn(fn)
    out = bs.forward(T(torch.rand(2, 6, 5), torch.rand(2, 1, 1, 6)))
    seq = torch.tensor([[[1, 2, 1, 1, 1], [1, 4, 2, 1, 1], [1, 4, 4, 2, 1]],
                        [[1, 2, 1, 1, 1], [1, 1, 2, 1, 1], [1, 3, 2, 1, 1]]], dtype=torch.float32)
    score = torch.tensor([[-1.2615868, -2.2131736, -3.1647604], [-1.3734006, -2.4668012, -2.715382]])
    assert torch.equal(out[1], seq)
    assert torch.allclose(out[2], score, atol=1e-5)


def test_attention_incremental_cache_equals_full_causal():
    RNG.setSeed(1)
    att = nn.Attention(8, 2, 1.0).evaluate()
    x = torch.randn(2, 5, 8)
    mask = nn.SelfAttentionMask().forward(x)
    full = att.forward(T(x, x, mask))
    cache = T()
    cache[att.getName() + "_k"] = torch.zeros(0)
    cache[att.getName() + "_v"] = torch.zeros(0)
    steps = []
    for i in range(5):
        xi = x[:, i:i + 1]
        steps.append(att.forward(T(xi, xi, T(torch.zeros(1, 1, 1, i + 1), cache))))
    assert torch.allclose(torch.cat(steps, 1), full, atol=1e-5)


def test_attention_and_ffn_gradients():
    RNG.setSeed(2)
    att = nn.Attention(8, 2, 1.0)
    x, y = torch.randn(2, 3, 8), torch.randn(2, 4, 8)
    bias = torch.zeros(2, 1, 1, 4)
    gc = GradientChecker(1e-2, 3e-2)
    assert gc.checkLayer(att, T(x, y, bias))[0]
    assert gc.checkWeight(att, T(x, y, bias))[0]
    ffn = nn.FeedForwardNetwork(8, 6, 1.0)
    assert gc.checkLayer(ffn, x)[0] and gc.checkWeight(ffn, x)[0]


def test_language_model_trains():
    RNG.setSeed(3)
    torch.manual_seed(0)
    tr = nn.Transformer(20, 16, 2, 32, 2, 1.0, 1.0, 1.0, withShareWeightsLinear=True)
    ids = torch.randint(1, 21, (4, 7)).float()
    crit = nn.TimeDistributedCriterion(nn.CrossEntropyCriterion())
    from bigdl_amd.optim import SGD

    w, g = tr.getParameters()
    sgd = SGD(0.01, momentum=0.9, dampening=0.0)
    losses = []
    for _ in range(15):
        def feval(_):
            tr.zeroGradParameters()
            out = tr.forward(ids)
            loss = crit.forward(out, ids)
            tr.backward(ids, crit.backward(out, ids))
            return float(loss), g
        sgd.optimize(feval, w)
        losses.append(crit.output if not isinstance(crit.output, torch.Tensor) else float(crit.output))
    assert losses[-1] < losses[0] * 0.7, losses


def test_translation_train_and_beam_predict():
    RNG.setSeed(4)
    bs = nn.SequenceBeamSearch(16, 3, 0.6, 5, 2.0, 0.0, 2, 8)
    tr = nn.Transformer(16, 8, 2, 12, 2, 1.0, 1.0, 1.0, withShareWeightsLinear=True,
                        transformerType=nn.Translation, beamSearch=bs)
    src = torch.tensor([[3., 4., 5., 0.], [6., 7., 0., 0.]])
    tgt = torch.tensor([[4., 5., 6., 2.], [7., 8., 9., 2.]])   # reference joins src/tgt on batch: equal lengths
    out = tr.forward(T(src, tgt))
    assert out.shape == (2, 4, 16)
    g = tr.backward(T(src, tgt), torch.randn_like(out))
    tr.evaluate()
    pred = tr.forward(src)
    assert pred[1].shape[0] == 2 and pred[2].shape == (2,)


def test_position_encode_values():
    pe = nn.TransformerOperation.getPositionEncode(3, 8)
    assert torch.allclose(pe[0], torch.tensor([0, 0, 0, 0, 1, 1, 1, 1.0]))
    assert abs(float(pe[1, 0]) - 0.84147096) < 1e-6
