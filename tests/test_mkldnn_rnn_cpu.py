"""nn.mkldnn.RNN (reference S/nn/mkldnn/RNN.scala; its spec S/nn/mkldnn/RNNSpec.scala compares against nn/LSTM,
nn/GRU and BiRecurrent with the gate orders remapped): LSTM against torch.nn.LSTM (same (i, f, g, o) gate order as the
primitive) for stacked, right-to-left and bidirectional runs, forward and gradients; GRU against the framework's own
Recurrent(GRU) / BiRecurrent(GRU) with the reference's (u, r, n) -> (r, z, n) mapping; layouts and argument checks."""
import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.nn import mkldnn as dnn


def _torch_lstm(rnn, layers, bidirectional, l0=0, d0=0):
    """torch.nn.LSTM with rnn's ldigo weights of layers l0.. (direction d0 for a one-direction module)."""
    H, I = rnn.hiddenSize, rnn.weight.shape[2]
    m = torch.nn.LSTM(I, H, num_layers=layers, bidirectional=bidirectional, batch_first=True)
    with torch.no_grad():
        for k in range(layers):
            for d in range(2 if bidirectional else 1):
                sfx = f"_l{k}" + ("_reverse" if d == 1 else "")
                dd = d if bidirectional else d0
                getattr(m, "weight_ih" + sfx).copy_(rnn.weight[l0 + k, dd].permute(1, 2, 0).reshape(4 * H, -1))
                getattr(m, "weight_hh" + sfx).copy_(rnn.weight_i[l0 + k, dd].permute(1, 2, 0).reshape(4 * H, H))
                getattr(m, "bias_ih" + sfx).copy_(rnn.bias[l0 + k, dd].reshape(4 * H))
                getattr(m, "bias_hh" + sfx).zero_()
    return m


def _run(rnn, x, gy):
    y = rnn.forward(x)
    gx = rnn.backward(x, gy)
    return y, gx


@pytest.mark.parametrize("layers", [1, 3])
def test_lstm_unidirectional_matches_torch(layers):
    torch.manual_seed(0)
    T, N, C = 5, 3, 6
    rnn = dnn.RNN(dnn.AlgKind.VanillaLstm, C, C, dnn.AlgKind.EltwiseTanh, dnn.Direction.UnidirectionalLeft2Right,
                  layers=layers)
    with torch.no_grad():
        rnn.bias.uniform_(-0.5, 0.5)
    x = torch.randn(T, N, C)
    gy = torch.randn(T, N, C)
    y, gx = _run(rnn, x, gy)
    ref = _torch_lstm(rnn, layers, False)
    xr = x.transpose(0, 1).clone().requires_grad_(True)
    yr, _ = ref(xr)
    yr.backward(gy.transpose(0, 1))
    assert torch.allclose(y, yr.transpose(0, 1), atol=1e-5)
    assert torch.allclose(gx, xr.grad.transpose(0, 1), atol=1e-5)
    for k in range(layers):
        gw = ref.__getattr__(f"weight_ih_l{k}").grad.reshape(4, C, -1).permute(2, 0, 1)
        gu = ref.__getattr__(f"weight_hh_l{k}").grad.reshape(4, C, C).permute(2, 0, 1)
        gb = ref.__getattr__(f"bias_ih_l{k}").grad.reshape(4, C)
        assert torch.allclose(rnn.gradWeight[k, 0], gw, atol=1e-5)
        assert torch.allclose(rnn.gradWeight_i[k, 0], gu, atol=1e-5)
        assert torch.allclose(rnn.gradBias[k, 0], gb, atol=1e-5)


def test_lstm_right_to_left_is_reversed_time():
    torch.manual_seed(1)
    T, N, C, H = 4, 2, 3, 5
    rnn = dnn.RNN(dnn.AlgKind.VanillaLstm, C, H, direction=dnn.Direction.UnidirectionalRight2Left)
    x = torch.rand(T, N, C)
    ref = _torch_lstm(rnn, 1, False)
    yr, _ = ref(x.flip(0).transpose(0, 1))
    assert torch.allclose(rnn.forward(x), yr.transpose(0, 1).flip(0), atol=1e-5)


def test_lstm_bidirectional_concat_matches_torch():
    torch.manual_seed(2)
    T, N, C, H = 4, 3, 3, 5
    rnn = dnn.RNN(dnn.AlgKind.VanillaLstm, C, H, direction=dnn.Direction.BidirectionalConcat)
    x = torch.rand(T, N, C)
    gy = torch.randn(T, N, 2 * H)
    y, gx = _run(rnn, x, gy)
    assert y.shape == (T, N, 2 * H) and rnn.outputSize() == 2 * H
    ref = _torch_lstm(rnn, 1, True)
    xr = x.transpose(0, 1).clone().requires_grad_(True)
    yr, _ = ref(xr)
    yr.backward(gy.transpose(0, 1))
    assert torch.allclose(y, yr.transpose(0, 1), atol=1e-5)
    assert torch.allclose(gx, xr.grad.transpose(0, 1), atol=1e-5)
    gu_rev = ref.weight_hh_l0_reverse.grad.reshape(4, H, H).permute(2, 0, 1)
    assert torch.allclose(rnn.gradWeight_i[0, 1], gu_rev, atol=1e-5)


def test_lstm_bidirectional_sum_two_layers():
    """Each layer's directions are summed, and the sum feeds the next layer (RNN.scala:100-109)."""
    torch.manual_seed(3)
    T, N, C = 4, 2, 6
    rnn = dnn.RNN(dnn.AlgKind.VanillaLstm, C, C, direction=dnn.Direction.BidirectionalSum, layers=2)
    x = torch.rand(T, N, C)
    gy = torch.randn(T, N, C)
    y, gx = _run(rnn, x, gy)
    xr = x.transpose(0, 1).clone().requires_grad_(True)
    seq = xr
    for k in range(2):
        fwd = _torch_lstm(rnn, 1, False, l0=k, d0=0)(seq)[0]
        bwd = _torch_lstm(rnn, 1, False, l0=k, d0=1)(seq.flip(1))[0].flip(1)
        seq = fwd + bwd
    seq.backward(gy.transpose(0, 1))
    assert torch.allclose(y, seq.detach().transpose(0, 1), atol=1e-5)
    assert torch.allclose(gx, xr.grad.transpose(0, 1), atol=1e-5)


def _gru_cells(rnn, l, d):
    """nn.GRU with rnn's (l, d) weights remapped: primitive (u, r, n) -> nn (r, z, n)."""
    H, I = rnn.hiddenSize, rnn.weight.shape[2]
    cell = nn.GRU(I, H)
    order = [1, 0, 2]
    with torch.no_grad():
        W = rnn.weight[l, d].permute(1, 2, 0)[order].reshape(3 * H, I)
        U = rnn.weight_i[l, d].permute(1, 2, 0)[order].reshape(3 * H, H)
        cell.preTopology.weight.copy_(W)
        cell.preTopology.bias.copy_(rnn.bias[l, d][order].reshape(3 * H))
        cell.h2g.weight.copy_(U[:2 * H])
        cell.h2n.weight.copy_(U[2 * H:])
    return cell


def test_gru_stacked_matches_recurrent_gru():
    torch.manual_seed(4)
    T, N, C = 5, 3, 4
    rnn = dnn.RNN(dnn.AlgKind.VanillaGru, C, C, layers=2)
    with torch.no_grad():
        rnn.bias.uniform_(-0.3, 0.3)
    x = torch.rand(T, N, C)
    gy = torch.randn(T, N, C)
    y, gx = _run(rnn, x, gy)
    blas = nn.Sequential()
    for k in range(2):
        blas.add(nn.Recurrent().add(_gru_cells(rnn, k, 0)))
    xb = x.transpose(0, 1).contiguous()
    yb = blas.forward(xb)
    gxb = blas.backward(xb, gy.transpose(0, 1).contiguous())
    assert torch.allclose(y, yb.transpose(0, 1), atol=1e-5)
    assert torch.allclose(gx, gxb.transpose(0, 1), atol=1e-5)
    # the recurrent weight gradient of layer 0, mapped back to the primitive's (u, r, n) ldigo layout
    cell = blas.modules[0].modules[0]
    H = C
    g_nn = torch.cat([cell.h2g.gradWeight, cell.h2n.gradWeight], 0).view(3, H, H)[[1, 0, 2]]
    assert torch.allclose(rnn.gradWeight_i[0, 0], g_nn.permute(2, 0, 1), atol=1e-5)


def test_gru_bidirectional_sum_matches_birecurrent():
    torch.manual_seed(5)
    T, N, C, H = 4, 2, 3, 5
    rnn = dnn.RNN(dnn.AlgKind.VanillaGru, C, H, direction=dnn.Direction.BidirectionalSum)
    x = torch.rand(T, N, C)
    bi = nn.BiRecurrent().add(_gru_cells(rnn, 0, 0))
    bi.revLayer.add(_gru_cells(rnn, 0, 1))
    yb = bi.forward(x.transpose(0, 1).contiguous())
    assert torch.allclose(rnn.forward(x), yb.transpose(0, 1), atol=1e-5)


def test_ntc_format_and_parameters_layout():
    torch.manual_seed(6)
    N, T, C, H = 2, 3, 4, 4
    a = dnn.RNN(dnn.AlgKind.VanillaLstm, C, H, layers=2)
    b = dnn.RNN(dnn.AlgKind.VanillaLstm, C, H, layers=2, inputFormat="ntc",
                initWeight=a.weight, initWeightIter=a.weight_i, initBias=a.bias)
    x = torch.rand(T, N, C)
    assert torch.allclose(a.forward(x), b.forward(x.transpose(0, 1).contiguous()).transpose(0, 1), atol=1e-6)
    ws, gs = a.parameters()
    assert [tuple(w.shape) for w in ws] == [(2, 1, C, 4, H), (2, 1, 4, H), (2, 1, H, 4, H)]
    assert len(gs) == 3
    g = dnn.RNN(dnn.AlgKind.VanillaGru, C, H, direction=dnn.Direction.BidirectionalConcat)
    assert tuple(g.parameters()[0][0].shape) == (1, 2, C, 3, H)


def test_argument_checks():
    with pytest.raises(ValueError):
        dnn.RNN(dnn.AlgKind.VanillaLstm, 3, 5, layers=2)                 # stacked needs input == hidden
    with pytest.raises(ValueError):
        dnn.RNN(dnn.AlgKind.VanillaLstm, 5, 5, direction=dnn.Direction.BidirectionalConcat, layers=2)
    with pytest.raises(ValueError):
        dnn.RNN("vanilla_rnn", 5, 5)
    rnn = dnn.RNN(dnn.AlgKind.VanillaLstm, 3, 5)
    with pytest.raises(ValueError):
        rnn.forward(torch.rand(2, 3, 4))


def test_dnn_lowering_merges_lstm_stacks():
    """ConversionUtils.convert(model, "dnn") for inference turns a chain of plain Recurrent(LSTM(H, H)) layers into
    ONE nn.mkldnn.RNN with layers = chain length (weights moved into the ldigo layout / primitive gate order); a first
    layer whose input size differs from H stays a Recurrent (the primitive stacks need inputSize == hiddenSize)."""
    from bigdl_amd.utils.intermediate import ConversionUtils

    torch.manual_seed(7)
    m = nn.Sequential()
    m.add(nn.Recurrent().add(nn.LSTM(5, 8)))
    for _ in range(3):
        m.add(nn.Recurrent().add(nn.LSTM(8, 8)))
    m.add(nn.TimeDistributed(nn.Linear(8, 4)))
    m.evaluate()
    x = torch.randn(2, 6, 5)
    ref = m.forward(x)
    g = ConversionUtils.convert(m, "dnn", device="cpu", train=False)
    layers = g.flattened_layers()
    rnns = [q for q in layers if isinstance(q, dnn.RNN)]
    assert len(rnns) == 1 and rnns[0].layers == 3 and rnns[0].inputFormat == "ntc"
    assert sum(isinstance(q, nn.Recurrent) for q in layers) == 1
    assert torch.allclose(g.forward(x), ref, atol=1e-5)
