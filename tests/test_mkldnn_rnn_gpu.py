"""nn.mkldnn.RNN on the GPU: every (layer, direction) through the whole-sequence persistent kernels
(csrc/lstm_seq.hip), against the same module's fp32 torch recurrences on the CPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("mode,direction,layers", [
    ("vanilla_lstm", "unidirectional_left2right", 2),
    ("vanilla_lstm", "bidirectional_sum", 2),
    ("vanilla_lstm", "bidirectional_concat", 1),
    ("vanilla_gru", "unidirectional_left2right", 2),
])
def test_rnn_gpu_matches_cpu(mode, direction, layers):
    from bigdl_amd import ops
    from bigdl_amd.nn import mkldnn as dnn

    T, N, H = 12, 32, 256
    C = ops.native.get()
    seq_ok = C.lstm_seq_supported(N, H) if mode == "vanilla_lstm" else C.gru_seq_supported(N, H)
    assert seq_ok, "this shape should take the whole-sequence persistent kernels"
    torch.manual_seed(7)
    cpu = dnn.RNN(mode, H, H, direction=direction, layers=layers)
    with torch.no_grad():
        cpu.weight.mul_(0.5)
        cpu.weight_i.mul_(0.5)
        cpu.bias.uniform_(-0.1, 0.1)
    gpu = dnn.RNN(mode, H, H, direction=direction, layers=layers, initWeight=cpu.weight,
                  initWeightIter=cpu.weight_i, initBias=cpu.bias).to("cuda")
    x = torch.randn(T, N, H) * 0.5
    gy = torch.randn(T, N, cpu.outputSize()) * 0.1
    y_c, gx_c = cpu.forward(x), cpu.backward(x, gy)
    y_g = gpu.forward(x.cuda())
    gx_g = gpu.backward(x.cuda(), gy.cuda())
    torch.cuda.synchronize()
    assert y_g.is_cuda and torch.isfinite(y_g).all()
    assert _rel(y_g, y_c) < 2e-2
    assert _rel(gx_g, gx_c) < 3e-2
    for gname in ("gradWeight", "gradWeight_i", "gradBias"):
        assert _rel(getattr(gpu, gname), getattr(cpu, gname)) < 3e-2, gname


def test_ptb_lm_dnn_lowering_on_gpu():
    """The PTB LM (LookupTable -> 2 x Recurrent(LSTM 256) -> TimeDistributed(Linear)) lowered for inference: the LSTM
    stack becomes one nn.mkldnn.RNN(layers = 2) on the persistent kernels, same output as the Recurrent stack."""
    from bigdl_amd.models.rnn import PTBModel
    from bigdl_amd.nn import mkldnn as dnn
    from bigdl_amd.utils.intermediate import ConversionUtils

    torch.manual_seed(8)
    m = PTBModel.lstm(500, 256, 500, 2)
    m.evaluate()
    ids = torch.randint(1, 501, (32, 20)).float()
    ref = m.forward(ids).float()
    g = ConversionUtils.convert(m, "dnn", device="cuda", train=False)
    rnns = [q for q in g.flattened_layers() if isinstance(q, dnn.RNN)]
    assert len(rnns) == 1 and rnns[0].layers == 2
    out = g.forward(ids.cuda()).float().cpu()
    assert _rel(out, ref) < 2e-2
