"""SimpleRNN language model (S/models/rnn/SimpleRNN.scala): Recurrent(RnnCell(tanh)) + TimeDistributed(Linear)."""
from .. import nn


def SimpleRNN(inputSize, hiddenSize, outputSize):
    return nn.Sequential().add(nn.Recurrent().add(nn.RnnCell(inputSize, hiddenSize, nn.Tanh()))) \
        .add(nn.TimeDistributed(nn.Linear(hiddenSize, outputSize)))


class PTBModel:
    """Word language models of the PTB example (S/example/languagemodel/PTBModel.scala:25-80)."""

    @staticmethod
    def transformer(inputSize=10000, hiddenSize=256, outputSize=10000, numLayers=2, keepProb=2.0):
        inp = nn.Input()
        tr = nn.Transformer(inputSize, hiddenSize, 4, hiddenSize * 4, numLayers, 1 - keepProb, 0.1, 0.1)
        out = nn.TimeDistributed(nn.Linear(hiddenSize, outputSize)).inputs(tr.inputs(inp))
        return nn.Graph(inp, out)

    @staticmethod
    def lstm(inputSize, hiddenSize, outputSize, numLayers, keepProb=2.0):
        """LookupTable -> (Dropout(keepProb) when keepProb < 1, the reference passes it as the drop rate)
        -> numLayers x Recurrent(LSTM) -> TimeDistributed(Linear)."""
        inp = nn.Input()
        x = nn.LookupTable(inputSize, hiddenSize).inputs(inp)
        if keepProb < 1:
            x = nn.Dropout(keepProb).inputs(x)
        for _ in range(numLayers):
            # bf16 sequence I/O between the projection GEMMs and the persistent recurrence (opt-in, GPU only)
            x = nn.Recurrent(bf16IO=True).add(nn.LSTM(hiddenSize, hiddenSize, 0)).inputs(x)
        return nn.Graph(inp, nn.TimeDistributed(nn.Linear(hiddenSize, outputSize)).inputs(x))
