"""Apply a trained text classifier as a batched prediction UDF over a DataFrame column, then query the result.

Reference: S/example/udfpredictor/DataframePredictor.scala (train or load the TextClassifier model, broadcast it,
register ``textClassifier`` as a Spark SQL UDF over the text column, then ``select ... where textClassifier(text)
= k``), Utils.scala (tokenise / shape / vectorise exactly like training).

Here the DataFrame is pandas and the UDF is a vectorised column function: texts are vectorised and scored in
batches of ``--batchSize`` (one forward per batch on the GPU, not one call per row), which is what the Spark UDF
amortises with its broadcast model.
"""
import argparse

import torch

from ._common import device_of
from .text_classifier import analyze_texts, build_model, synthetic_corpus, vectorize


class TextClassifierUDF:
    """Callable ``udf(pandas.Series[str]) -> pandas.Series[int]`` (1-based class)."""

    def __init__(self, model, word2index, seq_len, dim, device, batch=128):
        self.model, self.word2index, self.seq_len, self.dim = model.to(device), word2index, seq_len, dim
        self.device, self.batch = device, batch
        self.model.evaluate()

    def __call__(self, texts):
        import pandas as pd

        texts = list(texts)
        preds = []
        with torch.no_grad():
            for i in range(0, len(texts), self.batch):
                x = torch.stack(vectorize(texts[i:i + self.batch], self.word2index, self.seq_len, self.dim, {}))
                preds += (self.model.forward(x.to(self.device)).float().argmax(1) + 1).cpu().tolist()
        return pd.Series(preds)


def run(args):
    import pandas as pd

    from .. import nn
    from ..dataset.core import DataSet, Sample
    from ..optim import Adagrad, Optimizer, Trigger

    dev = device_of(args.device)
    texts, labels, classes = synthetic_corpus(n_docs=200, classes=args.classes)
    word2index = analyze_texts(texts, 20000, 0)
    feats = vectorize(texts, word2index, args.seqLen, args.dim, {})
    model = build_model(args.dim, args.seqLen, classes)
    opt = Optimizer(model=model, dataset=DataSet.array([Sample(f, torch.tensor([l])) for f, l in zip(feats, labels)]),
                    criterion=nn.ClassNLLCriterion(), batchSize=32)
    opt.device = dev
    opt.setOptimMethod(Adagrad(learningRate=0.05)).setEndWhen(Trigger.maxEpoch(args.epochs))
    model = opt.optimize()
    udf = TextClassifierUDF(model, word2index, args.seqLen, args.dim, dev)
    test_texts, test_labels, _ = synthetic_corpus(n_docs=60, classes=args.classes, seed=11)
    df = pd.DataFrame({"filename": [f"doc{i}" for i in range(len(test_texts))], "text": test_texts})
    df["textClassifier"] = udf(df["text"])                       # withColumn("textLabel", udf(col("text")))
    hits = df[df["textClassifier"] == args.queryClass]           # "select * from df where textLabel = k"
    acc = float((df["textClassifier"].values == [int(l) for l in test_labels]).mean())
    return {"rows": len(df), "query_rows": len(hits), "accuracy": acc}


def build_parser():
    p = argparse.ArgumentParser(prog="udfpredictor")
    p.add_argument("--classes", type=int, default=4)
    p.add_argument("--seqLen", type=int, default=72)
    p.add_argument("--dim", type=int, default=32)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--queryClass", type=int, default=2)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
