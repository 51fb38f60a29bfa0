"""Evaluation / validation (reference S/optim/Evaluator.scala:30-111, Validator.scala, DistriValidator.scala,
LocalValidator.scala, AbstractModule.evaluate :856-918).

Every rank evaluates its shard; ValidationResults are merged with one all-reduce of their tensor form
(the analogue of the reference's ``reduce(ValidationResult +)`` Spark action)."""
import torch

from ..dataset.core import AbstractDataSet, DataSet, MiniBatch, SampleToMiniBatch
from ..utils.engine import Engine


def _merge_distributed(results):
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return results
    out = []
    for r in results:
        if hasattr(r, "to_tensor") and hasattr(type(r), "from_tensor"):
            t = r.to_tensor().to(torch.float64)
            dev = torch.device("cuda", Engine.local_rank()) if dist.get_backend() == "nccl" else torch.device("cpu")
            t = t.to(dev)
            dist.all_reduce(t)
            out.append(type(r).from_tensor(t.cpu()))
        else:
            gathered = [None] * dist.get_world_size()
            dist.all_gather_object(gathered, r)
            acc = gathered[0]
            for g in gathered[1:]:
                acc = acc + g
            out.append(acc)
    return out


def evaluate_dataset(model, dataset, vMethods, batchSize=None, device=None):
    if device is None:
        device = model.device
    if isinstance(dataset, (list, tuple)):
        dataset = DataSet.array(dataset, shuffle=False)
    if batchSize is not None:
        dataset = dataset.transform(SampleToMiniBatch(batchSize))
    was_train = model.isTraining()
    model.evaluate()
    results = None
    with torch.no_grad():
        for batch in dataset.data(train=False):
            if not isinstance(batch, MiniBatch):
                raise TypeError("evaluate: dataset must yield MiniBatches (use a batchSize)")
            b = batch.to(device)
            out = model.forward(b.getInput())
            rs = [m(out, b.getTarget()) for m in vMethods]
            results = rs if results is None else [a + r for a, r in zip(results, rs)]
    if was_train:
        model.training()
    if results is None:
        results = []
    return _merge_distributed(results)


def evaluate_module(model, dataset, vMethods, batchSize=None):
    """``module.evaluate(dataset, vMethods, batchSize)`` → list of (ValidationResult, ValidationMethod)."""
    res = evaluate_dataset(model, dataset, vMethods, batchSize)
    return list(zip(res, vMethods))


class Evaluator:
    def __init__(self, model):
        self.model = model

    def test(self, dataset, vMethods, batchSize=None):
        return evaluate_module(self.model, dataset, vMethods, batchSize)


class Validator(Evaluator):
    pass


LocalValidator = Validator
DistriValidator = Validator
