"""Training runtimes: Optimizer (factory + fluent configuration), LocalOptimizer, DistriOptimizer.

Reference: S/optim/Optimizer.scala:47-699 (setters :93-470, factory :602-689), AbstractOptimizer.scala
(validate :93, checkpoint :205), DistriOptimizer.scala:43-1016 (iteration loop :97-517, retry :881-963,
straggler drop :171-178, :421-449), LocalOptimizer.scala:40-295, ParallelOptimizer.scala:42-791.

MI355X execution model: one process per GPU (torchrun) — "local[N]" = N ranks. Every rank runs the same
loop over its shard of the data (DataSet.rdd); one iteration is a TrainStep (forward/backward on the
native kernels, reduce-scatter of the flat gradient over RCCL, fused optimizer on this rank's ZeRO-1 shard,
all-gather of the bf16 compute weights). Scalars (loss, record counts, validation results) are all-reduced
in one small collective at logging / validation points instead of per-iteration driver accumulators.
"""
import logging
import math
import os
import time

import torch

from ..dataset.core import AbstractDataSet, DataSet, MiniBatch, SampleToMiniBatch
from ..utils.engine import Engine
from ..utils.table import Table
from .metrics import Metrics
from .sgd import SGD
from .train_step import TrainStep
from .trigger import Trigger

logger = logging.getLogger("bigdl_amd.optim")


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


class Optimizer:
    """Base class + factory. ``Optimizer(model, dataset, criterion, batchSize)`` returns a DistriOptimizer
    when the dataset is distributed (or the job has several ranks), else a LocalOptimizer."""

    def __new__(cls, *args, **kw):
        if cls is Optimizer:
            ds = kw.get("dataset", args[1] if len(args) > 1 else None)
            dist = (isinstance(ds, AbstractDataSet) and ds.isDistributed()) or Engine.world_size() > 1
            target = DistriOptimizer if dist else LocalOptimizer
            obj = object.__new__(target)
            return obj
        return object.__new__(cls)

    def __init__(self, model, dataset, criterion, batchSize=None, optimMethod=None, endTrigger=None,
                 featurePaddingParam=None, labelPaddingParam=None):
        self.model = model
        self.criterion = criterion
        self.batchSize = batchSize
        self.dataset = self._wrap_dataset(dataset, batchSize, featurePaddingParam, labelPaddingParam)
        self.optimMethods = {model.getName(): optimMethod or SGD()}
        self.endWhen = endTrigger or Trigger.maxEpoch(1)
        self.state = Table()
        self.validationTrigger = None
        self.validationDataSet = None
        self.validationMethods = None
        self.checkpointTrigger = None
        self.checkpointPath = None
        self.isOverWrite = False
        self.trainSummary = None
        self.validationSummary = None
        self.dropPercentage = 0.0
        self.maxDropPercentage = 0.0
        self.computeThresholdbatchSize = 100
        self.warmupIterationNum = 200
        self.constantClip = None
        self.l2NormClip = None
        self.logInterval = int(os.environ.get("BIGDL_LOG_INTERVAL", "10"))
        self.retryTimes = int(Engine.getProperty("bigdl.failure.retryTimes", 5))
        self.compress = Engine.getProperty("bigdl.compress", None)
        self.metrics = Metrics()
        self._step = None
        self.device = Engine.device()

    @staticmethod
    def _wrap_dataset(dataset, batchSize, fpad=None, lpad=None):
        if dataset is None:
            return None
        if isinstance(dataset, (list, tuple)):
            dataset = DataSet.rdd(dataset) if Engine.world_size() > 1 else DataSet.array(dataset)
        if batchSize is not None:
            return dataset.transform(SampleToMiniBatch(batchSize, fpad, lpad))
        return dataset

    # ---------------------------------------------------------------- fluent setters (reference API)
    def setValidation(self, trigger, dataset, vMethods, batchSize=None):
        self.validationTrigger = trigger
        self.validationDataSet = self._wrap_dataset(dataset, batchSize or self.batchSize)
        self.validationMethods = list(vMethods)
        return self

    def setCheckpoint(self, path, trigger):
        os.makedirs(path, exist_ok=True)
        self.checkpointPath = path
        self.checkpointTrigger = trigger
        return self

    def overWriteCheckpoint(self):
        self.isOverWrite = True
        return self

    def setTrainSummary(self, summary):
        self.trainSummary = summary
        return self

    def setValidationSummary(self, summary):
        self.validationSummary = summary
        return self

    def setModel(self, model):
        self.model = model
        return self

    def setTrainData(self, dataset, batchSize=None, featurePaddingParam=None, labelPaddingParam=None):
        self.dataset = self._wrap_dataset(dataset, batchSize or self.batchSize, featurePaddingParam,
                                          labelPaddingParam)
        return self

    def setCriterion(self, criterion):
        self.criterion = criterion
        return self

    def setState(self, state):
        self.state = state
        return self

    def setOptimMethod(self, method):
        self.optimMethods = {self.model.getName(): method}
        return self

    def setOptimMethods(self, methods):
        self.optimMethods = dict(methods)
        return self

    def setEndWhen(self, trigger):
        self.endWhen = trigger
        return self

    def setDropModuleProperty(self, dropPercentage, maxDropPercentage, batchsize=100, warmupIteration=200):
        self.dropPercentage, self.maxDropPercentage = dropPercentage, maxDropPercentage
        self.computeThresholdbatchSize, self.warmupIterationNum = batchsize, warmupIteration
        return self

    def setConstantGradientClipping(self, min, max):
        self.constantClip = (min, max)
        return self

    def setGradientClippingByl2Norm(self, clipNorm):
        self.l2NormClip = clipNorm
        return self

    def disableGradientClipping(self):
        self.constantClip = None
        self.l2NormClip = None
        return self

    def setLogInterval(self, n):
        self.logInterval = n
        return self

    def reserveOptim(self, reserve):
        self._reserve = reserve
        return self

    def prepareInput(self):
        pass

    # ---------------------------------------------------------------- core loop
    _overlap = False

    def _optim_method(self):
        if len(self.optimMethods) != 1:
            raise NotImplementedError("per-submodule optim methods: use ParallelOptimizer")
        return next(iter(self.optimMethods.values()))

    def _make_step(self, comm=None):
        return TrainStep(self.model, self.criterion, self._optim_method(), device=self.device, comm=comm,
                         compress=self.compress, overlap=self._overlap)

    def _processors(self):
        """Clipping as ParameterProcessors (reference ParameterOperations.scala), constant clipping first."""
        from ..parallel.processors import ConstantClippingProcessor, L2NormClippingProcessor

        out = []
        if self.constantClip is not None:
            out.append(ConstantClippingProcessor(*self.constantClip))
        if self.l2NormClip is not None:
            out.append(L2NormClippingProcessor(self.l2NormClip))
        return out

    def _clip(self, step):
        for p in self._processors():
            p(step.g_shard, step.comm)

    def _header(self, epoch, n, iteration, wall):
        return f"[Epoch {epoch} {n}/{self._epoch_size()}][Iteration {iteration}][Wall Clock {wall:.3f}s]"

    def _epoch_size(self):
        return self.dataset.size()

    def optimize(self):
        retries = 0
        while True:
            try:
                return self._optimize_once()
            except KeyboardInterrupt:
                raise
            except Exception:
                retries += 1
                if retries > self.retryTimes or self.checkpointPath is None:
                    raise
                logger.exception("training failed; retrying from the last checkpoint (%d/%d)", retries,
                                 self.retryTimes)
                self._restore_latest()

    def _restore_latest(self):
        from ..utils.serializer import load_module
        from .optim_method import OptimMethod

        files = [f for f in os.listdir(self.checkpointPath) if f.startswith("model.")]
        if not files:
            return
        last = max(files, key=lambda f: int(f.split(".")[1]) if f.split(".")[1].isdigit() else -1)
        suffix = last.split(".", 1)[1]
        m = load_module(os.path.join(self.checkpointPath, last))
        self.model = m
        om = os.path.join(self.checkpointPath, f"optimMethod.{suffix}")
        if os.path.exists(om):
            self.optimMethods = {m.getName(): OptimMethod.load(om)}
        self._step = None

    def _optimize_once(self):
        st = self.state
        st["epoch"] = st.get("epoch", 1)
        st["neval"] = st.get("neval", 1)
        st["recordsProcessedThisEpoch"] = st.get("recordsProcessedThisEpoch", 0)
        om = self._optim_method()
        om.state["epoch"] = st["epoch"]
        om.state["neval"] = st["neval"]
        if self._step is None:
            self._step = self._make_step()
        step = self._step
        world = step.comm.world
        rank = step.comm.rank
        it = iter(self.dataset.data(train=True))
        wall0 = time.perf_counter()
        pending = []  # (iteration, loss tensor, records)
        while not self.endWhen(st):
            t0 = time.perf_counter()
            batch = next(it)
            batch = batch.to(step.device, non_blocking=True)
            self.metrics.add("data fetch time", time.perf_counter() - t0)
            t1 = time.perf_counter()
            step.zero_grad()
            loss = step.forward_backward(batch.getInput(), batch.getTarget())
            if step.bucketed is not None:          # ParallelOptimizer: buckets already in flight
                self._clip(step)
                step.bucketed.update(loss)
            else:
                step.comm.reduce_scatter_gradients(step.g, out=step.g_shard)
                if self.constantClip is not None or self.l2NormClip is not None:
                    self._clip(step)
                om.optimize(lambda _: (loss, step.g_shard), step.w_shard)
                if world > 1:
                    step.comm.all_gather_weights(step.w16 if step.w16 is not None else step.w)
            self.metrics.add("computing time", time.perf_counter() - t1)
            records = batch.size() * world
            pending.append((st["neval"], loss.detach() if torch.is_tensor(loss) else torch.tensor(float(loss)),
                            records))
            st["neval"] += 1
            om.state["neval"] = st["neval"]
            st["recordsProcessedThisEpoch"] += records
            need_loss = (self.logInterval > 0 and (st["neval"] - 1) % self.logInterval == 0)
            if need_loss or self.endWhen(st) or isinstance(self.endWhen, Trigger.minLoss(0).__class__):
                self._flush_losses(step, pending, wall0)
                pending = []
            if st["recordsProcessedThisEpoch"] >= self._epoch_size():
                st["epoch"] += 1
                om.state["epoch"] = st["epoch"]
                st["recordsProcessedThisEpoch"] = 0
            self._validate(step)
            self._checkpoint(step)
        if pending:
            self._flush_losses(step, pending, wall0)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        return self.model

    def _flush_losses(self, step, pending, wall0):
        if not pending:
            return
        losses = torch.stack([p[1].float().reshape(()) for p in pending]).to(step.device)
        if step.comm.world > 1:
            step.comm.all_reduce_scalar(losses)
            losses = losses / step.comm.world
        vals = losses.cpu().tolist()
        st = self.state
        wall = time.perf_counter() - wall0
        for (itn, _, rec), v in zip(pending, vals):
            st["Loss"] = v
            if self.trainSummary is not None and step.comm.rank == 0:
                self._save_summary(itn, v, rec * step.comm.world / max(wall / len(pending), 1e-9))
        if step.comm.rank == 0:
            thr = sum(p[2] for p in pending) / max(self.metrics.get("computing time") * len(pending), 1e-9)
            logger.info("%s Trained %d records in %.4f seconds. Throughput is %.1f records/second. Loss is %.5f. %s",
                        self._header(st["epoch"], st["recordsProcessedThisEpoch"], st["neval"] - 1, wall),
                        pending[-1][2], self.metrics.get("computing time"), thr, vals[-1],
                        self._optim_method().getHyperParameter())

    def _save_summary(self, itn, loss, throughput):
        """Reference AbstractOptimizer.saveSummary (S/optim/AbstractOptimizer.scala:47): scalar tags gated by
        their TrainSummary triggers, parameter histograms under the "Parameters" trigger."""
        ts = self.trainSummary
        trig_state = dict(self.state.items()) if hasattr(self.state, "items") else dict(self.state)
        trig_state["neval"] = itn + 1
        values = {"Loss": loss, "Throughput": throughput,
                  "LearningRate": -self._optim_method().getLearningRate()}
        triggers = ts.getScalarTriggers() if hasattr(ts, "getScalarTriggers") else [("Loss", None)]
        for tag, trig in triggers:
            if tag in values and (trig is None or trig(trig_state)):
                ts.addScalar(tag, values[tag], itn)
        ptrig = ts.getSummaryTrigger("Parameters") if hasattr(ts, "getSummaryTrigger") else None
        if ptrig is not None and ptrig(trig_state):
            for m in self.model.flattened_layers():
                if m.modules_list():
                    continue
                for w, g in m._params:
                    t, gt = getattr(m, w, None), getattr(m, g, None)
                    if t is not None:
                        ts.addHistogram(f"{m.getName()}/{w}", t, itn)
                    if gt is not None:
                        ts.addHistogram(f"{m.getName()}/{g}", gt, itn)

    def _validate(self, step):
        if self.validationTrigger is None or self.validationDataSet is None:
            return
        if not self.validationTrigger(self.state):
            return
        from .evaluator import evaluate_dataset

        results = evaluate_dataset(self.model, self.validationDataSet, self.validationMethods, device=step.device)
        self.model.training()
        for r, m in zip(results, self.validationMethods):
            v, n = r.result()
            if step.comm.rank == 0:
                logger.info("%s is %s", m.format(), r)
            self.state["score"] = v
            if self.validationSummary is not None and step.comm.rank == 0:
                self.validationSummary.addScalar(m.format(), v, self.state["neval"] - 1)
        self._last_validation = results

    def _checkpoint(self, step):
        if self.checkpointTrigger is None or self.checkpointPath is None:
            return
        if not self.checkpointTrigger(self.state):
            return
        if step.comm.world > 1 and step.w16 is None:
            pass  # fp32 weights already all-gathered each iteration
        suffix = "" if self.isOverWrite else f".{self.state['neval'] - 1}"
        if step.comm.rank == 0:
            self.model.saveModule(os.path.join(self.checkpointPath, f"model{suffix or '.latest'}"), overWrite=True)
            self._optim_method().save(os.path.join(self.checkpointPath, f"optimMethod{suffix or '.latest'}"),
                                      overWrite=True)
        d = _dist()
        if d is not None:
            d.barrier()


class LocalOptimizer(Optimizer):
    """Single-process training (reference LocalOptimizer.scala:40-295)."""


class DistriOptimizer(Optimizer):
    """Synchronous data-parallel training over all ranks of the job (reference DistriOptimizer.scala)."""

    def _epoch_size(self):
        return self.dataset.size()


class ParallelOptimizer(DistriOptimizer):
    """Data-parallel training with layer-wise bucketed gradient reduce-scatter overlapped with backward
    (reference ParallelOptimizer.scala:42-791; mechanism in parallel/bucketed.py)."""

    _overlap = True

    def __new__(cls, *args, **kw):
        return object.__new__(cls)

    def _clip(self, step):
        if self.constantClip is not None or self.l2NormClip is not None:
            raise NotImplementedError("gradient clipping needs the whole gradient; use DistriOptimizer")


def create(model, training_set, criterion, end_trigger=None, batch_size=32, optim_method=None, **kw):
    """Python-API style factory (reference P/optim/optimizer.py:874 ``Optimizer.create``)."""
    return Optimizer(model, training_set, criterion, batch_size, optim_method, end_trigger)


Optimizer.create = staticmethod(create)


AbstractOptimizer = Optimizer   # reference AbstractOptimizer.scala:33 — shared validate / checkpoint / summary logic
