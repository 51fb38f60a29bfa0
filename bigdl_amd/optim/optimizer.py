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
import copy
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
        self.compress = Engine.getProperty("bigdl.compress", "auto")
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
    _expand = False
    _priorities = None

    def _optim_method(self):
        return next(iter(self.optimMethods.values()))

    def _make_step(self, comm=None):
        # gradient bucket size for the bucketed overlap (reference property bigdl.parallelOptimizer.parameterBlocks
        # counts blocks; buckets here are sized in elements: 8M fp32 = 32 MB runs the xGMI links near their rate)
        bucket = int(Engine.getProperty("bigdl.parallelOptimizer.bucketElems", 8 << 20) or (8 << 20))
        return TrainStep(self.model, self.criterion, dict(self.optimMethods), device=self.device, comm=comm,
                         compress=self.compress, overlap=self._overlap, processors=self._processors(),
                         expand_methods=self._expand, priorities=self._priorities, bucket_elems=bucket)

    def _processors(self):
        """Clipping as ParameterProcessors (reference ParameterOperations.scala), constant clipping first."""
        from ..parallel.processors import ConstantClippingProcessor, L2NormClippingProcessor

        out = []
        if self.constantClip is not None:
            out.append(ConstantClippingProcessor(*self.constantClip))
        if self.l2NormClip is not None:
            out.append(L2NormClippingProcessor(self.l2NormClip))
        return out

    def _header(self, epoch, n, iteration, wall):
        return f"[Epoch {epoch} {n}/{self._epoch_size()}][Iteration {iteration}][Wall Clock {wall:.3f}s]"

    def _epoch_size(self):
        return self.dataset.size()

    def optimize(self):
        """Train until ``endWhen``; returns the model holding the exact trained weights on every rank.

        Failure policy (reference DistriOptimizer.scala:881-963): argument errors propagate; any other error is
        retried from the latest checkpoint (model + per-method state, each method's history cleared) up to
        ``bigdl.failure.retryTimes``. In a multi-rank job a failing rank cannot re-enter the collectives of the
        others, so the error propagates and the launcher (torch.distributed.run --max-restarts) restarts the
        whole job, which resumes from the same checkpoint through ``bigdl.failure.resume``."""
        retries = 0
        if self.checkpointPath is not None and Engine.getProperty("bigdl.failure.resume", None) and \
                self._restore_latest():
            logger.info("resumed from the latest checkpoint in %s", self.checkpointPath)
        if self._step is None and not getattr(self, "_resumed", False):
            for om in self.optimMethods.values():      # reference optimize(): fresh optimizer history
                om.clearHistory()
        while True:
            try:
                return self._optimize_once()
            except (KeyboardInterrupt, ValueError, TypeError):
                raise
            except Exception:
                retries += 1
                if retries > self.retryTimes or self.checkpointPath is None or Engine.world_size() > 1:
                    raise
                logger.exception("training failed; retrying from the last checkpoint (%d/%d)", retries,
                                 self.retryTimes)
                if self._restore_latest():
                    for om in self.optimMethods.values():   # reference :946 newOptimMethod.clearHistory()
                        om.clearHistory()
                    self._resume_state = None

    @staticmethod
    def _latest(path, prefix):
        best, best_n = None, -1
        for f in os.listdir(path):
            if not f.startswith(prefix + "."):
                continue
            suf = f[len(prefix) + 1:]
            n = int(suf) if suf.isdigit() else (10 ** 12 if suf == "latest" else -1)
            if n > best_n:
                best, best_n = f, n
        return best

    def _restore_latest(self):
        """Reload the newest model and every method from ``checkpointPath`` (history cleared like the
        reference). Returns True when a model snapshot was found."""
        from ..utils.serializer import load_module
        from .optim_method import OptimMethod

        last = self._latest(self.checkpointPath, "model")
        if last is None:
            return False
        m = load_module(os.path.join(self.checkpointPath, last))
        old = self.model
        self.model = m
        methods = {}
        for name, om in self.optimMethods.items():
            key = m.getName() if name == old.getName() else name
            f = self._latest(self.checkpointPath, f"optimMethod-{name}")
            nm = OptimMethod.load(os.path.join(self.checkpointPath, f)) if f else om
            methods[key] = nm
        # the checkpoint holds each method's FULL per-element state (gather_optim_state); the TrainStep built next
        # slices it into this rank's pieces on its device (load_optim_state), so the method objects it owns start
        # without per-element tensors
        full = {}
        for key, nm in methods.items():
            full[key] = copy.deepcopy(nm)
            for k in list(nm.state.keys()):
                if torch.is_tensor(nm.state[k]) and nm.state[k].dim() >= 1:
                    del nm.state[k]
        self._resume_state = full
        self.optimMethods = methods
        first = next(iter(methods.values()))
        for k in ("epoch", "neval"):
            if first.state.get(k) is not None:
                self.state[k] = first.state[k]
        self._resumed = True
        self._step = None
        return True

    def _sync_states(self, st):
        for om in self.optimMethods.values():
            om.state["epoch"] = st["epoch"]
            om.state["neval"] = st["neval"]
            if "Loss" in st.keys():
                om.state["Loss"] = st["Loss"]
            if "score" in st.keys():
                om.state["score"] = st["score"]

    def _optimize_once(self):
        st = self.state
        st["epoch"] = st.get("epoch", 1)
        st["neval"] = st.get("neval", 1)
        st["recordsProcessedThisEpoch"] = st.get("recordsProcessedThisEpoch", 0)
        self._sync_states(st)
        if self._step is None:
            self._step = self._make_step()
            if getattr(self, "_resume_state", None):
                self._step.load_optim_state(self._resume_state)
                self._resume_state = None
        step = self._step
        world = step.comm.world
        drop = _StragglerDrop(self, world) if self.dropPercentage > 0 else None
        self._drop = drop
        if drop is not None:
            drop.forced = getattr(self, "_forced_votes", None)
        step.defer_sync = drop is not None
        from .device_feed import DeviceFeed

        it = DeviceFeed(iter(self.dataset.data(train=True)), step.device)
        wall0 = time.perf_counter()
        pending = []  # (iteration, loss tensor, records)
        # liveness: a rank stuck (dead peer in a collective, hung kernel) exits instead of hanging the job
        from ..utils.affinity import StepWatchdog
        wd_s = float(Engine.getProperty("bigdl.step.timeout", 0) or 0)
        watchdog = StepWatchdog(wd_s).start() if wd_s > 0 else None
        try:
            self._train_iterations(st, step, world, drop, it, wall0, pending, watchdog)
        finally:
            it.close()
            if self._graph is not None:
                torch.cuda.synchronize()
                self._graph.release()
                self._graph = None
            if watchdog is not None:
                watchdog.stop()
        step.gather_model()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        return self.model

    _graph = None
    _iteration_hook = None       # callable(neval) after every iteration (benchmarks, tests)

    def _use_graph(self, step, drop):
        """Capture the iteration in HIP graphs (reference per-iteration task launch, DistriOptimizer.scala:204-396)
        when the device is a GPU, every update is graph-safe (plain SGD), no straggler drop is active and
        ``bigdl.optim.graph`` is not "false"."""
        from .graphed import graphable

        flag = str(Engine.getProperty("bigdl.optim.graph", "auto")).lower()
        if step.comm.active:
            import torch.distributed as dist

            if dist.get_backend(step.comm.group) != "nccl":
                return False        # host-side (gloo) collectives cannot be replayed between graph segments
        return step.device.type == "cuda" and drop is None and flag not in ("0", "false", "no") and graphable(step)

    def _graph_keep(self, step, eager_ms, graph_ms, host_ms=0.0):
        """``bigdl.optim.graph`` = auto (default): keep the captured iteration only if its replays are faster on the
        device than the timed eager iteration (a launch-bound model gains from the graph; a large-batch model whose
        eager iteration overlaps its weight-gradient side stream better than the graph's replay does not). The
        timings are averaged over ranks so every rank takes the same path."""
        flag = str(Engine.getProperty("bigdl.optim.graph", "auto")).lower()
        if flag != "auto":
            return True
        t = torch.tensor([eager_ms, graph_ms, host_ms], device=step.device)
        if step.comm.world > 1:
            step.comm.all_reduce_scalar(t)
        eager_ms, graph_ms, host_ms = (float(v) for v in t.cpu())
        # eager only when clearly faster and the host has headroom (an eager iteration whose enqueue takes more than
        # half its device time turns host-bound on a busier CPU; a replay needs ~1 ms of host time)
        keep = not (eager_ms < 0.97 * graph_ms and host_ms < 0.5 * eager_ms)
        w = max(1, step.comm.world)
        logger.info("iteration: eager %.3f ms on the device (%.3f ms host), HIP graph %.3f ms -> %s", eager_ms / w,
                    host_ms / w, graph_ms / w, "graph" if keep else "eager")
        self.graph_decision = {"eager_ms": eager_ms / w, "graph_ms": graph_ms / w, "host_ms": host_ms / w,
                               "graph": keep}
        return keep

    def _train_iterations(self, st, step, world, drop, it, wall0, pending, watchdog):
        use_graph = self._use_graph(step, drop)
        eager_done = 0
        timing = {}            # device events: the 2nd eager iteration and graph replays 2-3 (auto mode)
        while not self.endWhen(st):
            t0 = time.perf_counter()
            batch = next(it)        # device-resident; its copy was issued during the previous iteration
            fetch = time.perf_counter() - t0
            self.metrics.add("data fetch time", fetch)
            t1 = time.perf_counter()
            finished = None
            x, y = batch.getInput(), batch.getTarget()
            g = self._graph
            if (use_graph and g is None and eager_done >= 2 and isinstance(x, torch.Tensor)
                    and isinstance(y, torch.Tensor)):
                from .graphed import GraphedTrainStep

                try:
                    g = self._graph = GraphedTrainStep(step, x, y, prewarmed=True)
                    logger.info("training iteration captured in %d HIP graph segment(s)", len(g.graph))
                except Exception as e:  # noqa: BLE001 - fall back to eager launches
                    from ..ops import side_stream

                    logger.warning("HIP graph capture failed (%s: %s); eager iterations", type(e).__name__, e)
                    side_stream.reset()
                    use_graph, g, self._graph = False, None, None
            if g is not None:
                if isinstance(x, torch.Tensor) and g.matches(x, y):
                    nrep = timing.get("replays", 0)
                    timing["replays"] = nrep + 1
                    if nrep == 1 and "e1" in timing:
                        timing["g1"] = torch.cuda.Event(enable_timing=True)
                        timing["g1"].record()
                    loss = g.replay(x, y).detach().clone()   # the graph's loss buffer is rewritten every replay
                    if nrep == 2 and "g1" in timing:
                        timing["g3"] = torch.cuda.Event(enable_timing=True)
                        timing["g3"].record()
                        timing["g3"].synchronize()
                        graph_ms = timing["g1"].elapsed_time(timing["g3"]) / 2
                        eager_ms = timing["e0"].elapsed_time(timing["e1"])
                        if not self._graph_keep(step, eager_ms, graph_ms, timing.get("host_ms", 0.0)):
                            g.release()
                            g, self._graph, use_graph = None, None, False
                            torch.cuda.synchronize()
                            torch.cuda.empty_cache()     # the graph's private pool back to the device
                else:
                    loss = g.eager(x, y)
                n_ok = 1
            elif drop is not None and drop.timed_out(fetch):
                # straggler: the deadline passed before compute could start — contribute nothing this iteration
                loss = torch.zeros(())          # host placeholder: nothing queued behind a slow device
                finished = 0.0
            else:
                if eager_done == 1 and use_graph:
                    timing["e0"] = torch.cuda.Event(enable_timing=True)
                    timing["e0"].record()
                    timing["h0"] = time.perf_counter()
                step.zero_grad()
                if drop is not None:
                    # straggler cancellation: past the deadline every module boundary raises StragglerTimeout, so
                    # a late rank abandons the rest of its forward / backward and joins the collective on time
                    loss, finished = drop.run(step, x, y, t0)
                else:
                    loss = step.forward_backward_step(x, y)
                eager_done += 1
            if g is not None:
                pass
            elif finished is not None:
                step.min_finished = world * (1.0 - self.maxDropPercentage)
                n_ok = drop.record(step.sync_and_update(loss, finished=finished), finished)
            else:
                step.sync_and_update(loss)
                n_ok = 1
                if "e0" in timing and "e1" not in timing:
                    timing["e1"] = torch.cuda.Event(enable_timing=True)
                    timing["e1"].record()
                    timing["host_ms"] = (time.perf_counter() - timing["h0"]) * 1e3
            if finished is None or finished:
                step.throttle()      # the host stays at most TrainStep.MAX_INFLIGHT iterations ahead of the device
                # device-timed phases of the iterations the device finished meanwhile (optim/phase_timer.py)
                from .phase_timer import METRIC_NAMES

                for ph in getattr(step, "phase_done", None) or ():
                    for k, name in METRIC_NAMES.items():
                        self.metrics.add(name, ph[k] / 1e3)
            # (a dropped rank skips it: its backlog must not hold the host, the pacer bounds it next iteration)
            self.metrics.add("computing time", time.perf_counter() - t1)
            records = batch.size() * world
            pending.append((st["neval"], loss.detach() if torch.is_tensor(loss) else torch.tensor(float(loss)),
                            records))
            st["neval"] += 1
            st["recordsProcessedThisEpoch"] += records
            self._sync_states(st)
            if drop is not None:
                with drop.control():
                    drop.maybe_update_threshold(step, st["neval"] - 1)
            need_loss = (self.logInterval > 0 and (st["neval"] - 1) % self.logInterval == 0)
            if need_loss or self.endWhen(st) or isinstance(self.endWhen, Trigger.minLoss(0).__class__):
                if drop is not None:
                    with drop.control():
                        self._flush_losses(step, pending, wall0)
                else:
                    self._flush_losses(step, pending, wall0)
                pending = []
            if st["recordsProcessedThisEpoch"] >= self._epoch_size():
                st["epoch"] += 1
                st["recordsProcessedThisEpoch"] = 0
                self._sync_states(st)
            self._validate(step)
            self._checkpoint(step)
            del n_ok
            if self._iteration_hook is not None:
                self._iteration_hook(st["neval"] - 1)
            if watchdog is not None:
                watchdog.kick()
        if pending:
            self._flush_losses(step, pending, wall0)

    def _flush_losses(self, step, pending, wall0):
        if not pending:
            return
        losses = torch.stack([p[1].float().reshape(()).to(step.device) for p in pending])
        if step.comm.world > 1:
            step.comm.all_reduce_scalar(losses)
            losses = losses / step.comm.world
        if losses.is_cuda:          # poll, not a blocking wait (train_step.wait_event)
            from .train_step import wait_event

            ev = torch.cuda.Event()
            ev.record()
            wait_event(ev)
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

        step.flush()
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
        """Reference AbstractOptimizer.checkpoint: the gathered model (getModel) as ``model.<neval>`` and every
        method as ``optimMethod-<name>.<neval>`` with its FULL optimizer state (gathered from every rank's
        shard pieces, so a checkpoint restores on any number of ranks). Collective."""
        if self.checkpointTrigger is None or self.checkpointPath is None:
            return
        if not self.checkpointTrigger(self.state):
            return
        step.gather_model()
        methods = step.gather_optim_state()
        neval = self.state["neval"] - 1
        suffix = ".latest" if self.isOverWrite else f".{neval}"
        if step.comm.rank == 0:
            self.model.saveModule(os.path.join(self.checkpointPath, f"model{suffix}"), overWrite=True)
            for name, om in methods.items():
                om.state["epoch"] = self.state["epoch"]
                om.state["neval"] = self.state["neval"]
                om.save(os.path.join(self.checkpointPath, f"optimMethod-{name}{suffix}"), overWrite=True)
        d = _dist()
        if d is not None:
            d.barrier()


class _StragglerDrop:
    """Straggler drop (reference DistriOptimizer.scala:171-178, 241-246, 343, 421-449).

    Every rank is one "sub-model". After ``warmupIterationNum`` iterations, every ``computeThresholdbatchSize``
    iterations the per-iteration times of all ranks are gathered and the threshold is set to the k-th largest
    (k = dropPercentage · batch · ranks, less the drops already seen). A rank whose iteration exceeds the
    threshold contributes a zero gradient with weight 0; the gradient is averaged over the ranks that finished
    and the update is skipped when fewer than (1 - maxDropPercentage) of the ranks did."""

    def __init__(self, opt, world):
        self.opt = opt
        self.world = world
        self.times = []
        self.threshold = float("inf")
        self.dropped = 0
        self.iteration = 0
        self.cancelled = 0
        self.history = []        # this rank's vote per iteration (1 finished, 0 dropped)
        self.forced = None       # {iteration: vote}: replay a recorded drop pattern (tests)
        self._ctrl = None

    def control(self):
        """Stream context for the straggler bookkeeping (votes, threshold gathers, loss flushes): a stream that does
        not wait for the compute stream, so a rank with a device backlog answers these collectives on time. Every
        tensor it reads is complete: finished iterations were drained (``run``), dropped ones left host placeholders."""
        import contextlib

        if not torch.cuda.is_available() or self.opt._step is None or self.opt._step.device.type != "cuda":
            return contextlib.nullcontext()
        if self._ctrl is None:
            from ..ops import side_stream

            self._ctrl = side_stream.peer_stream(self.opt._step.device)
        return torch.cuda.stream(self._ctrl)
    def timed_out(self, elapsed):
        return self.forced is None and elapsed > self.threshold

    def finished(self, elapsed):
        self.times.append(elapsed)
        return 0.0 if elapsed > self.threshold else 1.0

    def run(self, step, x, y, t0):
        """forward + backward under the iteration deadline t0 + threshold. Returns (loss, finished weight).

        GPU ranks are paced on device progress (nn/abstractnn.py DevicePacer): the iteration counts as finished only
        once the device has executed all of its backward, and the time recorded for the threshold is that
        device-inclusive time, so a slow GPU (not only a slow host) is timed out and dropped."""
        from ..nn.abstractnn import STRAGGLER_DEADLINE, STRAGGLER_PACER, DevicePacer, StragglerTimeout

        if self.forced is not None:         # replay of a recorded drop pattern: same math, no clocks
            loss = step.forward_backward_step(x, y)
            v = float(self.forced.get(self.iteration, 1.0))
            self.times.append(0.0)
            return (loss, 1.0) if v else (torch.zeros(()), 0.0)
        armed = self.threshold != float("inf")
        deadline = t0 + self.threshold if armed else float("inf")
        pacer = DevicePacer() if step.device.type == "cuda" else None
        if armed:
            STRAGGLER_DEADLINE[0] = deadline
            STRAGGLER_PACER[0] = pacer
        try:
            loss = step.forward_backward_step(x, y)
            if pacer is not None:
                pacer.drain(deadline)
        except StragglerTimeout:
            self.times.append(time.perf_counter() - t0)
            self.cancelled += 1
            return torch.zeros(()), 0.0
        finally:
            STRAGGLER_DEADLINE[0] = 0.0
            STRAGGLER_PACER[0] = None
        return loss, self.finished(time.perf_counter() - t0)

    def record(self, updated, finished):
        self.history.append(float(finished))
        self.iteration += 1
        if not finished:
            self.dropped += 1
        return updated

    def maybe_update_threshold(self, step, iteration):
        o = self.opt
        if iteration <= o.warmupIterationNum or iteration % o.computeThresholdbatchSize != 0:
            return
        local = torch.tensor(self.times[-o.computeThresholdbatchSize:] or [0.0], dtype=torch.float64)
        d = _dist()
        if d is not None and self.world > 1:
            n = torch.tensor([local.numel()], dtype=torch.int64, device=step.device)
            d.all_reduce(n, op=d.ReduceOp.MAX)
            buf = torch.zeros(int(n.item()), dtype=torch.float64, device=step.device)
            buf[:local.numel()] = local.to(step.device)
            allt = [torch.zeros_like(buf) for _ in range(self.world)]
            d.all_gather(allt, buf)
            times = torch.cat(allt).cpu()
            dropped = torch.tensor([float(self.dropped)], device=step.device)
            d.all_reduce(dropped)
            dropped = int(dropped.item())
        else:
            times, dropped = local, self.dropped
        k = int(o.dropPercentage * o.computeThresholdbatchSize * self.world)
        if k > dropped:
            vals = sorted(times.tolist(), reverse=True)
            self.threshold = vals[min(k - dropped, len(vals)) - 1]
        else:
            self.threshold = self.threshold * 1.01
        logger.info("threshold: %s", self.threshold)
        self.times = []
        self.dropped = 0


class LocalOptimizer(Optimizer):
    """Single-process training (reference LocalOptimizer.scala:40-295)."""


class DistriOptimizer(Optimizer):
    """Synchronous data-parallel training over all ranks of the job (reference DistriOptimizer.scala)."""

    def _epoch_size(self):
        return self.dataset.size()


class ParallelOptimizer(DistriOptimizer):
    """Data-parallel training with layer-wise bucketed gradient reduce-scatter overlapped with backward and the
    weight all-gather deferred into the next forward (reference ParallelOptimizer.scala:42-791; mechanism in
    parallel/bucketed.py). Every leaf layer without its own OptimMethod inherits its parent's
    (expandOptimMethods :642-670); layers are synchronised in priority order, default = execution order
    (defaultPrioritize :675-683); gradient clipping reduces the whole gradient before any layer updates."""

    _overlap = True
    _expand = True

    def __new__(cls, *args, **kw):
        return object.__new__(cls)

    def setPriorities(self, priorities):
        """{layer name: priority}; higher priorities are synchronised first."""
        self._priorities = dict(priorities)
        return self


def create(model, training_set, criterion, end_trigger=None, batch_size=32, optim_method=None, **kw):
    """Python-API style factory (reference P/optim/optimizer.py:874 ``Optimizer.create``)."""
    return Optimizer(model, training_set, criterion, batch_size, optim_method, end_trigger)


Optimizer.create = staticmethod(create)


AbstractOptimizer = Optimizer   # reference AbstractOptimizer.scala:33 — shared validate / checkpoint / summary logic
