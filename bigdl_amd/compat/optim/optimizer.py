"""``bigdl.optim.optimizer`` for bigdl_amd (reference P/optim/optimizer.py:41-1186): validation methods, triggers,
learning-rate schedules, optimisation methods, ``Optimizer`` / ``DistriOptimizer`` / ``LocalOptimizer``,
summaries and regularizers with the reference Python names and snake_case arguments. Each object keeps the
engine object it configures in ``.value``."""
import os

import numpy as np

from ...optim import methods as _M
from ...optim import sgd as _S
from ...optim import trigger as _T
from ...optim import validation as _V
from ...optim import regularizer as _R
from ...visualization import summary as _Sum
from .._convert import to_numpy, to_torch
from ..util.common import RDD, samples_to_engine, to_engine_dataset, to_list

DOUBLEMAX = 1.7976931348623157e308


class JavaValue:
    def __init__(self, value):
        self.value = value
        self.bigdl_type = "float"

    def __str__(self):
        return str(self.value)


def _v(x):
    return getattr(x, "value", x)


# ------------------------------------------------------------------------------ validation methods
class Top1Accuracy(JavaValue):
    def __init__(self, bigdl_type="float"):
        super().__init__(_V.Top1Accuracy())


class TreeNNAccuracy(JavaValue):
    def __init__(self, bigdl_type="float"):
        super().__init__(_V.TreeNNAccuracy())


class Top5Accuracy(JavaValue):
    def __init__(self, bigdl_type="float"):
        super().__init__(_V.Top5Accuracy())


class MeanAveragePrecision(JavaValue):
    def __init__(self, k, classes, bigdl_type="float"):
        super().__init__(_V.MeanAveragePrecision(k, classes))


class MeanAveragePrecisionObjectDetection(JavaValue):
    def __init__(self, classes, iou=0.5, use_voc2007=False, skip_class=-1, bigdl_type="float"):
        from ...optim.detection_map import (MAPPascalVoc2007, MAPPascalVoc2010,
                                            MeanAveragePrecisionObjectDetection as _D)

        super().__init__(_D(classes, iouThres=[iou], theType=MAPPascalVoc2007 if use_voc2007 else MAPPascalVoc2010,
                            skipClass=skip_class))


class Loss(JavaValue):
    def __init__(self, cri=None, bigdl_type="float"):
        from ... import nn

        super().__init__(_V.Loss(_v(cri) if cri is not None else nn.ClassNLLCriterion()))


class HitRatio(JavaValue):
    def __init__(self, k=10, neg_num=100, bigdl_type="float"):
        super().__init__(_V.HitRatio(k, neg_num))


class NDCG(JavaValue):
    def __init__(self, k=10, neg_num=100, bigdl_type="float"):
        super().__init__(_V.NDCG(k, neg_num))


class MAE(JavaValue):
    def __init__(self, bigdl_type="float"):
        super().__init__(_V.MAE())


# ------------------------------------------------------------------------------ triggers
class MaxIteration(JavaValue):
    def __init__(self, max, bigdl_type="float"):
        super().__init__(_T.Trigger.maxIteration(max))


class MaxEpoch(JavaValue):
    def __init__(self, max_epoch, bigdl_type="float"):
        super().__init__(_T.Trigger.maxEpoch(max_epoch))


class EveryEpoch(JavaValue):
    def __init__(self, bigdl_type="float"):
        super().__init__(_T.Trigger.everyEpoch())


class SeveralIteration(JavaValue):
    def __init__(self, interval, bigdl_type="float"):
        super().__init__(_T.Trigger.severalIteration(interval))


class MaxScore(JavaValue):
    def __init__(self, max, bigdl_type="float"):
        super().__init__(_T.Trigger.maxScore(max))


class MinLoss(JavaValue):
    def __init__(self, min, bigdl_type="float"):
        super().__init__(_T.Trigger.minLoss(min))


class TriggerAnd(JavaValue):
    def __init__(self, first, *other):
        super().__init__(_T.Trigger.and_(_v(first), *[_v(o) for o in other]))


class TriggerOr(JavaValue):
    def __init__(self, first, *other):
        super().__init__(_T.Trigger.or_(_v(first), *[_v(o) for o in other]))


# ------------------------------------------------------------------------------ learning-rate schedules
class Poly(JavaValue):
    def __init__(self, power, max_iteration, bigdl_type="float"):
        super().__init__(_S.Poly(power, max_iteration))


class Exponential(JavaValue):
    def __init__(self, decay_step, decay_rate, stair_case=False, bigdl_type="float"):
        super().__init__(_S.Exponential(decay_step, decay_rate, stair_case))


class Step(JavaValue):
    def __init__(self, step_size, gamma, bigdl_type="float"):
        super().__init__(_S.Step(step_size, gamma))


class Default(JavaValue):
    def __init__(self, bigdl_type="float"):
        super().__init__(_S.Default())


class Plateau(JavaValue):
    def __init__(self, monitor, factor=0.1, patience=10, mode="min", epsilon=1e-4, cooldown=0, min_lr=0.0,
                 bigdl_type="float"):
        super().__init__(_S.Plateau(monitor, factor, patience, mode, epsilon, cooldown, min_lr))


class Warmup(JavaValue):
    def __init__(self, delta, bigdl_type="float"):
        super().__init__(_S.Warmup(delta))


class SequentialSchedule(JavaValue):
    def __init__(self, iteration_per_epoch, bigdl_type="float"):
        super().__init__(_S.SequentialSchedule(iteration_per_epoch))

    def add(self, scheduler, max_iteration, bigdl_type="float"):
        self.value.add(_v(scheduler), max_iteration)
        return self


class MultiStep(JavaValue):
    def __init__(self, step_sizes, gamma, bigdl_type="float"):
        super().__init__(_S.MultiStep(step_sizes, gamma))


# ------------------------------------------------------------------------------ optimisation methods
class OptimMethod(JavaValue):
    @staticmethod
    def load(path, bigdl_type="float"):
        from ...optim.optim_method import OptimMethod as _O

        return OptimMethod(_O.load(path))

    def save(self, path, overWrite):
        self.value.save(path, overWrite)
        return self


def _arr(a):
    return None if a is None else to_torch(np.asarray(a, dtype=np.float32))


class SGD(OptimMethod):
    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, momentum=0.0,
                 dampening=DOUBLEMAX, nesterov=False, leaningrate_schedule=None, learningrates=None,
                 weightdecays=None, bigdl_type="float"):
        super().__init__(_S.SGD(learningrate, learningrate_decay, weightdecay, momentum, dampening, nesterov,
                                _v(leaningrate_schedule) if leaningrate_schedule else None, _arr(learningrates),
                                _arr(weightdecays)))


class Adagrad(OptimMethod):
    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, bigdl_type="float"):
        super().__init__(_M.Adagrad(learningrate, learningrate_decay, weightdecay))


class LBFGS(OptimMethod):
    def __init__(self, max_iter=20, max_eval=DOUBLEMAX, tolfun=1e-5, tolx=1e-9, ncorrection=100, learningrate=1.0,
                 verbose=False, linesearch=None, linesearch_options=None, bigdl_type="float"):
        if linesearch or linesearch_options:
            raise ValueError("linesearch and linesearch_options must be None in LBFGS")
        super().__init__(_M.LBFGS(max_iter, None if max_eval == DOUBLEMAX else max_eval, tolfun, tolx, ncorrection,
                                  learningrate, verbose))


class Adadelta(OptimMethod):
    def __init__(self, decayrate=0.9, epsilon=1e-10, bigdl_type="float"):
        super().__init__(_M.Adadelta(decayrate, epsilon))


class Adam(OptimMethod):
    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 bigdl_type="float"):
        super().__init__(_M.Adam(learningrate, learningrate_decay, beta1, beta2, epsilon))


class ParallelAdam(OptimMethod):
    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 parallel_num=-1, bigdl_type="float"):
        super().__init__(_M.ParallelAdam(learningrate, learningrate_decay, beta1, beta2, epsilon))


class Ftrl(OptimMethod):
    def __init__(self, learningrate=1e-3, learningrate_power=-0.5, initial_accumulator_value=0.1,
                 l1_regularization_strength=0.0, l2_regularization_strength=0.0,
                 l2_shrinkage_regularization_strength=0.0, bigdl_type="float"):
        super().__init__(_M.Ftrl(learningrate, learningrate_power, initial_accumulator_value,
                                 l1_regularization_strength, l2_regularization_strength,
                                 l2_shrinkage_regularization_strength))


class Adamax(OptimMethod):
    def __init__(self, learningrate=0.002, beta1=0.9, beta2=0.999, epsilon=1e-38, bigdl_type="float"):
        super().__init__(_M.Adamax(learningrate, beta1, beta2, epsilon))


class RMSprop(OptimMethod):
    def __init__(self, learningrate=1e-2, learningrate_decay=0.0, decayrate=0.99, epsilon=1e-8,
                 bigdl_type="float"):
        super().__init__(_M.RMSprop(learningrate, learningrate_decay, decayrate, epsilon))


# ------------------------------------------------------------------------------ regularizers
class L1L2Regularizer(JavaValue):
    def __init__(self, l1, l2, bigdl_type="float"):
        super().__init__(_R.L1L2Regularizer(l1, l2))


class L1Regularizer(JavaValue):
    def __init__(self, l1, bigdl_type="float"):
        super().__init__(_R.L1Regularizer(l1))


class L2Regularizer(JavaValue):
    def __init__(self, l2, bigdl_type="float"):
        super().__init__(_R.L2Regularizer(l2))


class ActivityRegularization(JavaValue):
    def __init__(self, l1, l2, bigdl_type="float"):
        from ... import nn

        super().__init__(nn.ActivityRegularization(l1, l2))


# ------------------------------------------------------------------------------ summaries
class TrainSummary(JavaValue):
    def __init__(self, log_dir, app_name, bigdl_type="float"):
        super().__init__(_Sum.TrainSummary(log_dir, app_name))

    def read_scalar(self, tag):
        """[(step, value, wall time)] as an ndarray (reference :1077)."""
        return np.array([tuple(r) for r in self.value.readScalar(tag)])

    def set_summary_trigger(self, name, trigger):
        self.value.setSummaryTrigger(name, _v(trigger))
        return self


class ValidationSummary(JavaValue):
    def __init__(self, log_dir, app_name, bigdl_type="float"):
        super().__init__(_Sum.ValidationSummary(log_dir, app_name))

    def read_scalar(self, tag):
        return np.array([tuple(r) for r in self.value.readScalar(tag)])


# ------------------------------------------------------------------------------ optimizers
def _methods(model, optim_method):
    if optim_method is None:
        return {model.value.getName(): _S.SGD()}
    if isinstance(optim_method, dict):
        return {k: _v(m) for k, m in optim_method.items()}
    return {model.value.getName(): _v(optim_method)}


class BaseOptimizer(JavaValue):
    def set_model(self, model):
        self.value.setModel(model.value)

    def set_criterion(self, criterion):
        self.value.setCriterion(_v(criterion))

    def set_checkpoint(self, checkpoint_trigger, checkpoint_path, isOverWrite=True):
        os.makedirs(checkpoint_path, exist_ok=True)
        self.value.setCheckpoint(checkpoint_path, _v(checkpoint_trigger))
        if isOverWrite:
            self.value.overWriteCheckpoint()

    def set_gradclip_const(self, min_value, max_value):
        self.value.setConstantGradientClipping(min_value, max_value)

    def set_gradclip_l2norm(self, clip_norm):
        self.value.setGradientClippingByl2Norm(clip_norm)

    def disable_gradclip(self):
        self.value.disableGradientClipping()

    def optimize(self):
        from ..nn.layer import Layer

        return Layer.of(self.value.optimize())

    def set_train_summary(self, summary):
        self.value.setTrainSummary(_v(summary))
        return self

    def set_val_summary(self, summary):
        self.value.setValidationSummary(_v(summary))
        return self

    def prepare_input(self):
        self.value.prepareInput()

    def set_end_when(self, end_when):
        self.value.setEndWhen(_v(end_when))
        return self


class Optimizer(BaseOptimizer):
    """``Optimizer(model, training_rdd, criterion, end_trigger, batch_size, optim_method)`` (reference :840)."""

    def __init__(self, model, training_rdd, criterion, end_trigger, batch_size, optim_method=None,
                 bigdl_type="float"):
        self.pvalue = DistriOptimizer(model, training_rdd, criterion, end_trigger, batch_size, optim_method)
        self.value = self.pvalue.value
        self.bigdl_type = bigdl_type

    @staticmethod
    def create(model, training_set, criterion, end_trigger=None, batch_size=32, optim_method=None, cores=None,
               bigdl_type="float"):
        end_trigger = end_trigger or MaxEpoch(1)
        optim_method = optim_method or SGD()
        if isinstance(training_set, tuple) and len(training_set) == 2:
            x, y = training_set
            return LocalOptimizer(X=x, Y=y, model=model, criterion=criterion, end_trigger=end_trigger,
                                  batch_size=batch_size, optim_method=optim_method, cores=cores)
        from ...dataset.core import AbstractDataSet

        if isinstance(training_set, (RDD, list, AbstractDataSet)):
            return DistriOptimizer(model, training_set, criterion, end_trigger, batch_size, optim_method)
        raise Exception(f"Not supported training set: {type(training_set)}")

    def set_validation(self, batch_size, val_rdd, trigger, val_method=None):
        methods = [_v(m) for m in to_list(val_method or [Top1Accuracy()])]
        self.value.setValidation(_v(trigger), to_engine_dataset(val_rdd, shuffle=False), methods, batch_size)

    def set_traindata(self, training_rdd, batch_size):
        self.value.setTrainData(to_engine_dataset(training_rdd), batch_size)


class DistriOptimizer(Optimizer):
    def __init__(self, model, training_rdd, criterion, end_trigger, batch_size, optim_method=None,
                 bigdl_type="float"):
        from ...optim.optimizer import DistriOptimizer as _DO

        methods = _methods(model, optim_method)
        opt = _DO(model.value, to_engine_dataset(training_rdd), _v(criterion), batch_size,
                  next(iter(methods.values())), _v(end_trigger))
        if len(methods) > 1 or next(iter(methods)) != model.value.getName():
            opt.setOptimMethods(methods)
        self.value = opt
        self.bigdl_type = bigdl_type


class LocalOptimizer(BaseOptimizer):
    """``LocalOptimizer(X, Y, model, criterion, end_trigger, batch_size, optim_method, cores)`` over ndarrays
    (reference :993)."""

    def __init__(self, X, Y, model, criterion, end_trigger, batch_size, optim_method=None, cores=None,
                 bigdl_type="float"):
        from ...dataset.core import DataSet
        from ...optim.optimizer import LocalOptimizer as _LO

        samples = samples_to_engine(zip(_list_of_arrays(X), np.asarray(Y)))
        methods = _methods(model, optim_method)
        opt = _LO(model.value, DataSet.array(samples), _v(criterion), batch_size, next(iter(methods.values())),
                  _v(end_trigger))
        if len(methods) > 1:
            opt.setOptimMethods(methods)
        self.value = opt
        self.bigdl_type = bigdl_type

    def set_validation(self, batch_size, X_val, Y_val, trigger, val_method=None):
        from ...dataset.core import DataSet

        samples = samples_to_engine(zip(_list_of_arrays(X_val), np.asarray(Y_val)))
        methods = [_v(m) for m in to_list(val_method or [Top1Accuracy()])]
        self.value.setValidation(_v(trigger), DataSet.array(samples, shuffle=False), methods, batch_size)


def _list_of_arrays(X):
    if isinstance(X, list):            # multiple inputs: one ndarray per input, records along axis 0
        return [list(r) for r in zip(*X)]
    return list(np.asarray(X))


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("os", "np")]
