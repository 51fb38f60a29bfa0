"""bigdl_amd.optim — optim methods, LR schedules, triggers, validation, training/inference runtimes."""
from .evaluator import DistriValidator, Evaluator, LocalValidator, Validator  # noqa: F401
from .methods import *  # noqa: F401,F403
from .metrics import Metrics  # noqa: F401
from .optim_method import OptimMethod  # noqa: F401
from .optimizer import AbstractOptimizer, DistriOptimizer, LocalOptimizer, Optimizer, ParallelOptimizer  # noqa: F401
from .predictor import LocalPredictor, PredictionService, Predictor  # noqa: F401
from .regularizer import L1L2Regularizer, L1Regularizer, L2Regularizer, Regularizer  # noqa: F401
from .sgd import *  # noqa: F401,F403
from .train_step import TrainStep  # noqa: F401
from .trigger import Trigger  # noqa: F401
from .validation import *  # noqa: F401,F403
from .detection_map import (MAPMultiIOUValidationResult, MAPValidationResult,  # noqa: F401,E402
                            MeanAveragePrecisionObjectDetection, cocoBBox, cocoSegmentation, pascalVOC)
from .validation import MeanAveragePrecision as _MAP  # noqa: E402

# reference `object MeanAveragePrecision` factories (S/optim/ValidationMethod.scala:761-840)
_MAP.pascalVOC = staticmethod(pascalVOC)
_MAP.cocoBBox = staticmethod(cocoBBox)
_MAP.cocoSegmentation = staticmethod(cocoSegmentation)
_MAP.classification = staticmethod(lambda nClasses, topK=-1: _MAP(topK, nClasses))
