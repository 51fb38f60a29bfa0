"""bigdl_amd.nn — BigDL-style layers, containers, graphs and criterions (reference S/nn/**)."""
from .abstractnn import (AbstractCriterion, AbstractModule, AutogradCriterion, AutogradModule,  # noqa: F401
                         MklInt8Convertible, TensorCriterion, TensorModule, all_module_classes, module_class)
from .activation import *  # noqa: F401,F403
from .containers import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .criterion import *  # noqa: F401,F403
from .dropout import *  # noqa: F401,F403
from .graph import *  # noqa: F401,F403
from .init_methods import *  # noqa: F401,F403
from .linear import *  # noqa: F401,F403
from .normalization import *  # noqa: F401,F403
from .pooling import *  # noqa: F401,F403
from .recurrent import *  # noqa: F401,F403
from .shape_ops import *  # noqa: F401,F403
from .table_ops import *  # noqa: F401,F403
from .transformer import *  # noqa: F401,F403
from .detection import *  # noqa: F401,F403
from .penalty import *  # noqa: F401,F403
from .tree_lstm import *  # noqa: F401,F403
from ..optim.regularizer import L1L2Regularizer, L1Regularizer, L2Regularizer  # noqa: F401
from ..utils.table import T, Table  # noqa: F401
from .module import Module  # noqa: F401
from . import primitive as NNPrimitive  # noqa: E402,F401
from . import mkldnn  # noqa: E402,F401  (nn.mkldnn.RNN: the fused multi-layer RNN primitive)
