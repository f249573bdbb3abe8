"""MI355X-native distributed K-FAC / KAISA gradient preconditioner.

API-compatible with ``kfac_pytorch`` 0.4.1 (``KFACPreconditioner(model).step()``
and its checkpoint format); hot paths are gfx950 HIP kernels
(``distributed_kfac_pytorch_amd._C``), communication is RCCL over xGMI through
``torch.distributed``.

Typical use::

    import distributed_kfac_pytorch_amd as kfac
    precond = kfac.KFACPreconditioner(model, factor_update_steps=10,
                                      inv_update_steps=100)
"""
from distributed_kfac_pytorch_amd import assignment
from distributed_kfac_pytorch_amd import base_preconditioner
from distributed_kfac_pytorch_amd import distributed
from distributed_kfac_pytorch_amd import enums
from distributed_kfac_pytorch_amd import hyperparams
from distributed_kfac_pytorch_amd import layers
from distributed_kfac_pytorch_amd import ops
from distributed_kfac_pytorch_amd import parallel
from distributed_kfac_pytorch_amd import preconditioner
from distributed_kfac_pytorch_amd import scheduler
from distributed_kfac_pytorch_amd import tracing
from distributed_kfac_pytorch_amd import warnings
from distributed_kfac_pytorch_amd.base_preconditioner import BaseKFACPreconditioner
from distributed_kfac_pytorch_amd.enums import AllreduceMethod
from distributed_kfac_pytorch_amd.enums import AssignmentStrategy
from distributed_kfac_pytorch_amd.enums import ComputeMethod
from distributed_kfac_pytorch_amd.enums import DistributedStrategy
from distributed_kfac_pytorch_amd.preconditioner import KFACPreconditioner
from distributed_kfac_pytorch_amd.scheduler import LambdaParamScheduler

__version__ = '0.4.1+mi355x.1'

__all__ = [
    'assignment',
    'base_preconditioner',
    'distributed',
    'enums',
    'hyperparams',
    'layers',
    'ops',
    'parallel',
    'preconditioner',
    'scheduler',
    'tracing',
    'warnings',
    'BaseKFACPreconditioner',
    'KFACPreconditioner',
    'LambdaParamScheduler',
    'AllreduceMethod',
    'AssignmentStrategy',
    'ComputeMethod',
    'DistributedStrategy',
]
