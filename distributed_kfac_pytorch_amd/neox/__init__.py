"""Tensor/pipeline-parallel K-FAC (the reference's ``kfac.gpt_neox``).

Self-contained: own (pipe, data, model) topology, Megatron-style
Column/Row-parallel linears, a minimal ``PipelineModule`` stage container,
the TP-aware eigen layer, the pipeline-stage assignment and the
preconditioner with per-layer factor checkpoint files.
"""
from distributed_kfac_pytorch_amd.neox import assignment
from distributed_kfac_pytorch_amd.neox import layer
from distributed_kfac_pytorch_amd.neox import modules
from distributed_kfac_pytorch_amd.neox import mpu
from distributed_kfac_pytorch_amd.neox import pipeline
from distributed_kfac_pytorch_amd.neox import preconditioner
from distributed_kfac_pytorch_amd.neox import topology
from distributed_kfac_pytorch_amd.neox import tp_layers
from distributed_kfac_pytorch_amd.neox.assignment import GPTNeoXAssignment
from distributed_kfac_pytorch_amd.neox.layer import GPTNeoXKFACEigenLayer
from distributed_kfac_pytorch_amd.neox.pipeline import PipelineModule
from distributed_kfac_pytorch_amd.neox.preconditioner import GPTNeoXKFACPreconditioner
from distributed_kfac_pytorch_amd.neox.topology import PipeModelDataParallelTopology
from distributed_kfac_pytorch_amd.neox.topology import ProcessTopology
from distributed_kfac_pytorch_amd.neox.tp_layers import ColumnParallelLinear
from distributed_kfac_pytorch_amd.neox.tp_layers import RowParallelLinear

__all__ = [
    'assignment', 'layer', 'modules', 'mpu', 'pipeline', 'preconditioner',
    'topology', 'tp_layers', 'GPTNeoXAssignment', 'GPTNeoXKFACEigenLayer',
    'PipelineModule', 'GPTNeoXKFACPreconditioner',
    'PipeModelDataParallelTopology', 'ProcessTopology',
    'ColumnParallelLinear', 'RowParallelLinear',
]
