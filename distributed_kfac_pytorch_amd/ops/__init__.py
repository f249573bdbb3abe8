"""Native-op layer: every hot tensor op of K-FAC, with a gfx950 HIP kernel
for GPU tensors and the reference's PyTorch math for CPU tensors.

Modules:
    _native       extension loader and GPU policy (fail loudly if missing)
    factors       SYRK factor accumulation, conv patch extraction
    linalg        batched eigensolver, damped SPD inverse
    precondition  eigen-basis scaling, KL-clip reduction, in-place grad write
    comm_pack     triangle / bucket packing for collectives
"""
from distributed_kfac_pytorch_amd.ops import comm_pack
from distributed_kfac_pytorch_amd.ops import factors
from distributed_kfac_pytorch_amd.ops import linalg
from distributed_kfac_pytorch_amd.ops import precondition
from distributed_kfac_pytorch_amd.ops._native import available as native_available
from distributed_kfac_pytorch_amd.ops._native import native

__all__ = [
    'comm_pack',
    'factors',
    'linalg',
    'precondition',
    'native',
    'native_available',
]
