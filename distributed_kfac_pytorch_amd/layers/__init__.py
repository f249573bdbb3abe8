"""Per-layer K-FAC state and module adapters."""
from distributed_kfac_pytorch_amd.layers import base
from distributed_kfac_pytorch_amd.layers import eigen
from distributed_kfac_pytorch_amd.layers import inverse
from distributed_kfac_pytorch_amd.layers import modules
from distributed_kfac_pytorch_amd.layers import register
from distributed_kfac_pytorch_amd.layers import utils
from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.inverse import KFACInverseLayer

__all__ = [
    'base',
    'eigen',
    'inverse',
    'modules',
    'register',
    'utils',
    'KFACBaseLayer',
    'KFACEigenLayer',
    'KFACInverseLayer',
]
