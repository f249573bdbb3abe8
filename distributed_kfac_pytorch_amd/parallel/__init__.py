"""Distribution: RCCL/gloo collectives, KAISA placement, TP/PP topology."""
from distributed_kfac_pytorch_amd.parallel import assignment
from distributed_kfac_pytorch_amd.parallel import comm

__all__ = ['assignment', 'comm']
