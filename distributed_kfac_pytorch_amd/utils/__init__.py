"""Training utilities (checkpoint I/O, metrics, LR schedules, data)."""
from distributed_kfac_pytorch_amd.utils import data
from distributed_kfac_pytorch_amd.utils import training

__all__ = ['data', 'training']
