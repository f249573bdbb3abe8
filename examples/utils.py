"""Example utilities (reference ``examples/utils.py``).

The implementations live in :mod:`distributed_kfac_pytorch_amd.utils` so the
benchmark and tests share them; this module keeps the reference import path
(``from examples.utils import Metric``) working.
"""
from distributed_kfac_pytorch_amd.utils.training import accuracy
from distributed_kfac_pytorch_amd.utils.training import create_lr_schedule
from distributed_kfac_pytorch_amd.utils.training import LabelSmoothLoss
from distributed_kfac_pytorch_amd.utils.training import latest_checkpoint
from distributed_kfac_pytorch_amd.utils.training import load_checkpoint
from distributed_kfac_pytorch_amd.utils.training import Metric
from distributed_kfac_pytorch_amd.utils.training import save_checkpoint

__all__ = [
    'accuracy', 'create_lr_schedule', 'LabelSmoothLoss', 'latest_checkpoint',
    'load_checkpoint', 'Metric', 'save_checkpoint',
]
