"""Model families used by the examples, tests and benchmarks."""
from distributed_kfac_pytorch_amd.models import cifar_resnet
from distributed_kfac_pytorch_amd.models import resnet
from distributed_kfac_pytorch_amd.models import tiny
from distributed_kfac_pytorch_amd.models import transformer

__all__ = ['cifar_resnet', 'resnet', 'tiny', 'transformer']
