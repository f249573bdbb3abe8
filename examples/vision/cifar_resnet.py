"""CIFAR ResNets (reference ``examples/vision/cifar_resnet.py``); the models
live in :mod:`distributed_kfac_pytorch_amd.models.cifar_resnet`."""
from distributed_kfac_pytorch_amd.models.cifar_resnet import *  # noqa: F401,F403
from distributed_kfac_pytorch_amd.models.cifar_resnet import get_model  # noqa: F401
