"""CIFAR-10 ResNets (He et al. 2015, section 4.2): ResNet-20/32/44/56/110/1202.

Same family as the reference's ``examples/vision/cifar_resnet.py:86-208``:
3 stages of 16/32/64 channels, BasicBlocks with ``bias=False`` 3x3 convs,
option-A (parameter-free) shortcuts that subsample and zero-pad channels,
global average pool and a Linear classifier.  ResNet-32 has 32 weight layers
(31 convs + fc) and ~0.46M parameters.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.ops.bnact import BatchNormAct2d

__all__ = [
    'CifarResNet',
    'resnet20',
    'resnet32',
    'resnet44',
    'resnet56',
    'resnet110',
    'resnet1202',
    'get_model',
]


class _ShortcutA(nn.Module):
    """Option-A shortcut: stride-2 subsample + zero-pad the channel dim."""

    def __init__(self, pad: int) -> None:
        super().__init__()
        self.pad = pad

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return F.pad(x[:, :, ::2, ::2], (0, 0, 0, 0, self.pad, self.pad))


class _Block(nn.Module):
    expansion = 1

    def __init__(self, cin: int, cout: int, stride: int = 1) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)
        self.bn1 = BatchNormAct2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1, bias=False)
        self.bn2 = BatchNormAct2d(cout)
        self.shortcut: nn.Module = nn.Identity()
        if stride != 1 or cin != cout:
            self.shortcut = _ShortcutA((cout - cin) // 2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # BN (+ shortcut) + ReLU: one fused native op in bf16 channels_last
        # training (ops/bnact.py), the same math through PyTorch otherwise
        y = self.bn1.act(self.conv1(x))
        return self.bn2.act(self.conv2(y), residual=self.shortcut(x))


class CifarResNet(nn.Module):
    def __init__(self, num_blocks: list[int], num_classes: int = 10) -> None:
        super().__init__()
        self.in_planes = 16
        self.conv1 = nn.Conv2d(3, 16, 3, padding=1, bias=False)
        self.bn1 = BatchNormAct2d(16)
        self.layer1 = self._stage(16, num_blocks[0], 1)
        self.layer2 = self._stage(32, num_blocks[1], 2)
        self.layer3 = self._stage(64, num_blocks[2], 2)
        self.linear = nn.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.kaiming_normal_(m.weight)

    def _stage(self, planes: int, blocks: int, stride: int) -> nn.Sequential:
        mods = []
        for s in [stride] + [1] * (blocks - 1):
            mods.append(_Block(self.in_planes, planes, s))
            self.in_planes = planes
        return nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.bn1.act(self.conv1(x))
        x = self.layer3(self.layer2(self.layer1(x)))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.linear(x)


def resnet20(num_classes: int = 10) -> CifarResNet:
    return CifarResNet([3, 3, 3], num_classes)


def resnet32(num_classes: int = 10) -> CifarResNet:
    return CifarResNet([5, 5, 5], num_classes)


def resnet44(num_classes: int = 10) -> CifarResNet:
    return CifarResNet([7, 7, 7], num_classes)


def resnet56(num_classes: int = 10) -> CifarResNet:
    return CifarResNet([9, 9, 9], num_classes)


def resnet110(num_classes: int = 10) -> CifarResNet:
    return CifarResNet([18, 18, 18], num_classes)


def resnet1202(num_classes: int = 10) -> CifarResNet:
    return CifarResNet([200, 200, 200], num_classes)


def get_model(name: str, num_classes: int = 10) -> CifarResNet:
    table = {
        'resnet20': resnet20,
        'resnet32': resnet32,
        'resnet44': resnet44,
        'resnet56': resnet56,
        'resnet110': resnet110,
        'resnet1202': resnet1202,
    }
    try:
        return table[name.lower()](num_classes)
    except KeyError:
        raise ValueError(f'unknown CIFAR model {name!r}') from None
