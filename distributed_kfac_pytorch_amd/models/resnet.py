"""ImageNet ResNets (v1.5: stride on the 3x3 conv), written for MI355X training.

The reference's ImageNet example pulls ``torchvision.models.resnet50``
(reference ``examples/torch_imagenet_resnet.py:304-309``).  torchvision is not
available in this image, so this is an independent implementation with the
same module tree and parameter names (``conv1``, ``bn1``, ``layer1.0.conv1``,
``layer1.0.downsample.0``, ``fc`` ...) so that K-FAC layer names, and therefore
the K-FAC checkpoint keys, match a torchvision model of the same depth.

MI355X notes: the model is meant to run in ``channels_last`` memory format
under bf16 autocast.  In NHWC the 1x1 convolutions' K-FAC input factor is a
plain SYRK of a ``[B*H*W, C]`` view (no im2col), and the G factor of every
conv is a SYRK of a ``[B*H*W, C_out]`` view of grad_output.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.nn as nn

from distributed_kfac_pytorch_amd.ops.bnact import BatchNormAct2d
from distributed_kfac_pytorch_amd.ops.conv import ResidualGradSlot
from distributed_kfac_pytorch_amd.ops.conv import StridedConv1x1
from distributed_kfac_pytorch_amd.ops.conv import _fuse_residual_grad
from distributed_kfac_pytorch_amd.ops.conv import residual_tap
from distributed_kfac_pytorch_amd.ops.pool import MaxPool2dNHWC

__all__ = [
    'Bottleneck',
    'BasicBlock',
    'ResNet',
    'resnet18',
    'resnet34',
    'resnet50',
    'resnet101',
    'resnet152',
    'get_model',
]


def _conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def _conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    # strided projection shortcuts: subsample + stride-1 conv, same module
    # attributes and values (MIOpen's strided 1x1 backward-data is not
    # HIP-graph safe: ops/conv.py)
    cls = StridedConv1x1 if stride != 1 else nn.Conv2d
    return cls(cin, cout, 1, stride=stride, bias=False)


def _shortcut(ds: nn.Module | None, x: torch.Tensor) -> torch.Tensor:
    """Identity or projection (conv + BN, the BN through the fused path)."""
    if ds is None:
        return x
    if isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[1], BatchNormAct2d):
        return ds[1].act(ds[0](x), relu=False)
    return ds(x)


class BasicBlock(nn.Module):
    """Two 3x3 convs with identity / projection shortcut."""

    expansion = 1

    def __init__(
        self,
        inplanes: int,
        planes: int,
        stride: int = 1,
        downsample: nn.Module | None = None,
    ) -> None:
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = BatchNormAct2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = BatchNormAct2d(planes)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = _shortcut(self.downsample, x)
        y = self.bn1.act(self.conv1(x))
        return self.bn2.act(self.conv2(y), residual=idt)


class Bottleneck(nn.Module):
    """1x1 reduce -> 3x3 (strided) -> 1x1 expand, ResNet v1.5."""

    expansion = 4

    def __init__(
        self,
        inplanes: int,
        planes: int,
        stride: int = 1,
        downsample: nn.Module | None = None,
    ) -> None:
        super().__init__()
        self.conv1 = _conv1x1(inplanes, planes)
        self.bn1 = BatchNormAct2d(planes)
        self.conv2 = _conv3x3(planes, planes, stride)
        self.bn2 = BatchNormAct2d(planes)
        self.conv3 = _conv1x1(planes, planes * self.expansion)
        self.bn3 = BatchNormAct2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # BN (+ residual) + ReLU are one fused native op in bf16 training
        # (ops/bnact.py); elsewhere the same math through PyTorch
        if self.downsample is None and x.requires_grad and _fuse_residual_grad():
            # identity shortcut: its gradient is added by conv1's input-
            # gradient GEMM (ops/conv.py ResidualGradSlot) when conv1 takes
            # the slot; the tap is made after conv3 so its backward runs first
            slot = ResidualGradSlot()
            self.conv1._dgrad_slot = slot
            try:
                y = self.bn1.act(self.conv1(x))
            finally:
                self.conv1.__dict__.pop('_dgrad_slot', None)
            y = self.conv3(self.bn2.act(self.conv2(y)))
            return self.bn3.act(y, residual=residual_tap(x, slot) if slot.armed else x)
        if (self.downsample is not None and x.requires_grad and _fuse_residual_grad()
                and isinstance(self.downsample, nn.Sequential) and len(self.downsample) == 2):
            # projection shortcut: conv1's input gradient is parked and the
            # shortcut's backward (which runs after conv1's) accumulates into
            # it -- at the kept pixels for a strided projection, in the GEMM
            # epilogue for a stride-1 one -- instead of autograd's add
            slot = ResidualGradSlot()
            ds = self.downsample[0]
            ds._dgrad_slot = slot
            try:
                idt = _shortcut(self.downsample, x)
            finally:
                ds.__dict__.pop('_dgrad_slot', None)
            if slot.armed:
                self.conv1._dgrad_park = slot
            try:
                y = self.bn1.act(self.conv1(x))
            finally:
                self.conv1.__dict__.pop('_dgrad_park', None)
        else:
            idt = _shortcut(self.downsample, x)
            y = self.bn1.act(self.conv1(x))
        y = self.bn2.act(self.conv2(y))
        return self.bn3.act(self.conv3(y), residual=idt)


class ResNet(nn.Module):
    """ImageNet ResNet with a torchvision-compatible parameter layout."""

    def __init__(
        self,
        block: type[BasicBlock] | type[Bottleneck],
        layers: list[int],
        num_classes: int = 1000,
        zero_init_residual: bool = False,
    ) -> None:
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(64)
        self.relu = nn.ReLU(inplace=True)
        # native NHWC kernels on the GPU (ops/pool.py), nn.MaxPool2d elsewhere
        self.maxpool = MaxPool2dNHWC(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(
                    m.weight,
                    mode='fan_out',
                    nonlinearity='relu',
                )
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)
        # every convolution whose output goes straight into a BN: a native
        # convolution then also writes the BN's statistics partials
        # (ops/conv.py take_bn_part), sparing the BN its pass over the output
        pairs = [(self.conv1, self.bn1)]
        for m in self.modules():
            if isinstance(m, (Bottleneck, BasicBlock)):
                pairs += [(m.conv1, m.bn1), (m.conv2, m.bn2)]
                if isinstance(m, Bottleneck):
                    pairs.append((m.conv3, m.bn3))
                if isinstance(m.downsample, nn.Sequential) and len(m.downsample) == 2:
                    pairs.append((m.downsample[0], m.downsample[1]))
        for conv, bn in pairs:
            if isinstance(bn, BatchNormAct2d):
                conv._feeds_bn = True

    def _make_layer(
        self,
        block: type[BasicBlock] | type[Bottleneck],
        planes: int,
        blocks: int,
        stride: int = 1,
    ) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, planes * block.expansion, stride),
                BatchNormAct2d(planes * block.expansion),
            )
        mods: list[nn.Module] = [
            block(self.inplanes, planes, stride, downsample),
        ]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            mods.append(block(self.inplanes, planes))
        return nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.bn1.act(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(**kw: int) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw: int) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw: int) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw: int) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw: int) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)


_MODELS: dict[str, Callable[..., ResNet]] = {
    'resnet18': resnet18,
    'resnet34': resnet34,
    'resnet50': resnet50,
    'resnet101': resnet101,
    'resnet152': resnet152,
}


def get_model(name: str, **kw: int) -> ResNet:
    """Return an ImageNet ResNet by name (``resnet50`` etc.)."""
    try:
        return _MODELS[name.lower()](**kw)
    except KeyError:
        raise ValueError(f'unknown ImageNet model {name!r}') from None
