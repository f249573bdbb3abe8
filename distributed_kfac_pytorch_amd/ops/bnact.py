"""Fused training-mode BatchNorm2d (+ residual) (+ ReLU) for the ResNets.

``BatchNormAct2d`` is an ``nn.BatchNorm2d`` (same parameters, buffers and
state-dict keys as torchvision's) with one extra entry point,
``act(x, residual=None, relu=True)`` = ``relu(bn(x) + residual)``.  In
training mode on NHWC (channels_last) bf16 or fp32 activations -- the
layouts of a ResNet under bf16 autocast or in fp32 on MI355X -- it runs the native
kernels of ``csrc/bnact.hip``: 3 launches forward and 3 backward per layer,
replacing MIOpen's BN kernels, its tensor ops, the separate ReLU forward /
backward, the residual add and the ``num_batches_tracked`` increment.
Everything else (eval mode, NCHW inputs, CPU) takes the PyTorch path with
identical semantics.  ``KFAC_FUSED_BN=0`` disables the kernels,
``KFAC_FUSED_BN_FP32=0`` only their fp32 use.
"""
from __future__ import annotations

from typing import Any

import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops.conv import take_bn_part
from distributed_kfac_pytorch_amd.utils.env import getenv

__all__ = ['BatchNormAct2d', 'bn_act']


def _enabled() -> bool:
    return getenv('KFAC_FUSED_BN', '1') != '0'


def _dtypes() -> tuple[torch.dtype, ...]:
    # KFAC_FUSED_BN_FP32=0 keeps fp32 activations on the PyTorch / MIOpen path
    if getenv('KFAC_FUSED_BN_FP32', '1') == '0':
        return (torch.bfloat16,)
    return (torch.bfloat16, torch.float32)


class _BNActFunction(torch.autograd.Function):
    """Python reference wrapper of the same kernels (tests compare the C++
    autograd node ``native().bn_act`` against it)."""

    @staticmethod
    def forward(  # type: ignore[override]
        ctx: Any,
        x: torch.Tensor,
        weight: torch.Tensor | None,
        bias: torch.Tensor | None,
        running_mean: torch.Tensor | None,
        running_var: torch.Tensor | None,
        num_batches: torch.Tensor | None,
        residual: torch.Tensor | None,
        relu: bool,
        momentum: float,
        eps: float,
    ) -> torch.Tensor:
        y, stats = native().bn_act_forward(
            x, residual, weight, bias, running_mean, running_var, num_batches,
            momentum, eps, relu,
        )
        ctx.save_for_backward(x, y, weight, stats)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.has_weight = weight is not None
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, y, weight, stats = ctx.saved_tensors
        dx, dw, db, dres = native().bn_act_backward(
            x, dy, y, weight, stats, ctx.relu, ctx.has_res,
        )
        return (
            dx,
            dw if ctx.has_weight else None,
            db if ctx.has_bias else None,
            None, None, None,
            dres if ctx.has_res else None,
            None, None, None,
        )


def _fusable(bn: nn.BatchNorm2d, x: torch.Tensor, residual: torch.Tensor | None) -> bool:
    if not (_enabled() and bn.training and bn.track_running_stats and bn.momentum is not None
            and bn.affine):
        return False
    if not x.is_cuda or x.dtype not in _dtypes():
        return False
    lib = native()
    if lib is None or not lib.bn_act_supported(x):
        return False
    if residual is not None:
        if residual.dtype != x.dtype or residual.shape != x.shape:
            return False
        if not lib.bn_act_supported(residual):
            return False
    return True


def bn_act(
    bn: nn.BatchNorm2d,
    x: torch.Tensor,
    residual: torch.Tensor | None = None,
    relu: bool = True,
) -> torch.Tensor:
    """``relu(bn(x) + residual)`` (ReLU / residual optional)."""
    # statistics partials from the native convolution that produced x
    # (ops/conv.py take_bn_part): the fused BN then skips its pass over x
    part = take_bn_part(x)
    if _fusable(bn, x, residual):
        # C++ autograd node (csrc/bindings.cpp BNActFn): no Python in the
        # forward or backward of the layer
        return native().bn_act(
            x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
            bn.num_batches_tracked, float(bn.momentum), float(bn.eps), relu,
            part if x.dtype == torch.float32 else None,
        )
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with a fused ``act`` entry point (see module doc)."""

    def act(
        self,
        x: torch.Tensor,
        residual: torch.Tensor | None = None,
        relu: bool = True,
    ) -> torch.Tensor:
        return bn_act(self, x, residual, relu)
