"""Native NHWC max pooling (csrc/pool.hip): the forward keeps a one-byte
argmax code per output element instead of torch's int64 indices, the
backward is a fixed-order gather (no atomics: bit-reproducible).

``MaxPool2dNHWC`` is a drop-in ``nn.MaxPool2d`` (ResNet's stem pool,
``models/resnet.py``): channels_last fp32 (C % 4 == 0) / bf16 (C % 8 == 0)
CUDA inputs with dilation 1, floor mode and no returned indices take the
native kernels; everything else -- the CPU, other layouts or dtypes, or
``KFAC_NATIVE_MAXPOOL=0`` -- runs ``nn.MaxPool2d``'s own path.  Reference
counterpart: the reference's models use ``torch.nn.MaxPool2d`` unchanged.
"""
from __future__ import annotations

from typing import Any

import torch
from torch import nn

from distributed_kfac_pytorch_amd.ops import _native as _nat
from distributed_kfac_pytorch_amd.utils.env import getenv


def _enabled() -> bool:
    return getenv('KFAC_NATIVE_MAXPOOL', '1') == '1'


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, k: int, s: int, p: int, lib: Any) -> torch.Tensor:
        y, code = lib.maxpool_nhwc_fwd(x, k, s, p)
        ctx.save_for_backward(code)
        ctx.conf = (x.shape[2], x.shape[3], k, s, p, lib)
        ctx.mark_non_differentiable(code)
        return y

    @staticmethod
    def backward(ctx: Any, gy: torch.Tensor) -> tuple:  # type: ignore[override]
        (code,) = ctx.saved_tensors
        h, w, k, s, p, lib = ctx.conf
        gy = gy.contiguous(memory_format=torch.channels_last)
        return lib.maxpool_nhwc_bwd(gy, code, h, w, k, s, p), None, None, None, None


def _geometry(m: nn.MaxPool2d) -> tuple[int, int, int] | None:
    def one(v: Any) -> int | None:
        if isinstance(v, int):
            return v
        v = tuple(v)
        return v[0] if len(set(v)) == 1 else None

    k, s, p, d = (one(m.kernel_size), one(m.stride if m.stride is not None else m.kernel_size),
                  one(m.padding), one(m.dilation))
    if None in (k, s, p, d) or d != 1 or m.ceil_mode or m.return_indices:
        return None
    if not (1 <= k <= 15 and s >= 1 and 0 <= 2 * p <= k):  # type: ignore[operator]
        return None
    return k, s, p  # type: ignore[return-value]


class MaxPool2dNHWC(nn.MaxPool2d):
    """``nn.MaxPool2d`` on the native NHWC kernels where they apply."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        geo = _geometry(self)
        if (geo is not None and x.is_cuda and x.dim() == 4 and _enabled()
                and x.dtype in (torch.float32, torch.bfloat16)
                and x.shape[1] % (4 if x.dtype == torch.float32 else 8) == 0
                and x.is_contiguous(memory_format=torch.channels_last)
                and x.data_ptr() % 16 == 0):
            lib = _nat.native()
            if lib is not None:
                return _MaxPoolNHWC.apply(x, *geo, lib)
        return super().forward(x)
