"""Kronecker-factor accumulation ops (K-HIP-1 SYRK, K-HIP-2 patches).

``cov_accumulate_(out, x, bias=..., alpha=..., beta=...)`` computes

    out = beta * out + alpha * Xt^T Xt,   Xt = [x, 1] if bias else x

for a 2D ``x`` of shape [N, K].  ``out`` is either the dense [D, D] factor
or its packed upper triangle (1-D, D (D + 1) / 2, row-major -- the layout of
the factor all-reduce wire, see ``parallel/comm.py``
``PackedFactorBuffer``): the SYRK epilogue then updates the triangle in
place and writes nothing else.  On MI355X this is one MFMA SYRK launch
(csrc/syrk.hip) that reads ``x`` once in its native dtype (bf16 under
autocast, fp32 otherwise), synthesises the bias column, and writes an exactly
symmetric fp32 result with the EMA / averaging weights folded into
``alpha`` / ``beta``.  On CPU it is the reference's math
(``kfac/layers/utils.py:17-58``).
"""
from __future__ import annotations

import math

import torch

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native
from distributed_kfac_pytorch_amd.utils.env import getenv


def _torch_cov_accumulate_(
    out: torch.Tensor,
    x: torch.Tensor,
    bias: bool,
    alpha: float,
    beta: float,
    alpha_scale: torch.Tensor | None = None,
) -> None:
    xc = x.to(out.dtype)
    if bias:
        xc = torch.cat([xc, xc.new_ones(xc.shape[0], 1)], dim=1)
    cov = xc.t() @ xc
    cov = (cov + cov.t()) / 2.0
    if alpha_scale is not None:
        cov = cov * alpha_scale.to(cov.dtype)
    if beta == 0.0:
        torch.mul(cov, alpha, out=out)
    else:
        out.mul_(beta).add_(cov, alpha=alpha)


def fp32_exact() -> bool:
    """fp32 SYRK inputs: exact-product fp32 MFMA (``KFAC_SYRK_FP32=exact``)
    instead of the default three-term bf16 split (csrc/syrk.hip)."""
    return getenv('KFAC_SYRK_FP32', 'bf16x3').lower() == 'exact'


def _splits() -> int:
    """Split-K slab count of the SYRK (``KFAC_SYRK_SPLITS``; 0 = the
    kernel's own choice, 1 = no split-K workspace)."""
    return int(getenv('KFAC_SYRK_SPLITS', '0'))


def packed_dim(out: torch.Tensor) -> int:
    """D of a packed D x D upper triangle held in the 1-D ``out``."""
    n = out.numel()
    d = int((math.isqrt(8 * n + 1) - 1) // 2)
    if d * (d + 1) // 2 != n:
        raise ValueError(f'{n} elements is not a packed triangle')
    return d


def _packed_emulate_(out: torch.Tensor, fn) -> None:  # type: ignore[no-untyped-def]
    """Apply a dense in-place update to a packed triangle (CPU / fallback)."""
    from distributed_kfac_pytorch_amd.ops import comm_pack

    d = packed_dim(out)
    dense = out.new_empty((d, d))
    comm_pack.triu_unpack_(dense, out, 1.0)
    fn(dense)
    out.copy_(comm_pack.triu_pack(dense))


def cov_accumulate_(
    out: torch.Tensor,
    x: torch.Tensor,
    *,
    bias: bool = False,
    alpha: float = 1.0,
    beta: float = 0.0,
    alpha_scale: torch.Tensor | None = None,
) -> torch.Tensor:
    """In-place ``out = beta*out + alpha*Xt^T Xt`` (see module docstring).
    ``alpha_scale``: optional 1-element device tensor multiplying ``alpha``
    (the AMP loss-scale correction, applied without a host sync)."""
    if x.dim() != 2:
        raise ValueError(f'expected a 2D input, got shape {tuple(x.shape)}')
    d = x.shape[1] + int(bias)
    if out.dim() == 1:
        if out.numel() != d * (d + 1) // 2:
            raise ValueError(f'packed output must hold {d * (d + 1) // 2} elements')
    elif out.shape != (d, d):
        raise ValueError(
            f'output must be [{d}, {d}], got {tuple(out.shape)}',
        )
    if use_native(x, out) and out.dtype == torch.float32:
        xin = x
        if xin.dtype not in (torch.bfloat16, torch.float32):
            xin = xin.float()
        if xin.stride(1) != 1 or (xin.shape[0] > 1 and xin.stride(0) < xin.shape[1]):
            xin = xin.contiguous()
        native().syrk(xin, out, bias, float(alpha), float(beta), _splits(), alpha_scale,
                      fp32_exact())
        return out
    if out.dim() == 1:
        _packed_emulate_(out, lambda dense: _torch_cov_accumulate_(
            dense, x, bias, alpha, beta, alpha_scale))
        return out
    _torch_cov_accumulate_(out, x, bias, alpha, beta, alpha_scale)
    return out


def conv_cov_accumulate_(
    out: torch.Tensor,
    x: torch.Tensor,
    kernel: tuple[int, int],
    stride: tuple[int, int],
    padding: tuple[int, int],
    *,
    bias: bool = False,
    alpha: float = 1.0,
    beta: float = 0.0,
) -> bool:
    """Implicit-im2col SYRK (K-HIP-2): ``out = beta*out + alpha*P^T P`` with
    ``P`` the natural-order (kh, kw, c) patch matrix of the NHWC conv input
    ``x``, computed without materialising ``P`` (the SYRK tile loader reads
    the patches from ``x``).  Returns False when the fast path does not
    apply (CPU, NCHW input, dtype, channel count not a multiple of one
    16-byte vector); the caller then builds the patch matrix explicitly."""
    if not (use_native(x, out) and out.dtype == torch.float32 and is_channels_last(x)):
        return False
    if x.dtype not in (torch.bfloat16, torch.float32):
        return False
    vec = 4 if x.dtype == torch.float32 else 8
    st = x.stride()
    if (
        x.shape[1] % vec
        or any(v % vec for v in (st[0], st[2], st[3]))
        or x.data_ptr() % 16
        or (out.dim() == 2 and out.stride(1) != 1)
    ):
        return False
    native().syrk_conv(x, out, kernel[0], kernel[1], stride[0], stride[1],
                       padding[0], padding[1], bias, float(alpha), float(beta), _splits(),
                       None, fp32_exact())
    return True


def identity_(out: torch.Tensor) -> torch.Tensor:
    """Fill a square matrix with the identity (factor initialisation)."""
    if use_native(out) and out.dtype == torch.float32 and out.stride(1) == 1:
        native().fill_identity(out)
        return out
    out.zero_()
    out.diagonal().fill_(1)
    return out


def conv_out_hw(
    h: int,
    w: int,
    kernel: tuple[int, int],
    stride: tuple[int, int],
    padding: tuple[int, int],
) -> tuple[int, int]:
    oh = (h + 2 * padding[0] - kernel[0]) // stride[0] + 1
    ow = (w + 2 * padding[1] - kernel[1]) // stride[1] + 1
    return oh, ow


def is_channels_last(x: torch.Tensor) -> bool:
    """True if a 4D tensor is laid out NHWC with contiguous channel rows."""
    if x.dim() != 4:
        return False
    b, c, h, w = x.shape
    st = x.stride()
    return st[1] == 1 and st[3] == c and st[2] == w * c


def conv_patches(
    x: torch.Tensor,
    kernel: tuple[int, int],
    stride: tuple[int, int],
    padding: tuple[int, int],
    natural: bool,
) -> tuple[torch.Tensor, int]:
    """Patch matrix [B*OH*OW, C*kh*kw] of a conv input and OH*OW.

    ``natural`` selects (kh, kw, c) column order from an NHWC input;
    otherwise the reference (c, kh, kw) order.  A 1x1 / stride-1 / no-pad
    conv on an NHWC input returns a zero-copy view.
    """
    b, c, h, w = x.shape
    oh, ow = conv_out_hw(h, w, kernel, stride, padding)
    kk = kernel[0] * kernel[1]
    if (
        kernel == (1, 1)
        and stride == (1, 1)
        and padding == (0, 0)
        and is_channels_last(x)
    ):
        return x.permute(0, 2, 3, 1).reshape(b * h * w, c), oh * ow
    if use_native(x) and x.dtype in (
        torch.bfloat16,
        torch.float32,
        torch.float16,
    ):
        out_dtype = torch.float32 if x.dtype == torch.float32 else torch.bfloat16
        k = c * kk
        ld = (k + 7) // 8 * 8  # 16-B aligned rows for the SYRK vector loads
        buf = torch.empty(b * oh * ow, ld, dtype=out_dtype, device=x.device)
        nat = natural and x.stride(1) == 1
        native().im2col(
            x,
            buf,
            kernel[0],
            kernel[1],
            stride[0],
            stride[1],
            padding[0],
            padding[1],
            nat,
        )
        return buf[:, :k], oh * ow
    # CPU / reference math: pad + unfold (kfac/layers/modules.py:210-237)
    if natural:
        xp = torch.nn.functional.pad(
            x,
            (padding[1], padding[1], padding[0], padding[0]),
        )
        # [B, C, OH, OW, kh, kw] -> [B, OH, OW, kh, kw, C]
        u = xp.unfold(2, kernel[0], stride[0]).unfold(3, kernel[1], stride[1])
        u = u.permute(0, 2, 3, 4, 5, 1).reshape(b * oh * ow, kk * c)
        return u, oh * ow
    xp = x
    if padding[0] + padding[1] > 0:
        xp = torch.nn.functional.pad(
            x,
            (padding[1], padding[1], padding[0], padding[0]),
        )
    u = xp.unfold(2, kernel[0], stride[0]).unfold(3, kernel[1], stride[1])
    u = u.permute(0, 2, 3, 1, 4, 5).reshape(b * oh * ow, c * kk)
    return u, oh * ow


def rows_nhwc(g: torch.Tensor) -> torch.Tensor:
    """[B, C, H, W] -> [B*H*W, C] (a view when the tensor is channels_last)."""
    b, c, h, w = g.shape
    return g.permute(0, 2, 3, 1).reshape(b * h * w, c)
