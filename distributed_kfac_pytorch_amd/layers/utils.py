"""Small factor utilities kept for API parity (reference
``kfac/layers/utils.py:7-82``).

The hot path does not use these: factor accumulation goes through
``ops.factors.cov_accumulate_`` (one fused SYRK on MI355X).  They remain the
documented, tested building blocks of the CPU reference math.
"""
from __future__ import annotations

import torch


def append_bias_ones(tensor: torch.Tensor) -> torch.Tensor:
    """Append a column of ones along the last dimension ([.., d] -> [.., d+1])."""
    ones = tensor.new_ones(*tensor.shape[:-1], 1)
    return torch.cat([tensor, ones], dim=-1)


def get_cov(
    a: torch.Tensor,
    b: torch.Tensor | None = None,
    scale: float | None = None,
) -> torch.Tensor:
    """Empirical second moment ``a^T a / scale`` (``scale`` defaults to rows).

    With ``b`` the (unsymmetrized) cross moment ``a^T b / scale`` is returned;
    without it the result is symmetrized as ``(C + C^T) / 2``.
    """
    if a.dim() != 2:
        raise ValueError(
            'Input tensor must have 2 dimensions. Got tensor with shape '
            f'{a.shape}',
        )
    if b is not None and a.shape != b.shape:
        raise ValueError(
            f'Input tensors must have same shape. Got tensors of shape '
            f'{a.shape} and {b.shape}.',
        )
    s = a.shape[0] if scale is None else scale
    if b is not None:
        return a.t() @ (b / s)
    cov = a.t() @ (a / s)
    return (cov + cov.t()) / 2.0


def reshape_data(
    data_list: list[torch.Tensor],
    batch_first: bool = True,
    collapse_dims: bool = False,
) -> torch.Tensor:
    """Concatenate tensors along the batch dim; optionally flatten to 2D."""
    d = torch.cat(data_list, dim=0 if batch_first else 1)
    if collapse_dims and d.dim() > 2:
        d = d.reshape(-1, d.shape[-1])
    return d
