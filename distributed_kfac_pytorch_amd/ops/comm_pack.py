"""Triangle packing and bucket (un)packing for K-FAC collectives (K-HIP-6).

GPU tensors: native kernels (csrc/pack.hip).  CPU tensors: torch indexing
with the same packed layout as the reference's ``get_triu`` / ``fill_triu``
(``kfac/distributed.py:416-459``, i.e. ``torch.triu_indices`` order).
"""
from __future__ import annotations

import torch

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native


def packed_numel(t: torch.Tensor, symmetric: bool) -> int:
    if symmetric:
        r, c = t.shape[0], t.shape[1]
        if r == c:
            return r * (r + 1) // 2
        return int(torch.triu_indices(r, c).shape[1])
    return t.numel()


def triu_pack(t: torch.Tensor) -> torch.Tensor:
    """Flattened upper triangle (incl. diagonal), row-major."""
    n, m = t.shape
    if n == m and t.stride(1) == 1 and use_native(t) and t.dtype in (
        torch.float32,
        torch.float64,
        torch.bfloat16,
    ):
        out = torch.empty(n * (n + 1) // 2, dtype=t.dtype, device=t.device)
        native().triu_pack(t, out)
        return out
    idx = torch.triu_indices(n, m, device=t.device)
    return t[idx[0], idx[1]]


def triu_unpack_(out: torch.Tensor, packed: torch.Tensor, scale: float) -> None:
    """out = scale * symmetric matrix with upper triangle ``packed``."""
    n, m = out.shape
    if n == m and out.stride(1) == 1 and use_native(out) and out.dtype in (
        torch.float32,
        torch.float64,
        torch.bfloat16,
    ):
        native().triu_unpack(out, packed.contiguous(), float(scale))
        return
    idx = torch.triu_indices(n, m, device=out.device)
    vals = packed if scale == 1.0 else packed * scale
    out[idx[0], idx[1]] = vals.to(out.dtype)
    low = torch.triu_indices(n, n, 1, device=out.device)
    out.transpose(0, 1)[low[0], low[1]] = out[low[0], low[1]]


def scale_copy_(dst: torch.Tensor, src: torch.Tensor, scale: float) -> None:
    """dst = scale * src (same numel, contiguous)."""
    if (
        use_native(dst)
        and dst.is_contiguous()
        and src.is_contiguous()
        and dst.dtype == src.dtype
        and dst.dtype in (torch.float32, torch.float64, torch.bfloat16)
    ):
        native().scale_copy(dst, src, float(scale))
        return
    if scale == 1.0:
        dst.copy_(src.view(dst.shape))
    else:
        torch.mul(src.view(dst.shape), scale, out=dst)


def pack_flat(flat: torch.Tensor, entries: list[tuple[torch.Tensor, bool]]) -> None:
    """Write each (tensor, symmetric) into consecutive slices of ``flat``."""
    off = 0
    for t, sym in entries:
        n = packed_numel(t, sym)
        sl = flat[off: off + n]
        if sym:
            sq = t.shape[0] == t.shape[1]
            if sq and use_native(t) and t.stride(1) == 1 and t.dtype in (
                torch.float32,
                torch.float64,
                torch.bfloat16,
            ):
                native().triu_pack(t, sl)
            else:
                sl.copy_(triu_pack(t))
        else:
            sl.copy_(t.reshape(-1))
        off += n


def unpack_slice_(
    target: torch.Tensor,
    sl: torch.Tensor,
    symmetric: bool,
    scale: float,
) -> None:
    """Write a reduced bucket slice back into ``target`` (in place)."""
    if symmetric:
        triu_unpack_(target, sl, scale)
    else:
        scale_copy_(target, sl, scale)
