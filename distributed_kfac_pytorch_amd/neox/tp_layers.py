"""Tensor-parallel linear layers (Megatron-style), native to this framework.

The reference GPT-NeoX path preconditions DeepSpeed/Megatron
``ColumnParallelLinear`` / ``RowParallelLinear`` modules
(``kfac/gpt_neox/preconditioner.py:447-512``).  Those libraries are not part
of this stack, so these are self-contained equivalents over
``torch.distributed`` (RCCL on MI355X):

* ``ColumnParallelLinear``: weight ``[out/mp, in]``; the input is replicated,
  the output is sharded along the feature dim (optionally all-gathered).
* ``RowParallelLinear``: weight ``[out, in/mp]``; the input is sharded along
  the feature dim (or split here), partial outputs are all-reduced, the bias
  is replicated.

Weights are initialised from a full-size master tensor and sliced, so a
model built with any MP degree starts from the same function.  The K-FAC
registration matches them by (lower-cased) class name exactly like the
reference does, so third-party Megatron layers with these names are picked up
too.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size


def _rank_in(group: dist.ProcessGroup | None) -> int:
    if group is None or not dist.is_initialized():
        return get_rank(group)
    return dist.get_rank(group)


class _CopyToRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        if get_world_size(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        if get_world_size(group) > 1:
            x = x.contiguous()
            dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        return g, None


class _GatherFromRegion(torch.autograd.Function):
    """All-gather along the last dim; backward keeps this rank's slice."""

    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        ctx.group = group
        world = get_world_size(group)
        if world == 1:
            return x
        x = x.contiguous()
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x, group=group)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        world = get_world_size(ctx.group)
        if world == 1:
            return g, None
        r = _rank_in(ctx.group)
        return g.chunk(world, dim=-1)[r].contiguous(), None


class _ScatterToRegion(torch.autograd.Function):
    """Keep this rank's slice of the last dim; backward all-gathers."""

    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        ctx.group = group
        world = get_world_size(group)
        if world == 1:
            return x
        return x.chunk(world, dim=-1)[_rank_in(group)].contiguous()

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        world = get_world_size(ctx.group)
        if world == 1:
            return g, None
        g = g.contiguous()
        parts = [torch.empty_like(g) for _ in range(world)]
        dist.all_gather(parts, g, group=ctx.group)
        return torch.cat(parts, dim=-1), None


def _master_init(out_f: int, in_f: int, seed: int) -> tuple[torch.Tensor, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    bound = 1.0 / math.sqrt(in_f)
    w = (torch.rand(out_f, in_f, generator=g) * 2 - 1) * bound
    b = (torch.rand(out_f, generator=g) * 2 - 1) * bound
    return w, b


class ColumnParallelLinear(torch.nn.Module):
    """y = x W^T + b with W split by output rows across the MP group."""

    def __init__(
        self,
        in_features: int,
        out_features: int,
        bias: bool = True,
        gather_output: bool = True,
        group: dist.ProcessGroup | None = None,
        init_seed: int = 0,
    ) -> None:
        super().__init__()
        self.group = group
        self.world = get_world_size(group)
        if out_features % self.world != 0:
            raise ValueError('out_features must be divisible by the MP size')
        self.in_features = in_features
        self.out_features = out_features
        self.out_per_rank = out_features // self.world
        self.gather_output = gather_output
        r = _rank_in(group)
        w, b = _master_init(out_features, in_features, init_seed)
        sl = slice(r * self.out_per_rank, (r + 1) * self.out_per_rank)
        self.weight = torch.nn.Parameter(w[sl].clone())
        self.bias = torch.nn.Parameter(b[sl].clone()) if bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = _CopyToRegion.apply(x, self.group)
        y = F.linear(x, self.weight, self.bias)
        if self.gather_output:
            y = _GatherFromRegion.apply(y, self.group)
        return y


class RowParallelLinear(torch.nn.Module):
    """y = x W^T + b with W split by input columns across the MP group."""

    def __init__(
        self,
        in_features: int,
        out_features: int,
        bias: bool = True,
        input_is_parallel: bool = False,
        group: dist.ProcessGroup | None = None,
        init_seed: int = 0,
    ) -> None:
        super().__init__()
        self.group = group
        self.world = get_world_size(group)
        if in_features % self.world != 0:
            raise ValueError('in_features must be divisible by the MP size')
        self.in_features = in_features
        self.out_features = out_features
        self.in_per_rank = in_features // self.world
        self.input_is_parallel = input_is_parallel
        r = _rank_in(group)
        w, b = _master_init(out_features, in_features, init_seed)
        sl = slice(r * self.in_per_rank, (r + 1) * self.in_per_rank)
        self.weight = torch.nn.Parameter(w[:, sl].clone())
        self.bias = torch.nn.Parameter(b.clone()) if bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.input_is_parallel:
            x = _ScatterToRegion.apply(x, self.group)
        y = F.linear(x, self.weight)
        y = _ReduceFromRegion.apply(y, self.group)
        if self.bias is not None:
            y = y + self.bias
        return y
