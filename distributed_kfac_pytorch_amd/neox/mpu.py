"""Model-parallel communication helpers (reference ``kfac/gpt_neox/mpu.py``).

MI355X-first differences: the reference emulates a gather with an
``all_gather`` on every rank (every rank receives every shard, ``mpu.py:
56-66``) and a scatter with a ``reduce_scatter`` of zero tensors
(``gpt_neox/layer.py:289-304``).  Here a gather is a true ``dist.gather``
(RCCL point-to-point sends into one preallocated receive buffer on the
destination) and a scatter is a true ``dist.scatter``, halving the bytes
over xGMI and allocating nothing on non-destination ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size


def gather_from_model_parallel_region(
    input_: torch.Tensor,
    dst: int,
    model_parallel_group: dist.ProcessGroup | None,
    fp32_allreduce: bool = False,
    dim: int = -1,
) -> torch.Tensor | None:
    """Concatenate the shards of ``input_`` along ``dim`` on global rank
    ``dst``; other ranks get None.  ``fp32_allreduce`` moves bf16 shards in
    fp32 and casts the result back."""
    world = get_world_size(model_parallel_group)
    if world == 1:
        return input_
    dtype = input_.dtype
    x = input_
    if fp32_allreduce and dtype == torch.bfloat16:
        x = x.float()
    x = x.contiguous()
    if get_rank() == dst:
        buf = torch.empty((world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        dist.gather(x, gather_list=list(buf.unbind(0)), dst=dst, group=model_parallel_group)
        d = dim % x.dim()
        out = torch.cat(list(buf.unbind(0)), dim=d)
        return out.to(dtype)
    dist.gather(x, gather_list=None, dst=dst, group=model_parallel_group)
    return None


def scatter_to_model_parallel_region(
    chunks: list[torch.Tensor] | None,
    out: torch.Tensor,
    src: int,
    model_parallel_group: dist.ProcessGroup | None,
) -> torch.Tensor:
    """Every rank receives its chunk (in rank order of the group) into
    ``out``; only ``src`` passes ``chunks``."""
    if get_world_size(model_parallel_group) == 1:
        assert chunks is not None
        out.copy_(chunks[0])
        return out
    dist.scatter(
        out,
        scatter_list=[c.contiguous() for c in chunks] if get_rank() == src else None,
        src=src,
        group=model_parallel_group,
    )
    return out


def get_group_with_rank(rank: int, groups: list[list[int]]) -> list[int]:
    """The rank list in ``groups`` that contains ``rank``."""
    for g in groups:
        if rank in g:
            return g
    raise ValueError(f'rank {rank} not found in any group')


def split_tensor_along_dim(
    tensor: torch.Tensor,
    num_partitions: int,
    dim: int = -1,
    contiguous_split_chunks: bool = False,
) -> tuple[torch.Tensor, ...]:
    """Split into ``num_partitions`` equal chunks along ``dim``."""
    size = tensor.shape[dim]
    if size % num_partitions != 0:
        raise ValueError(
            f'{size} is not divisible by {num_partitions} partitions',
        )
    chunks = torch.split(tensor, size // num_partitions, dim=dim)
    if contiguous_split_chunks:
        return tuple(c.contiguous() for c in chunks)
    return chunks
