"""Work placement for distributed K-FAC (reference ``kfac/assignment.py``).

``KAISAAssignment`` implements the KAISA layout.  With ``w`` ranks and a
gradient-worker fraction ``f`` there are ``m = max(1, w*f)`` gradient
workers per layer.  Ranks form an ``m x (w/m)`` grid (row-major):

* gradient-worker groups are the grid COLUMNS ``{i, i+p, i+2p, ...}``
  (``p = w/m``) -- every layer is owned by one column; its factors are
  decomposed on one rank of that column (the inverse worker) and the
  result is broadcast to the rest of the column;
* gradient-receiver groups are the grid ROWS ``{r*p, ..., r*p+p-1}`` -- the
  column member of a row preconditions the layer's gradient and broadcasts
  it along the row.

Load balancing is greedy LPT: layers by decreasing total cost go to the
least-loaded column, then to its least-loaded rank (or, without
colocation, each factor separately by decreasing (cost, name)).

On MI355X each distinct column / row group becomes an RCCL sub-communicator
(``dist.new_group`` on the nccl backend == ``ncclCommSplit``); groups are
created in a deterministic sorted order on every rank.  For 8 GPUs with
``f = 0.5`` that is 2 column comms of 4 ranks and 4 row comms of 2 ranks:
inverse broadcasts fan out over 3 distinct xGMI links from the source, and
gradient broadcasts are single-link peer copies.
"""
from __future__ import annotations

from abc import ABCMeta
from abc import abstractmethod
from dataclasses import dataclass
from typing import Any
from typing import Callable

import torch.distributed as dist


@dataclass(frozen=True)
class _Group:
    """Ranks of a communication group and its handle."""

    ranks: frozenset[int]
    group: Any


class WorkAssignment(metaclass=ABCMeta):
    """Interface the preconditioner queries to place K-FAC work."""

    def __repr__(self) -> str:
        rows = []
        for layer in self.get_layers():
            invs = {f: self.inv_worker(layer, f) for f in self.get_factors(layer)}
            rows.append(
                f'  layer="{layer}": '
                f'is_grad_worker={self.is_grad_worker(layer)}, '
                f'src_grad_worker={self.src_grad_worker(layer)}, '
                f'inv_workers={invs}',
            )
        body = ',\n'.join(rows)
        return f'{self.__class__.__name__}(\n{body}\n)'

    @abstractmethod
    def broadcast_gradients(self) -> bool:
        """Whether preconditioned gradients must be broadcast."""

    @abstractmethod
    def broadcast_inverses(self) -> bool:
        """Whether second-order results must be broadcast."""

    @abstractmethod
    def get_layers(self) -> tuple[str, ...]:
        """Names of the assigned layers."""

    @abstractmethod
    def get_factors(self, layer: str) -> tuple[str, ...]:
        """Factor names of a layer (e.g. ('A', 'G'))."""

    @abstractmethod
    def inv_worker(self, layer: str, factor: str) -> int:
        """Rank computing the decomposition of ``factor`` of ``layer``."""

    @abstractmethod
    def is_grad_worker(self, layer: str) -> bool:
        """Whether this rank preconditions ``layer``'s gradient."""

    @abstractmethod
    def src_grad_worker(self, layer: str) -> int:
        """Rank this rank receives ``layer``'s preconditioned gradient from."""

    @abstractmethod
    def factor_group(self, layer: str, factor: str) -> dist.ProcessGroup | None:
        """Group over which the factor is all-reduced."""

    @abstractmethod
    def grad_worker_group(self, layer: str) -> dist.ProcessGroup | None:
        """Group for the second-order broadcast of ``layer``."""

    @abstractmethod
    def grad_receiver_group(self, layer: str) -> dist.ProcessGroup | None:
        """Group for the preconditioned-gradient broadcast of ``layer``."""


class KAISAAssignment(WorkAssignment):
    """KAISA gradient-worker / receiver placement with LPT load balancing."""

    def __init__(
        self,
        work: dict[str, dict[str, float]],
        *,
        local_rank: int,
        world_size: int,
        grad_worker_fraction: float,
        group_func: Callable[[list[int]], dist.ProcessGroup | None],
        colocate_factors: bool = True,
    ) -> None:
        """Init KAISAAssignment.

        Args:
            work: ``{layer: {factor: cost}}``.
            local_rank: this process's rank.
            world_size: number of ranks.
            grad_worker_fraction: fraction of ranks preconditioning each layer;
                ``world_size * fraction`` must be an integer (or < 1).
            group_func: ``ranks -> process group`` (``dist.new_group``, or an
                identity function to simulate ranks in tests).
            colocate_factors: put all factors of a layer on one rank.
        """
        if not 0 <= grad_worker_fraction <= 1:
            raise ValueError(
                'grad_worker_fraction must be in [0, 1]. '
                f'Got {grad_worker_fraction}.',
            )
        if local_rank < 0:
            raise ValueError('local_rank must be >= 0')
        if world_size < 0:
            raise ValueError('world_size must be > 0')
        gw = max(1, world_size * grad_worker_fraction)
        if gw != int(gw):
            raise ValueError(
                'world_size*grad_worker_fraction must produce an integer '
                f'value. Found {world_size}*{grad_worker_fraction}={gw}.',
            )
        gw = int(gw)
        if local_rank >= world_size:
            raise ValueError(
                f'local_rank={local_rank} larger than world_size={world_size}',
            )
        self.local_rank = local_rank
        self.world_size = world_size
        self.grad_worker_fraction = grad_worker_fraction
        self.grad_workers = gw
        self.group_func = group_func
        self.colocate_factors = colocate_factors

        columns = self.partition_grad_workers(world_size, gw)
        rows = self.partition_grad_receivers(world_size, gw)
        handles: dict[frozenset[int], Any] = {}
        # deterministic creation order on every rank: all columns, then rows,
        # each sorted by smallest member
        for ranks in sorted(columns, key=min) + sorted(rows, key=min):
            if ranks not in handles:
                handles[ranks] = group_func(sorted(ranks))

        column_lists = [sorted(c) for c in sorted(columns, key=min)]
        self._inv_assignments = self.greedy_assignment(
            work,
            column_lists,
            world_size,
            colocate_factors,
        )
        self._grad_worker_groups: dict[str, _Group] = {}
        self._grad_receiver_groups: dict[str, _Group] = {}
        my_row = next(r for r in rows if local_rank in r)
        for layer, factors in self._inv_assignments.items():
            owner = next(iter(factors.values()))
            col = next(c for c in columns if owner in c)
            self._grad_worker_groups[layer] = _Group(col, handles[col])
            self._grad_receiver_groups[layer] = _Group(my_row, handles[my_row])

    @staticmethod
    def greedy_assignment(
        work: dict[str, dict[str, float]],
        worker_groups: list[list[int]],
        world_size: int,
        colocate_factors: bool,
    ) -> dict[str, dict[str, int]]:
        """Greedy LPT placement of factors onto ranks.

        Layers are visited by decreasing summed cost (stable for ties).  Each
        goes to the worker group with the lowest summed load (first on ties);
        inside it either the whole layer goes to the least-loaded rank
        (``colocate_factors``) or each factor, by decreasing (cost, name),
        goes to the then least-loaded rank.
        """
        loads = [0.0] * world_size
        result = {layer: {f: -1 for f in fs} for layer, fs in work.items()}
        totals = {layer: sum(fs.values()) for layer, fs in work.items()}
        for layer in sorted(totals, key=lambda k: totals[k], reverse=True):
            group_loads = [sum(loads[r] for r in g) for g in worker_groups]
            group = worker_groups[group_loads.index(min(group_loads))]

            def least_loaded() -> int:
                inner = [loads[r] for r in group]
                return group[inner.index(min(inner))]

            if colocate_factors:
                rank = least_loaded()
                loads[rank] += totals[layer]
                for f in work[layer]:
                    result[layer][f] = rank
            else:
                for f, cost in sorted(
                    work[layer].items(),
                    key=lambda kv: (kv[1], kv[0]),
                    reverse=True,
                ):
                    rank = least_loaded()
                    loads[rank] += cost
                    result[layer][f] = rank
        for layer, fs in result.items():
            for f, r in fs.items():
                assert r >= 0, (layer, f)
        return result

    @staticmethod
    def partition_grad_workers(world_size: int, grad_workers: int) -> set[frozenset[int]]:
        """Columns of the ``grad_workers x world/grad_workers`` rank grid."""
        if world_size <= 0:
            raise ValueError('world_size must be > 0')
        if world_size % grad_workers != 0:
            raise ValueError(
                'world_size must be an integer multiple of the gradient '
                'worker count',
            )
        p = world_size // grad_workers
        return {frozenset(range(i, world_size, p)) for i in range(p)}

    @staticmethod
    def partition_grad_receivers(world_size: int, grad_workers: int) -> set[frozenset[int]]:
        """Rows of the ``grad_workers x world/grad_workers`` rank grid."""
        if world_size <= 0:
            raise ValueError('world_size must be > 0')
        if world_size % grad_workers != 0:
            raise ValueError(
                'world_size must be an integer multiple of the gradient '
                'worker count',
            )
        p = world_size // grad_workers
        return {frozenset(range(i * p, (i + 1) * p)) for i in range(grad_workers)}

    def broadcast_gradients(self) -> bool:
        return self.grad_workers < self.world_size

    def broadcast_inverses(self) -> bool:
        return self.grad_workers > 1

    def get_layers(self) -> tuple[str, ...]:
        return tuple(self._inv_assignments)

    def get_factors(self, layer: str) -> tuple[str, ...]:
        return tuple(self._inv_assignments[layer])

    def inv_worker(self, layer: str, factor: str) -> int:
        return self._inv_assignments[layer][factor]

    def is_grad_worker(self, layer: str) -> bool:
        return self.local_rank in self._grad_worker_groups[layer].ranks

    def src_grad_worker(self, layer: str) -> int:
        both = (
            self._grad_worker_groups[layer].ranks
            & self._grad_receiver_groups[layer].ranks
        )
        return next(iter(both))

    def factor_group(self, layer: str, factor: str) -> dist.ProcessGroup | None:
        # KAISA is data parallel: every rank contributes to every factor.
        return None

    def grad_worker_group(self, layer: str) -> dist.ProcessGroup | None:
        return self._grad_worker_groups[layer].group

    def grad_receiver_group(self, layer: str) -> dist.ProcessGroup | None:
        return self._grad_receiver_groups[layer].group
