"""3-D process topology (pipeline x data x model parallel).

The reference's GPT-NeoX path reads DeepSpeed's
``PipeModelDataParallelTopology`` (``kfac/gpt_neox/assignment.py:61-64``,
``gpt_neox/preconditioner.py:258-264``).  DeepSpeed is not part of this
stack, so this module provides the same topology semantics natively:

* axes ``('pipe', 'data', 'model')`` with the model axis fastest, i.e.
  ``rank = (pipe * DP + data) * MP + model`` -- tensor-parallel peers are
  adjacent ranks, which on an 8-GPU MI355X node puts a TP group on GPUs that
  share direct xGMI links and keeps the hot activation gathers one hop;
* ``get_coord(rank)`` (namedtuple with ``.pipe/.data/.model``),
  ``get_rank(**coords)``, ``get_axis_comm_lists(axis)`` (all rank lists that
  vary only along ``axis``), ``get_dim(axis)``, ``world_size()``.
"""
from __future__ import annotations

import itertools
from collections import namedtuple
from typing import Any


class ProcessTopology:
    """Cartesian mapping between ranks and named coordinates."""

    def __init__(self, axes: list[str], dims: list[int]) -> None:
        if len(axes) != len(dims):
            raise ValueError('axes and dims must have the same length')
        if any(d < 1 for d in dims):
            raise ValueError('every dim must be >= 1')
        self.axes = list(axes)
        self.dims = list(dims)
        self.ProcessCoord = namedtuple('ProcessCoord', self.axes)  # type: ignore
        self.mapping: dict[Any, int] = {}
        ranges = [range(d) for d in self.dims]
        for rank, coord in enumerate(itertools.product(*ranges)):
            key = dict(zip(self.axes, coord))
            self.mapping[self.ProcessCoord(**key)] = rank
        self._coords = {r: c for c, r in self.mapping.items()}

    def world_size(self) -> int:
        n = 1
        for d in self.dims:
            n *= d
        return n

    def get_dim(self, axis: str) -> int:
        return self.dims[self.axes.index(axis)] if axis in self.axes else 0

    def get_rank(self, **coords: int) -> int:
        if len(coords) != len(self.axes):
            raise ValueError('get_rank() needs every axis coordinate')
        return self.mapping[self.ProcessCoord(**coords)]

    def get_coord(self, rank: int) -> Any:
        if rank not in self._coords:
            raise ValueError(f'rank {rank} not in topology')
        return self._coords[rank]

    def get_axis_comm_lists(self, axis: str) -> list[list[int]]:
        """Rank lists whose members differ only in ``axis`` (sorted)."""
        if axis not in self.axes:
            return []
        others = [a for a in self.axes if a != axis]
        lists = []
        for other in itertools.product(*[range(self.get_dim(a)) for a in others]):
            fixed = dict(zip(others, other))
            ranks = [
                self.get_rank(**{**fixed, axis: i})
                for i in range(self.get_dim(axis))
            ]
            lists.append(ranks)
        return lists

    def filter_match(self, **filters: int) -> list[int]:
        """Ranks whose coordinates match every given axis value."""
        out = []
        for coord, rank in self.mapping.items():
            if all(getattr(coord, k) == v for k, v in filters.items()):
                out.append(rank)
        return sorted(out)

    def __repr__(self) -> str:
        return f'{self.__class__.__name__}(axes={self.axes}, dims={self.dims})'


class PipeModelDataParallelTopology(ProcessTopology):
    """``(pipe, data, model)`` topology with model-parallel ranks adjacent."""

    def __init__(self, num_pp: int, num_mp: int, num_dp: int) -> None:
        super().__init__(axes=['pipe', 'data', 'model'], dims=[num_pp, num_dp, num_mp])
