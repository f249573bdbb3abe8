"""Minimal pipeline-stage container exposing ``topology()``.

The reference GPT-NeoX preconditioner requires a DeepSpeed ``PipelineModule``
(``kfac/gpt_neox/preconditioner.py:159-163``) and only uses it for (a) its
module tree and (b) ``model.topology()``.  This container provides both: it
instantiates only the layers of this rank's pipeline stage (contiguous,
balanced partition by layer count unless ``partition`` is given) and runs
them in sequence.  Scheduling micro-batches across stages is out of its
scope -- K-FAC needs only the stage-local modules and the topology.
"""
from __future__ import annotations

from typing import Callable

import torch

from distributed_kfac_pytorch_amd.neox.topology import ProcessTopology
from distributed_kfac_pytorch_amd.parallel.comm import get_rank


class PipelineModule(torch.nn.Module):
    def __init__(
        self,
        layers: list[Callable[[], torch.nn.Module]],
        topology: ProcessTopology,
        partition: list[int] | None = None,
        rank: int | None = None,
    ) -> None:
        """Args:
            layers: zero-argument constructors, one per pipeline layer.
            topology: (pipe, data, model) topology of the job.
            partition: stage boundaries ``[0, b1, ..., len(layers)]``.
            rank: this process's global rank (default: torch.distributed).
        """
        super().__init__()
        self._topo = topology
        stages = topology.get_dim('pipe')
        n = len(layers)
        if partition is None:
            partition = [round(i * n / stages) for i in range(stages + 1)]
        if len(partition) != stages + 1 or partition[0] != 0 or partition[-1] != n:
            raise ValueError('partition must be [0, ..., len(layers)] with one entry per stage boundary')
        r = get_rank() if rank is None else rank
        self.stage_id = topology.get_coord(r).pipe
        self.parts = partition
        lo, hi = partition[self.stage_id], partition[self.stage_id + 1]
        self.layers = torch.nn.ModuleList([layers[i]() for i in range(lo, hi)])

    def topology(self) -> ProcessTopology:
        return self._topo

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for layer in self.layers:
            x = layer(x)
        return x
