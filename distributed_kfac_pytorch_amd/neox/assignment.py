"""Pipeline/tensor-parallel-aware work placement
(reference ``kfac/gpt_neox/assignment.py:1-235``).

Semantics (MEM-OPT over each pipeline stage):

* a layer's factors are decomposed on ONE rank among its pipeline-stage
  peers (ranks with the same pipe coordinate), chosen by greedy LPT on the
  summed factor cost (ties by layer name, descending); factors are always
  colocated;
* every rank of that inverse worker's model-parallel group is a gradient
  worker (they all take part in the gathered/scattered preconditioning);
* the preconditioned shards are broadcast over the data-parallel group from
  the rank of the inverse worker's MP group with the same model coordinate;
* inverses are never broadcast; factors are reduced by the layer itself
  (DP group for the sharded side, pipe-stage peers for the replicated side).
"""
from __future__ import annotations

from typing import Any
from typing import Callable

import torch.distributed as dist

from distributed_kfac_pytorch_amd.neox.mpu import get_group_with_rank
from distributed_kfac_pytorch_amd.neox.topology import ProcessTopology
from distributed_kfac_pytorch_amd.parallel.assignment import WorkAssignment


class GPTNeoXAssignment(WorkAssignment):
    def __init__(
        self,
        work: dict[str, dict[str, float]],
        *,
        local_rank: int,
        topology: ProcessTopology,
        data_parallel_group: dist.ProcessGroup | None,
        model_parallel_group: dist.ProcessGroup | None,
        group_func: Callable[[list[int]], Any] | None = None,
    ) -> None:
        """Init GPTNeoXAssignment.

        Args:
            work: ``{layer: {factor: cost}}`` for the layers of this stage.
            local_rank: global rank of this process.
            topology: (pipe, data, model) topology.
            data_parallel_group: this rank's DP group handle.
            model_parallel_group: this rank's MP group handle.
            group_func: creates a group for the pipe-stage peers when it is
                neither the DP nor the MP group (default ``dist.new_group``).
        """
        if not isinstance(topology, ProcessTopology):
            raise TypeError(
                f'Expected topology to be a ProcessTopology but got {type(topology)}.',
            )
        self.local_rank = local_rank
        self.topology = topology
        self.data_parallel_group = data_parallel_group
        self.model_parallel_group = model_parallel_group
        self.data_parallel_groups = topology.get_axis_comm_lists('data')
        self.model_parallel_groups = topology.get_axis_comm_lists('model')
        self.pipe_parallel_groups = topology.get_axis_comm_lists('pipe')
        self.data_parallel_peers = get_group_with_rank(local_rank, self.data_parallel_groups)
        self.model_parallel_peers = get_group_with_rank(local_rank, self.model_parallel_groups)
        self.pipe_parallel_rank = topology.get_coord(local_rank).pipe
        self.pipe_parallel_peers = [
            r for r in range(topology.world_size())
            if topology.get_coord(r).pipe == self.pipe_parallel_rank
        ]
        if set(self.pipe_parallel_peers) == set(self.model_parallel_peers):
            self.pipe_parallel_peer_group = model_parallel_group
        elif set(self.pipe_parallel_peers) == set(self.data_parallel_peers):
            self.pipe_parallel_peer_group = data_parallel_group
        else:
            # every rank must enter every group creation, in the same order
            # (torch.distributed.new_group); the reference creates only its
            # own stage's group (kfac/gpt_neox/assignment.py:86-92), which
            # deadlocks once pp > 1 and the stage peers are neither the DP
            # nor the MP group
            make = group_func if group_func is not None else dist.new_group
            self.pipe_parallel_peer_group = None
            for stage in range(topology.get_dim('pipe')):
                peers = [r for r in range(topology.world_size())
                         if topology.get_coord(r).pipe == stage]
                g = make(peers)
                if stage == self.pipe_parallel_rank:
                    self.pipe_parallel_peer_group = g

        loads = [0.0] * len(self.pipe_parallel_peers)
        self._inv_assignments: dict[str, dict[str, int]] = {
            layer: {f: -1 for f in fs} for layer, fs in work.items()
        }
        ranked = sorted(
            ((layer, sum(fs.values())) for layer, fs in work.items()),
            key=lambda kv: (kv[1], kv[0]),
            reverse=True,
        )
        for layer, cost in ranked:
            i = loads.index(min(loads))
            for f in self._inv_assignments[layer]:
                self._inv_assignments[layer][f] = self.pipe_parallel_peers[i]
            loads[i] += cost

    def broadcast_gradients(self) -> bool:
        return True

    def broadcast_inverses(self) -> bool:
        return False

    def get_layers(self) -> tuple[str, ...]:
        return tuple(self._inv_assignments)

    def get_factors(self, layer: str) -> tuple[str, ...]:
        return tuple(self._inv_assignments[layer])

    def inv_worker(self, layer: str, factor: str) -> int:
        return self._inv_assignments[layer][factor]

    def _owner(self, layer: str) -> int:
        owners = set(self._inv_assignments[layer].values())
        assert len(owners) == 1
        return owners.pop()

    def factor_worker(self, layer: str, factor: str) -> int:
        """The rank of MY model-parallel group that owns the full factors
        (the 'primary'): the one sharing the inverse worker's DP group."""
        dp = get_group_with_rank(self._owner(layer), self.data_parallel_groups)
        both = set(dp) & set(self.model_parallel_peers)
        assert len(both) == 1
        return both.pop()

    def is_grad_worker(self, layer: str) -> bool:
        return self._owner(layer) in self.model_parallel_peers

    def src_grad_worker(self, layer: str) -> int:
        mp = get_group_with_rank(self._owner(layer), self.model_parallel_groups)
        both = set(self.data_parallel_peers) & set(mp)
        assert len(both) == 1
        return both.pop()

    def factor_group(self, layer: str, factor: str) -> dist.ProcessGroup | None:
        return None

    def grad_worker_group(self, layer: str) -> dist.ProcessGroup | None:
        raise NotImplementedError(
            'The GPT-NeoX assignment only supports MEM-OPT and never '
            'broadcasts inverses.',
        )

    def grad_receiver_group(self, layer: str) -> dist.ProcessGroup | None:
        return self.data_parallel_group
