"""Test doubles (the role of reference ``testing/assignment.py``)."""
from __future__ import annotations

import torch.distributed as dist

from distributed_kfac_pytorch_amd.parallel.assignment import WorkAssignment


class LazyAssignment(WorkAssignment):
    """Every rank is inverse worker and grad worker for every layer; all
    groups are the world; broadcasting is a switch.  Drives every branch of
    the preconditioner in one process."""

    def __init__(self, rank: int = 0, broadcast: bool = False) -> None:
        self.rank = rank
        self.broadcast = broadcast

    def broadcast_gradients(self) -> bool:
        return self.broadcast

    def broadcast_inverses(self) -> bool:
        return self.broadcast

    def get_layers(self) -> tuple[str, ...]:
        return ()

    def get_factors(self, layer: str) -> tuple[str, ...]:
        return ('A', 'G')

    def inv_worker(self, layer: str, factor: str) -> int:
        return self.rank

    def is_grad_worker(self, layer: str) -> bool:
        return True

    def src_grad_worker(self, layer: str) -> int:
        return self.rank

    def factor_group(self, layer: str, factor: str) -> dist.ProcessGroup | None:
        return None

    def grad_worker_group(self, layer: str) -> dist.ProcessGroup | None:
        return None

    def grad_receiver_group(self, layer: str) -> dist.ProcessGroup | None:
        return None
