"""Training utilities shared by the example CLIs and the benchmark
(reference ``examples/utils.py``: checkpointing, label smoothing, metrics,
LR schedules), reworked for MI355X:

* ``Metric`` accumulates on the device and all-reduces only when read
  (the reference all-reduces synchronously on every update).
* ``save_checkpoint`` / ``load_checkpoint`` write/read the reference's
  ``{'model', 'optimizer', 'preconditioner', 'lr_scheduler'}`` dict and load
  with ``weights_only=True`` (no pickle code execution).
"""
from __future__ import annotations

import glob
import os
import re
from typing import Any
from typing import Callable

import torch
import torch.distributed as dist


def save_checkpoint(
    model: torch.nn.Module,
    optimizer: torch.optim.Optimizer,
    preconditioner: Any,
    lr_scheduler: Any,
    filepath: str,
) -> None:
    """Save the reference-format training checkpoint (rank 0 should call)."""
    state = {
        'model': model.state_dict(),
        'optimizer': optimizer.state_dict(),
        'preconditioner': (
            preconditioner.state_dict() if preconditioner is not None else None
        ),
        'lr_scheduler': lr_scheduler.state_dict() if lr_scheduler is not None else None,
    }
    d = os.path.dirname(filepath)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = filepath + '.tmp'
    torch.save(state, tmp)
    os.replace(tmp, filepath)


def load_checkpoint(filepath: str, map_location: Any = None) -> dict[str, Any]:
    """Load a checkpoint written by ``save_checkpoint`` (weights only)."""
    return torch.load(filepath, map_location=map_location, weights_only=True)


def latest_checkpoint(pattern: str) -> tuple[str, int] | None:
    """Newest ``checkpoint_{epoch}``-style file matching ``pattern`` (a
    format string with ``{epoch}``), for auto-resume."""
    glob_pat = pattern.replace('{epoch}', '*')
    rx = re.compile(re.escape(pattern).replace(re.escape('{epoch}'), r'(\d+)') + '$')
    best = None
    for f in glob.glob(glob_pat):
        m = rx.search(f)
        if m:
            e = int(m.group(1))
            if best is None or e > best[1]:
                best = (f, e)
    return best


class LabelSmoothLoss(torch.nn.Module):
    """Cross entropy with label smoothing ``s`` (reference examples/utils.py:
    40-62; equivalent to ``CrossEntropyLoss(label_smoothing=s*K/(K-1))``)."""

    def __init__(self, smoothing: float = 0.0) -> None:
        super().__init__()
        self.smoothing = smoothing

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        log_prob = torch.log_softmax(input, dim=-1)
        k = input.shape[-1]
        weight = torch.full_like(log_prob, self.smoothing / (k - 1))
        weight.scatter_(-1, target.unsqueeze(-1), 1.0 - self.smoothing)
        return (-weight * log_prob).sum(dim=-1).mean()


class Metric:
    """Running average kept on the device; reduced across ranks lazily."""

    def __init__(self, name: str, device: torch.device | str = 'cpu') -> None:
        self.name = name
        self._sum = torch.zeros((), dtype=torch.float64, device=device)
        self._n = torch.zeros((), dtype=torch.float64, device=device)

    def update(self, value: torch.Tensor | float, n: int = 1) -> None:
        v = value.detach().to(self._sum) if isinstance(value, torch.Tensor) else value
        self._sum += v * n
        self._n += n

    @property
    def avg(self) -> float:
        t = torch.stack([self._sum, self._n])
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(t)
        return float(t[0] / t[1].clamp(min=1))


def accuracy(output: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Top-1 accuracy as a device scalar."""
    return (output.argmax(dim=1) == target).float().mean()


def create_lr_schedule(
    workers: int,
    warmup_epochs: int,
    decay_schedule: list[int],
    alpha: float = 0.1,
) -> Callable[[int], float]:
    """LambdaLR factor: linear warmup from 1/workers to 1, then x alpha at
    each epoch in ``decay_schedule`` (reference examples/utils.py:91-113)."""

    def lr_schedule(epoch: int) -> float:
        lr_adj = 1.0
        if epoch < warmup_epochs:
            lr_adj = 1.0 / workers * (epoch * (workers - 1) / warmup_epochs + 1)
        else:
            for e in sorted(decay_schedule):
                if epoch >= e:
                    lr_adj *= alpha
        return lr_adj

    return lr_schedule
