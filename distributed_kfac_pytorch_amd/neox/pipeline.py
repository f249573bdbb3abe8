"""Pipeline-parallel stage container and micro-batch schedule.

The reference GPT-NeoX preconditioner requires a DeepSpeed ``PipelineModule``
(``kfac/gpt_neox/preconditioner.py:159-163``) and uses it for its module tree
and ``model.topology()``; DeepSpeed's engine runs the micro-batch schedule.
DeepSpeed is not part of this stack, so both halves live here:

* ``PipelineModule`` instantiates only the layers of this rank's pipeline
  stage (contiguous, balanced partition by layer count unless ``partition``
  is given) and exposes ``topology()``;
* ``PipelineModule.train_batch`` runs one optimizer step's worth of
  micro-batches through the stages with a GPipe schedule (all forwards,
  then all backwards in reverse micro-batch order): activations go to the
  next stage and activation gradients back with point-to-point
  ``dist.send`` / ``dist.recv`` (RCCL p2p over xGMI on MI355X, gloo on the
  CPU) between the ranks that share the data and model coordinates;
* ``allreduce_gradients`` averages the stage's gradients over its
  data-parallel group (DDP's reducer assumes one forward per backward, a
  pipeline runs several).

K-FAC: construct ``GPTNeoXKFACPreconditioner`` on the stage module with
``accumulation_steps`` = the number of micro-batches; each stage's layers
accumulate their factors over the micro-batches (forward and backward
contributions are counted separately, so the GPipe order -- every forward
before any backward -- folds the full step's statistics exactly once) and
the KL clip sums over the stages through ``pipeline_parallel_group``.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.neox.topology import ProcessTopology
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size


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
        self.global_rank = r
        self.num_stages = stages
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

    # -------------------------------------------------------------- schedule
    @property
    def is_first_stage(self) -> bool:
        return self.stage_id == 0

    @property
    def is_last_stage(self) -> bool:
        return self.stage_id == self.num_stages - 1

    def _peer(self, delta: int) -> int:
        c = self._topo.get_coord(self.global_rank)
        return self._topo.get_rank(pipe=c.pipe + delta, data=c.data, model=c.model)

    def train_batch(
        self,
        inputs: torch.Tensor | None,
        labels: torch.Tensor | None,
        loss_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
        micro_batches: int,
        activation_shape: tuple[int, ...],
        activation_dtype: torch.dtype = torch.float32,
        autocast_dtype: torch.dtype | None = None,
    ) -> torch.Tensor | None:
        """Forward + backward of one batch as ``micro_batches`` micro-batches
        (GPipe).  ``inputs`` is needed on the first stage, ``labels`` on the
        last; ``activation_shape`` is the shape of one micro-batch's
        inter-stage activation.  Gradients accumulate into ``.grad`` (the
        loss is the micro-batch mean); returns the batch loss on the last
        stage, None elsewhere."""
        m = micro_batches
        dev = next(self.parameters()).device
        xs = inputs.chunk(m) if self.is_first_stage and inputs is not None else None
        ys = labels.chunk(m) if self.is_last_stage and labels is not None else None
        saved: list[tuple[torch.Tensor | None, torch.Tensor]] = []
        total = torch.zeros((), device=dev)

        def run(x: torch.Tensor) -> torch.Tensor:
            if autocast_dtype is None:
                return self(x)
            with torch.autocast(dev.type, dtype=autocast_dtype):
                return self(x)

        for i in range(m):
            if self.is_first_stage:
                assert xs is not None, 'the first stage needs inputs'
                x_in = None
                out = run(xs[i])
            else:
                x_in = torch.empty(activation_shape, dtype=activation_dtype, device=dev)
                dist.recv(x_in, src=self._peer(-1))
                x_in.requires_grad_()
                out = run(x_in)
            if self.is_last_stage:
                assert ys is not None, 'the last stage needs labels'
                loss = loss_fn(out, ys[i]) / m
                total += loss.detach()
                saved.append((x_in, loss))
            else:
                dist.send(out.detach().to(activation_dtype).contiguous(), dst=self._peer(1))
                saved.append((x_in, out))
        for i in reversed(range(m)):
            x_in, out = saved[i]
            if self.is_last_stage:
                out.backward()
            else:
                g = torch.empty(out.shape, dtype=activation_dtype, device=dev)
                dist.recv(g, src=self._peer(1))
                torch.autograd.backward(out, g.to(out.dtype))
            if x_in is not None:
                dist.send(x_in.grad.contiguous(), dst=self._peer(-1))
            saved[i] = (None, out.detach())
        return total if self.is_last_stage else None


def allreduce_gradients(module: torch.nn.Module, group: dist.ProcessGroup | None) -> None:
    """Average ``.grad`` over ``group`` (the stage's data-parallel peers)
    through one flat buffer per dtype."""
    world = get_world_size(group)
    if world == 1:
        return
    by_dtype: dict[torch.dtype, list[torch.Tensor]] = {}
    for p in module.parameters():
        if p.grad is not None:
            by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
    for grads in by_dtype.values():
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, group=group)
        flat.mul_(1.0 / world)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off: off + n].view_as(g))
            off += n
