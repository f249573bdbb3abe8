"""Model-parallel-aware eigen layer (reference ``kfac/gpt_neox/layer.py``).

Row-parallel ("input") layers gather their sharded input to the primary
rank of the model-parallel (MP) group, which owns the full A factor and
all-reduces it over its data-parallel (DP) group; G is replicated across MP
ranks and all-reduced over the pipeline-stage peers.  Column-parallel
("output") layers mirror this for G.  Preconditioning (reference
``kfac/gpt_neox/layer.py:203-310``) gathers the weight (and sharded bias)
gradient to the primary, preconditions the full matrix and scatters the
shards back -- with a true ``dist.gather`` into persistent buffers and ONE
``dist.scatter`` of [weight shard | bias] per layer (see ``neox/mpu.py``)
rather than the reference's all-gather / zero-padded reduce-scatter
emulation.  The preconditioner runs the three phases over all layers, so
the primary's GEMMs are one grouped MFMA launch (``ops/precondition.py``).
"""
from __future__ import annotations

from typing import Any
from typing import Literal

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.neox.mpu import gather_from_model_parallel_region
from distributed_kfac_pytorch_amd.neox.mpu import scatter_to_model_parallel_region
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size

_UNSET = -1


class GPTNeoXKFACEigenLayer(KFACEigenLayer):
    """Eigen layer for Column/Row-parallel linears."""

    def __init__(
        self,
        module: Any,
        *,
        parallelism: Literal['input', 'output'],
        model_parallel_group: dist.ProcessGroup | None,
        data_parallel_group: dist.ProcessGroup | None | int = _UNSET,
        pipe_parallel_peer_group: dist.ProcessGroup | None | int = _UNSET,
        primary_rank: int | None = None,
        **kwargs: Any,
    ) -> None:
        self.parallelism = parallelism
        self.primary_rank = primary_rank
        self.data_parallel_group = data_parallel_group
        self.model_parallel_group = model_parallel_group
        self.pipe_parallel_peer_group = pipe_parallel_peer_group
        super().__init__(module, **kwargs)
        # persistent MP buffers (primary only): gathered full Wg / bias grad,
        # full P, row-parallel gather staging and scatter packing
        self._full_w: torch.Tensor | None = None
        self._full_b: torch.Tensor | None = None
        self._full_p: torch.Tensor | None = None
        self._gather_w: torch.Tensor | None = None
        self._scatter_p: torch.Tensor | None = None

    # --------------------------------------------------------------- checks
    def _check(self) -> None:
        if self.primary_rank is None:
            raise RuntimeError('primary rank has not been set yet.')
        if isinstance(self.data_parallel_group, int) or isinstance(
            self.pipe_parallel_peer_group, int,
        ):
            raise RuntimeError(
                'data_parallel_group or pipe_parallel_peer_group has not been '
                'set yet.',
            )

    def _is_primary(self) -> bool:
        return get_rank() == self.primary_rank

    # ------------------------------------------------------------ reductions
    def reduce_a_factor(self, group: dist.ProcessGroup | None = None) -> None:
        self._check()
        if self.parallelism == 'input':
            if not self._is_primary():
                return
            super().reduce_a_factor(self.data_parallel_group)  # type: ignore[arg-type]
        else:
            super().reduce_a_factor(self.pipe_parallel_peer_group)  # type: ignore[arg-type]

    def reduce_g_factor(self, group: dist.ProcessGroup | None = None) -> None:
        self._check()
        if self.parallelism == 'input':
            super().reduce_g_factor(self.pipe_parallel_peer_group)  # type: ignore[arg-type]
        else:
            if not self._is_primary():
                return
            super().reduce_g_factor(self.data_parallel_group)  # type: ignore[arg-type]

    # ---------------------------------------------------------- accumulation
    def _gather_input(self, a: torch.Tensor) -> torch.Tensor | None:
        if self.module.input_sharded:
            return gather_from_model_parallel_region(
                a, dst=self.primary_rank, model_parallel_group=self.model_parallel_group,
            )
        return a

    def _gather_grad(self, g: torch.Tensor) -> torch.Tensor | None:
        if self.module.output_sharded:
            return gather_from_model_parallel_region(
                g, dst=self.primary_rank, model_parallel_group=self.model_parallel_group,
            )
        return g

    def save_layer_input(self, input: list[torch.Tensor]) -> None:
        self._check()
        a = self._gather_input(input[0])
        if a is not None:
            self._save_a(a)

    def save_layer_grad_output(self, grad_output: tuple[torch.Tensor, ...]) -> None:
        self._check()
        g = self._gather_grad(grad_output[0])
        if g is not None:
            self._save_g(g)

    def save_and_update_a(self, input: list[torch.Tensor], alpha: float) -> None:
        self._check()
        a = self._gather_input(input[0])
        if a is not None:
            self._save_and_update_a(a, alpha)

    def save_and_update_g(self, grad_output: tuple[torch.Tensor, ...], alpha: float) -> None:
        self._check()
        g = self._gather_grad(grad_output[0])
        if g is not None:
            self._save_and_update_g(g, alpha)

    # ------------------------------------------------------------- gradients
    # The stock eigen math (``KFACEigenLayer.preconditioned_grad``, or the
    # grouped MFMA GEMM of ``ops.precondition.GroupedPrecondition``) runs on
    # the primary over the gathered FULL gradient: ``precond_operands`` /
    # ``precond_out`` point it at persistent full-size buffers.
    stock_precondition_math = True

    def _mp_world(self) -> int:
        return get_world_size(self.model_parallel_group)

    @property
    def kl_bias_scale(self) -> float:
        """A row-parallel bias gradient is replicated on every MP rank: each
        counts 1/mp of it so the MP all-reduce of the KL sum counts it once."""
        if self.parallelism == 'input' and self.module.has_bias():
            return 1.0 / max(1, self._mp_world())
        return 1.0

    def grad_shape(self) -> tuple[int, int]:
        w = self.module.module.weight
        return (w.shape[0], w.shape[1] + int(self.module.has_bias()))

    def _full_shape(self) -> tuple[int, int]:
        return (self.module.g_factor_shape[0], self.module.a_factor_shape[0])

    def precond_operands(self) -> tuple[torch.Tensor, torch.Tensor | None, bool]:
        if self._mp_world() == 1:
            return super().precond_operands()
        if self._full_w is None:
            raise RuntimeError('gather_full_grad() must run before preconditioning')
        return self._full_w, self._full_b, True

    def precond_out(self, device: torch.device) -> torch.Tensor:
        if self._mp_world() == 1:
            return self._grad_buffer(device)
        return self._buf('_full_p', self._full_shape(), torch.float32, device)

    def gather_full_grad(self) -> None:
        """Collective over the MP group: assemble the full weight (and bias)
        gradient in persistent buffers on the primary.  Column-parallel
        shards are row blocks, gathered straight into the full matrix;
        row-parallel shards are column blocks, gathered into a staging
        buffer and interleaved with one copy (the replicated bias is local)."""
        self._check()
        world = self._mp_world()
        if world == 1:
            return
        mp = self.model_parallel_group
        primary = self._is_primary()
        w_part = self.module.get_weight_grad().contiguous()
        has_bias = self.module.has_bias()
        b_part = self.module.get_bias_grad().contiguous() if has_bias else None
        dev, dt = w_part.device, w_part.dtype
        rows, cols = w_part.shape
        if self.parallelism == 'output':
            full_w = self._buf('_full_w', (rows * world, cols), dt, dev) if primary else None
            dist.gather(w_part, gather_list=list(full_w.view(world, rows, cols).unbind(0))
                        if primary else None, dst=self.primary_rank, group=mp)
            full_b = None
            if has_bias:
                assert b_part is not None
                full_b = self._buf('_full_b', (rows * world,), b_part.dtype, dev) if primary else None
                dist.gather(b_part, gather_list=list(full_b.view(world, rows).unbind(0))
                            if primary else None, dst=self.primary_rank, group=mp)
        else:
            stage = self._buf('_gather_w', (world, rows, cols), dt, dev) if primary else None
            dist.gather(w_part, gather_list=list(stage.unbind(0)) if primary else None,
                        dst=self.primary_rank, group=mp)
            full_w = full_b = None
            if primary:
                full_w = self._buf('_full_w', (rows, cols * world), dt, dev)
                full_w.view(rows, world, cols).copy_(stage.permute(1, 0, 2))
                full_b = b_part
        if primary:
            self._full_w, self._full_b = full_w, full_b

    def scatter_grad(self) -> None:
        """Collective over the MP group: every rank receives its shard of the
        primary's full P -- weight columns and bias together -- in ONE
        scatter, straight into its persistent local grad buffer (the layout
        ``update_grad`` / the multi-tensor apply read)."""
        world = self._mp_world()
        if world == 1:
            return
        mp = self.model_parallel_group
        primary = self._is_primary()
        local = self._grad_buffer(self.module.device)
        chunks = None
        if primary:
            p = self.grad
            assert p is not None
            if self.parallelism == 'output':
                # row blocks of P are contiguous: scatter views, no copies
                chunks = list(p.view(world, local.shape[0], local.shape[1]).unbind(0))
            else:
                rows, lcols = local.shape
                c = lcols - int(self.module.has_bias())
                pack = self._buf('_scatter_p', (world, rows, lcols), torch.float32, p.device)
                pack[:, :, :c].copy_(p[:, :c * world].view(rows, world, c).permute(1, 0, 2))
                if self.module.has_bias():
                    pack[:, :, c].copy_(p[:, c * world].expand(world, rows))
                chunks = list(pack.unbind(0))
        scatter_to_model_parallel_region(chunks, local, self.primary_rank, mp)
        self.grad = local

    def preconditioned_grad(self, damping: float = 0.001) -> None:
        """Every MP rank enters: gather -> precondition on the primary ->
        scatter (the preconditioner batches these phases over all layers so
        the primary's GEMMs run as one grouped launch)."""
        self._check()
        primary = self._is_primary()
        if primary and (
            self.qa is None
            or self.qg is None
            or (not self.prediv_eigenvalues and (self.da is None or self.dg is None))
            or (self.prediv_eigenvalues and self.dgda is None)
        ):
            raise RuntimeError(
                'Eigendecompositions for both A and G have not been computed',
            )
        self.gather_full_grad()
        if primary:
            KFACEigenLayer.preconditioned_grad(self, damping)
        self.scatter_grad()
