"""Tensor/pipeline-parallel K-FAC preconditioner (experimental)
(reference ``kfac/gpt_neox/preconditioner.py:39-512``).

Registers only ``ColumnParallelLinear`` ("output"-sharded) and
``RowParallelLinear`` ("input"-sharded) modules, matched by lower-cased
class name; balances the second-order work over each pipeline stage's peers
(``GPTNeoXAssignment``); EIGEN method only.

Checkpointing: ``state_dict()`` collects every layer's factors from its
inverse worker by per-layer RCCL broadcasts (the reference pickles CPU
copies through ``all_gather_object`` on an extra gloo group) and returns
them on every rank as CPU tensors in the reference layout; with
``factor_checkpoint_dir`` each inverse worker also writes
``<dir>/<layer name>`` files (``torch.save`` of ``{'A', 'G'}``), loaded back
with ``weights_only=True``.
"""
from __future__ import annotations

import logging
import os
import warnings
from typing import Any
from typing import Callable

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.base_preconditioner import BaseKFACPreconditioner
from distributed_kfac_pytorch_amd.enums import AllreduceMethod
from distributed_kfac_pytorch_amd.enums import AssignmentStrategy
from distributed_kfac_pytorch_amd.enums import ComputeMethod
from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.register import any_match
from distributed_kfac_pytorch_amd.layers.register import get_flattened_modules
from distributed_kfac_pytorch_amd.layers.register import requires_grad
from distributed_kfac_pytorch_amd.neox.assignment import GPTNeoXAssignment
from distributed_kfac_pytorch_amd.neox.layer import GPTNeoXKFACEigenLayer
from distributed_kfac_pytorch_amd.neox.modules import GPTNeoXLinearModuleHelper
from distributed_kfac_pytorch_amd.neox.topology import ProcessTopology
from distributed_kfac_pytorch_amd.ops import precondition as pops
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import TorchDistributedCommunicator
from distributed_kfac_pytorch_amd.warnings import ExperimentalFeatureWarning

logger = logging.getLogger(__name__)


class GPTNeoXKFACPreconditioner(BaseKFACPreconditioner):
    """K-FAC for Megatron-style TP / PP models (MEM-OPT per pipeline stage)."""

    def __init__(
        self,
        model: torch.nn.Module,
        *,
        factor_update_steps: Callable[[int], int] | int = 1,
        inv_update_steps: Callable[[int], int] | int = 1,
        damping: Callable[[int], float] | float = 0.001,
        factor_decay: Callable[[int], float] | float = 0.95,
        kl_clip: Callable[[int], float] | float | None = 0.001,
        lr: Callable[[int], float] | float = 0.1,
        accumulation_steps: int = 1,
        allreduce_bucket_cap_mb: float = 25.0,
        assignment_strategy: AssignmentStrategy | str = AssignmentStrategy.COMPUTE,
        compute_method: ComputeMethod | str = ComputeMethod.EIGEN,
        compute_eigenvalue_outer_product: bool = False,
        symmetry_aware: bool = False,
        data_parallel_group: dist.ProcessGroup | None = None,
        model_parallel_group: dist.ProcessGroup | None = None,
        pipeline_parallel_group: dist.ProcessGroup | None = None,
        grad_scaler: torch.cuda.amp.GradScaler | Callable[[], float] | None = None,
        factor_dtype: torch.dtype | None = None,
        inv_dtype: torch.dtype = torch.float32,
        factor_checkpoint_dir: str | None = None,
        skip_layers: list[str] | None = None,
        update_factors_in_hook: bool = True,
        loglevel: int = logging.DEBUG,
    ) -> None:
        """Init GPTNeoXKFACPreconditioner (arguments as ``KFACPreconditioner``
        plus the DP / MP / PP groups and ``factor_checkpoint_dir``)."""
        warnings.warn(
            'KFAC support for GPT-NeoX training is experimental.',
            ExperimentalFeatureWarning,
        )
        topo_fn = getattr(model, 'topology', None)
        if topo_fn is None or not isinstance(topo_fn(), ProcessTopology):
            raise ValueError(
                'model must provide topology() returning a ProcessTopology '
                '(e.g. neox.pipeline.PipelineModule). Got an instance of '
                f'{type(model)}.',
            )
        if allreduce_bucket_cap_mb < 0:
            raise ValueError('allreduce_bucket_cap_mb must be >= 0')
        if isinstance(assignment_strategy, str):
            assignment_strategy = AssignmentStrategy[assignment_strategy.upper()]
        if isinstance(compute_method, str):
            compute_method = ComputeMethod[compute_method.upper()]
        if compute_method == ComputeMethod.INVERSE:
            raise ValueError('Inverse method not supported with GPT NeoX.')
        self.allreduce_bucket_cap_mb = allreduce_bucket_cap_mb
        self.assignment_strategy = assignment_strategy
        self.compute_eigenvalue_outer_product = compute_eigenvalue_outer_product
        self.compute_method = compute_method
        self.grad_scaler = grad_scaler
        self.factor_dtype = factor_dtype
        self.inv_dtype = inv_dtype
        self.factor_checkpoint_dir = factor_checkpoint_dir
        self.skip_layers = [] if skip_layers is None else skip_layers
        self.symmetry_aware = symmetry_aware
        self.data_parallel_group = data_parallel_group
        self.model_parallel_group = model_parallel_group
        self.pipeline_parallel_group = pipeline_parallel_group
        self.allreduce_method = (
            AllreduceMethod.ALLREDUCE_BUCKETED
            if allreduce_bucket_cap_mb > 0
            else AllreduceMethod.ALLREDUCE
        )
        self.tdc = TorchDistributedCommunicator(bucket_cap_mb=allreduce_bucket_cap_mb)
        layer_kwargs = dict(
            allreduce_method=self.allreduce_method,
            grad_scaler=self.grad_scaler,
            factor_dtype=self.factor_dtype,
            inv_dtype=self.inv_dtype,
            symmetry_aware=self.symmetry_aware,
            tdc=self.tdc,
            prediv_eigenvalues=self.compute_eigenvalue_outer_product,
        )
        kfac_layers = register_modules(
            model,
            model_parallel_group=self.model_parallel_group,
            skip_layers=self.skip_layers,
            **layer_kwargs,
        )
        for name, layer in kfac_layers.values():
            logger.log(loglevel, f'Registered name="{name}": {layer!r} on global-rank={get_rank()}')

        power = 3 if assignment_strategy == AssignmentStrategy.COMPUTE else 2

        def cost(n: int) -> float:
            return float(n) ** power
        work = {
            name: {
                'A': cost(layer.module.a_factor_shape[0]),
                'G': cost(layer.module.g_factor_shape[0]),
            }
            for name, layer in kfac_layers.values()
        }
        assignment = GPTNeoXAssignment(
            work,
            local_rank=get_rank(),
            topology=model.topology(),
            data_parallel_group=self.data_parallel_group,
            model_parallel_group=self.model_parallel_group,
        )
        logger.log(loglevel, f'KFAC layer assignments: {assignment}')
        for name, layer in kfac_layers.values():
            assert isinstance(layer, GPTNeoXKFACEigenLayer)
            layer.primary_rank = assignment.factor_worker(name, 'A')
            layer.data_parallel_group = self.data_parallel_group
            layer.pipe_parallel_peer_group = assignment.pipe_parallel_peer_group

        defaults = {
            'allreduce_bucket_cap_mb': self.allreduce_bucket_cap_mb,
            'allreduce_method': self.allreduce_method,
            'assignment_strategy': self.assignment_strategy,
            'compute_eigenvalue_outer_product': self.compute_eigenvalue_outer_product,
            'compute_method': self.compute_method,
            'grad_scaler': self.grad_scaler is not None,
            'factor_checkpoint_dir': self.factor_checkpoint_dir,
            'factor_dtype': self.factor_dtype,
            'inv_dtype': self.inv_dtype,
            'skip_layers': self.skip_layers,
            'symmetry_aware': self.symmetry_aware,
        }
        super().__init__(
            kfac_layers,
            factor_update_steps=factor_update_steps,
            inv_update_steps=inv_update_steps,
            factor_decay=factor_decay,
            damping=damping,
            kl_clip=kl_clip,
            lr=lr,
            accumulation_steps=accumulation_steps,
            assignment=assignment,
            update_factors_in_hook=update_factors_in_hook,
            defaults=defaults,
            tdc=self.tdc,
            loglevel=loglevel,
        )

    # ------------------------------------------------------- precondition
    def _precondition_all(self, ordered: list) -> None:
        """Three phases over ALL layers instead of gather / GEMMs / scatter
        per layer: (1) every layer's gradient is gathered to its primary,
        (2) each rank preconditions the layers it is primary for -- one
        grouped MFMA launch set on the GPU (``GroupedPrecondition``), the
        stock per-layer math otherwise, (3) one scatter per layer returns the
        shards.  Collectives are issued in the same layer order on every MP
        rank.  Data-parallel replicas then receive from their grad worker
        (bucketed broadcasts, as the base preconditioner)."""
        damping = self.damping
        workers = [layer for name, layer in ordered if self._assignment.is_grad_worker(name)]
        for layer in workers:
            layer.gather_full_grad()
        mine = [layer for layer in workers if layer._is_primary()]
        for layer in mine:
            if layer.qa is None or layer.qg is None:
                raise RuntimeError('Eigendecompositions for both A and G have not been computed')
        grouped = False
        if mine and mine[0].module.device.type == 'cuda':
            if self._grouped is None:
                self._grouped = pops.make_grouped()
            grouped = self._grouped.run(mine, damping)
        if not grouped:
            for layer in mine:
                KFACEigenLayer.preconditioned_grad(layer, damping)
        for layer in workers:
            layer.scatter_grad()
        for name, layer in ordered:
            layer.broadcast_grad(
                src=self._assignment.src_grad_worker(name),
                group=self._assignment.grad_receiver_group(name),
                bucketed=True,
            )
        self._tdc.flush_broadcast_buckets()
        self._tdc.flush_allreduce_buckets()

    # ------------------------------------------------------------ KL clip
    def _kl_reduce(self, vg: torch.Tensor) -> None:
        """Sum the per-rank KL partial over the model-parallel (and, if
        given, pipeline) group, in place."""
        from distributed_kfac_pytorch_amd.parallel.comm import get_world_size

        if not dist.is_initialized():
            return
        if get_world_size(self.model_parallel_group) > 1:
            dist.all_reduce(vg, group=self.model_parallel_group)
        if self.pipeline_parallel_group is not None and get_world_size(
            self.pipeline_parallel_group,
        ) > 1:
            dist.all_reduce(vg, group=self.pipeline_parallel_group)

    def _kl_needs_reduce(self) -> bool:
        from distributed_kfac_pytorch_amd.parallel.comm import get_world_size

        return dist.is_initialized() and (
            get_world_size(self.model_parallel_group) > 1
            or (self.pipeline_parallel_group is not None
                and get_world_size(self.pipeline_parallel_group) > 1)
        )

    def _apply_gradients(self, ordered: list, kl: float | None) -> None:
        """KL clip over the WHOLE model: each rank sums <P, grad> over its
        shards (a replicated row-parallel bias weighted 1/mp), the partial
        sums are all-reduced over the model-parallel group (and the pipeline
        group, if given), and every shard is scaled by the same factor.  The
        reference (``kfac/gpt_neox/preconditioner.py``) sums only rank-local
        shards, so its MP ranks clip with different scales.

        GPU: the native multi-tensor path (``MultiLayerApply``): one
        KL-partials launch, a fixed-order fold to one fp64 scalar, ONE
        all-reduce of that scalar, the finalise and one apply launch for the
        whole model.  CPU / fallback: per-layer fp64 torch reductions."""
        if not ordered:
            return
        layers = [layer for _, layer in ordered]
        if self._multi_apply is None:
            self._multi_apply = pops.MultiLayerApply()
        reduce_fn = self._kl_reduce if kl is not None and self._kl_needs_reduce() else None
        if self._multi_apply.run(layers, kl, float(self.lr) if kl is not None else 0.0,
                                 reduce_fn=reduce_fn):
            return
        if kl is None:
            for layer in layers:
                layer.update_grad(scale=None)
            return
        dev = layers[0].module.device
        vg = torch.zeros(1, dtype=torch.float64, device=dev)
        for layer in layers:
            p = layer.grad
            if p is None:
                raise AssertionError('layer gradient has not been preconditioned')
            m = layer.module
            wm = m.weight_grad_matrix()
            ncol = wm.shape[1]
            vg += (p[:, :ncol].double() * wm.double()).sum()
            if m.has_bias():
                vg += (p[:, ncol].double() * m.get_bias_grad().double()).sum() * layer.kl_bias_scale
        if self._kl_needs_reduce():
            self._kl_reduce(vg)
        lr = float(self.lr)
        vg = (vg * lr * lr).abs()
        scale = torch.where(
            vg == 0,
            torch.ones_like(vg),
            torch.clamp(torch.sqrt(float(kl) / vg), max=1.0),
        ).float()
        for layer in layers:
            layer.update_grad(scale=scale)

    # ------------------------------------------------------------ checkpoint
    def state_dict(self, include_factors: bool = True) -> dict[str, Any]:
        """All ranks must enter.  Factors are collected from each layer's
        inverse worker and returned on every rank (CPU tensors)."""
        self._join_factor_streams()
        sd = super().state_dict(include_factors=False)
        if not include_factors:
            return sd
        if self.factor_checkpoint_dir is not None:
            # factors live in the per-layer files: the dict stays small
            # (reference ``kfac/gpt_neox/preconditioner.py:350-363``)
            self.save_factors_to_dir()
            return sd
        me = get_rank()
        layers: dict[str, dict[str, torch.Tensor]] = {}
        for name, layer in self._layers.values():
            owner = self._assignment.inv_worker(name, 'A')
            out = {}
            for f, shape in (('A', layer.module.a_factor_shape), ('G', layer.module.g_factor_shape)):
                if me == owner:
                    t = layer.a_factor if f == 'A' else layer.g_factor
                    if t is None:
                        raise RuntimeError(f'{name}: factor {f} not computed on its inverse worker')
                    t = t.contiguous()
                else:
                    dt = self.factor_dtype or torch.float32
                    t = torch.empty(shape, dtype=dt, device=layer.module.device)
                if dist.is_initialized() and dist.get_world_size() > 1:
                    dist.broadcast(t, src=owner)
                out[f] = t.cpu()
            layers[name] = out
        sd['layers'] = layers
        return sd

    def load_state_dict(self, state_dict: dict[str, Any], compute_inverses: bool = True) -> None:
        """Restore hyperparameters; load factors on their primary ranks."""
        self._join_factor_streams()
        state_dict = dict(state_dict)
        layers = state_dict.pop('layers', None)
        super().load_state_dict(state_dict, compute_inverses=False)
        if self.factor_checkpoint_dir is not None:
            # the per-layer files are the source of truth (reference
            # ``kfac/gpt_neox/preconditioner.py:314-328``)
            self.load_factors_from_dir(compute_inverses)
            return
        if layers is None:
            return
        me = get_rank()
        for name, layer in self._layers.values():
            if name in layers and self._assignment.factor_worker(name, 'A') == me:
                layer.load_state_dict(layers[name])
                if compute_inverses:
                    layer.compute_a_inv(damping=self.damping)
                    layer.compute_g_inv(damping=self.damping)
        if dist.is_initialized():
            dist.barrier()

    def save_factors_to_dir(self) -> None:
        """Each inverse worker writes ``<dir>/<layer name>`` for its layers."""
        self._join_factor_streams()
        if self.factor_checkpoint_dir is None:
            raise ValueError('factor_checkpoint_dir is None')
        if get_rank() == 0:
            os.makedirs(self.factor_checkpoint_dir, exist_ok=True)
        if dist.is_initialized():
            dist.barrier()
        for name, layer in self._layers.values():
            if get_rank() == self._assignment.inv_worker(name, 'A'):
                path = os.path.join(self.factor_checkpoint_dir, name)
                logger.info(f'saving KFAC factors for {name} to {path}')
                torch.save(layer.state_dict(), path)
        if dist.is_initialized():
            dist.barrier()  # every file is complete when any rank returns

    def load_factors_from_dir(self, compute_inverses: bool = True) -> None:
        """Load per-layer factor files on the primary ranks (missing files
        are skipped)."""
        self._join_factor_streams()
        if self.factor_checkpoint_dir is None:
            raise ValueError('factor_checkpoint_dir is None.')
        if not os.path.isdir(self.factor_checkpoint_dir):
            warnings.warn(
                f'factor_checkpoint_dir={self.factor_checkpoint_dir} is not a '
                'directory. Skipping KFAC checkpoint load.',
            )
            return
        me = get_rank()
        for name, layer in self._layers.values():
            if self._assignment.factor_worker(name, 'A') != me:
                continue
            path = os.path.join(self.factor_checkpoint_dir, name)
            if not os.path.exists(path):
                continue
            logger.info(f'loading KFAC factors for {name} on rank {me}')
            layer.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
            if compute_inverses:
                layer.compute_a_inv(damping=self.damping)
                layer.compute_g_inv(damping=self.damping)


def register_modules(
    model: torch.nn.Module,
    model_parallel_group: dist.ProcessGroup | None,
    skip_layers: list[str],
    **layer_kwargs: Any,
) -> dict[torch.nn.Module, tuple[str, KFACBaseLayer]]:
    """Register Column/RowParallelLinear modules (by lower-cased class name;
    ``skip_layers`` regexes are matched against names and lower-cased class
    names)."""
    layers: dict[torch.nn.Module, tuple[str, KFACBaseLayer]] = {}
    for name, module in get_flattened_modules(model):
        cls = module.__class__.__name__.lower()
        if any_match(name, skip_layers) or any_match(cls, skip_layers):
            continue
        if not requires_grad(module):
            continue
        if cls == 'columnparallellinear':
            parallelism = 'output'
        elif cls == 'rowparallellinear':
            parallelism = 'input'
        else:
            continue
        helper = GPTNeoXLinearModuleHelper(module, model_parallel_group, parallelism)
        layers[module] = (
            name,
            GPTNeoXKFACEigenLayer(
                helper,
                parallelism=parallelism,
                model_parallel_group=model_parallel_group,
                **layer_kwargs,
            ),
        )
    return layers
