"""KAISA K-FAC preconditioner: the user entry point
(reference ``kfac/preconditioner.py:30-330``).

Example::

    model = torch.nn.parallel.DistributedDataParallel(model, ...)
    optimizer = torch.optim.SGD(model.parameters(), ...)
    preconditioner = KFACPreconditioner(model, ...)
    for x, y in loader:
        optimizer.zero_grad()
        loss = criterion(model(x), y)
        loss.backward()
        preconditioner.step()
        optimizer.step()
"""
from __future__ import annotations

import logging
import warnings
from typing import Callable

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.base_preconditioner import (
    BaseKFACPreconditioner,
)
from distributed_kfac_pytorch_amd.enums import AllreduceMethod
from distributed_kfac_pytorch_amd.enums import AssignmentStrategy
from distributed_kfac_pytorch_amd.enums import ComputeMethod
from distributed_kfac_pytorch_amd.enums import DistributedStrategy
from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.inverse import KFACInverseLayer
from distributed_kfac_pytorch_amd.layers.register import register_modules
from distributed_kfac_pytorch_amd.parallel.assignment import KAISAAssignment
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size
from distributed_kfac_pytorch_amd.parallel.comm import (
    TorchDistributedCommunicator,
)

logger = logging.getLogger(__name__)


def resolve_grad_worker_fraction(
    grad_worker_fraction: DistributedStrategy | float,
    world_size: int,
) -> tuple[float, DistributedStrategy]:
    """Map a strategy enum or a fraction to ``(fraction, strategy)``
    (reference ``kfac/preconditioner.py:169-197``)."""
    if isinstance(grad_worker_fraction, DistributedStrategy):
        strategy = grad_worker_fraction
        if strategy == DistributedStrategy.COMM_OPT:
            frac = 1.0
        elif strategy == DistributedStrategy.HYBRID_OPT:
            frac = 0.5
        elif strategy == DistributedStrategy.MEM_OPT:
            frac = 1.0 / world_size
        else:  # pragma: no cover
            raise AssertionError(f'Unknown enum {grad_worker_fraction}')
        return frac, strategy
    frac = float(grad_worker_fraction)
    if not 0 <= frac <= 1:
        raise ValueError('grad_worker_fraction must in [0, 1]')
    if frac == 0:
        frac = 1.0 / world_size
    if world_size % max(1, round(world_size * frac)) != 0:
        raise ValueError('grad_worker_fraction must produce groups of equal size')
    if frac == 1:
        return 1.0, DistributedStrategy.COMM_OPT
    if frac <= 1 / world_size:
        return frac, DistributedStrategy.MEM_OPT
    return frac, DistributedStrategy.HYBRID_OPT


def _add_embeddings(
    model: torch.nn.Module,
    layers: dict,
    compute_method: ComputeMethod,
    skip_layers: list[str],
    layer_kwargs: dict,
) -> dict:
    """Register ``nn.Embedding`` modules too, keeping model order."""
    from distributed_kfac_pytorch_amd.layers.embedding import EmbeddingModuleHelper
    from distributed_kfac_pytorch_amd.layers.embedding import KFACEmbeddingEigenLayer
    from distributed_kfac_pytorch_amd.layers.embedding import KFACEmbeddingInverseLayer
    from distributed_kfac_pytorch_amd.layers.register import get_flattened_modules

    def factory(m: torch.nn.Module) -> EmbeddingModuleHelper | None:
        if isinstance(m, torch.nn.Embedding) and not m.sparse and m.max_norm is None:
            return EmbeddingModuleHelper(m)
        return None

    if compute_method == ComputeMethod.EIGEN:
        emb_type: type[KFACBaseLayer] = KFACEmbeddingEigenLayer
        kw = layer_kwargs
    else:
        emb_type = KFACEmbeddingInverseLayer
        kw = {k: v for k, v in layer_kwargs.items() if k != 'prediv_eigenvalues'}
    emb = register_modules(model, emb_type, skip_layers, helper_factory=factory, **kw)
    merged = {}
    for _, m in get_flattened_modules(model):
        if m in layers:
            merged[m] = layers[m]
        elif m in emb:
            merged[m] = emb[m]
    return merged


_GROUPS: dict = {}


def _cached_new_group(ranks: list[int]) -> dist.ProcessGroup:
    """``dist.new_group(ranks)``, created once per process and default group.

    Every ``KFACPreconditioner`` asks for the same KAISA groups (reference:
    one ``new_group`` per unique rank set per preconditioner,
    ``kfac/preconditioner.py:283-295``).  On RCCL each group is a
    communicator (init time and buffers per group), so a process that builds
    several preconditioners -- the bench times K-FAC three times, a job that
    rebuilds its model -- reuses them.  Every rank builds the same sequence
    of preconditioners, so every rank hits or misses the cache together
    (``new_group`` stays a collective called in the same order)."""
    default = dist.distributed_c10d._get_default_group()
    key = (id(default), tuple(sorted(ranks)))
    pg = _GROUPS.get(key)
    if pg is None or pg not in dist.distributed_c10d._world.pg_map:
        pg = dist.new_group(ranks)
        _GROUPS[key] = pg
    return pg


class KFACPreconditioner(BaseKFACPreconditioner):
    """KFAC distributed gradient preconditioner with KAISA placement."""

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
        colocate_factors: bool = True,
        compute_method: ComputeMethod | str = ComputeMethod.EIGEN,
        compute_eigenvalue_outer_product: bool = True,
        grad_worker_fraction: DistributedStrategy | float = DistributedStrategy.COMM_OPT,
        symmetry_aware: bool = False,
        grad_scaler: torch.cuda.amp.GradScaler | Callable[[], float] | None = None,
        factor_dtype: torch.dtype | None = None,
        inv_dtype: torch.dtype = torch.float32,
        skip_layers: list[str] | None = None,
        update_factors_in_hook: bool = True,
        loglevel: int = logging.DEBUG,
        register_embeddings: bool = False,
        cost_model: str = 'auto',
    ) -> None:
        """Init KFACPreconditioner.

        Args:
            model: model to precondition (usually DDP-wrapped).
            factor_update_steps: steps between factor updates (or callable).
            inv_update_steps: steps between second-order updates (or callable).
            damping: Tikhonov damping (or callable).
            factor_decay: running-average weight (or callable).
            kl_clip: KL-clip parameter (or callable, or None to disable).
            lr: learning rate for the KL clip (or callable).
            accumulation_steps: micro-batches per optimizer step.
            allreduce_bucket_cap_mb: factor all-reduce bucket cap (decimal
                MB); 0 disables bucketing.
            assignment_strategy: ``COMPUTE`` (cost n^3) or ``MEMORY`` (n^2).
            colocate_factors: decompose A and G of a layer on one rank.
            compute_method: ``EIGEN`` or ``INVERSE``.
            compute_eigenvalue_outer_product: prediv ``1/(dG (x) dA + l)`` on
                the decomposition worker (requires ``colocate_factors``).
            grad_worker_fraction: ``DistributedStrategy`` or a fraction.
            symmetry_aware: send only upper triangles of symmetric tensors.
            grad_scaler: AMP GradScaler (or callable returning the scale).
            factor_dtype: factor storage dtype (None: see KFACBaseLayer).
            inv_dtype: dtype of eigenbases / inverses.
            skip_layers: regexes of module names / class names to skip.
            update_factors_in_hook: update factors inside the hooks.
            loglevel: logging level of registration messages.
            register_embeddings: also precondition ``nn.Embedding`` layers
                (diagonal A factor, ``layers.embedding``).  Off by default
                for parity with the reference, which ignores embeddings.
            cost_model: factor cost of the ``COMPUTE`` placement: ``'flops'``
                (the reference's n^3), ``'measured'`` (the MI355X per-size
                solver-time table, ``parallel/costmodel.py``) or ``'auto'``
                (measured for the eigen method on a CUDA model, else flops).
        """
        if allreduce_bucket_cap_mb < 0:
            raise ValueError('allreduce_bucket_cap_mb must be >= 0')
        if isinstance(compute_method, str):
            compute_method = ComputeMethod[compute_method.upper()]
        if isinstance(assignment_strategy, str):
            assignment_strategy = AssignmentStrategy[assignment_strategy.upper()]
        if (
            compute_method == ComputeMethod.EIGEN
            and compute_eigenvalue_outer_product
            and not colocate_factors
        ):
            raise ValueError(
                'colocate_factors must be True to use '
                'compute_eigenvalue_outer_product',
            )
        size = get_world_size()
        frac, strategy = resolve_grad_worker_fraction(grad_worker_fraction, size)
        if not colocate_factors and strategy is DistributedStrategy.MEM_OPT:
            warnings.warn(
                'grad_worker_frac=1/world_size (MEM_OPT) requires '
                'colocate_factors=True. Enabling colocate_factors.',
            )
            colocate_factors = True

        self.allreduce_bucket_cap_mb = allreduce_bucket_cap_mb
        self.assignment_strategy = assignment_strategy
        self.colocate_factors = colocate_factors
        self.compute_eigenvalue_outer_product = compute_eigenvalue_outer_product
        self.compute_method = compute_method
        self.distributed_strategy = strategy
        self.grad_worker_fraction = frac
        self.grad_scaler = grad_scaler
        self.factor_dtype = factor_dtype
        self.inv_dtype = inv_dtype
        self.skip_layers = [] if skip_layers is None else skip_layers
        self.symmetry_aware = symmetry_aware
        self.allreduce_method = (
            AllreduceMethod.ALLREDUCE_BUCKETED
            if allreduce_bucket_cap_mb > 0
            else AllreduceMethod.ALLREDUCE
        )
        self.tdc = TorchDistributedCommunicator(bucket_cap_mb=allreduce_bucket_cap_mb)

        layer_kwargs: dict = dict(
            allreduce_method=self.allreduce_method,
            grad_scaler=self.grad_scaler,
            factor_dtype=self.factor_dtype,
            inv_dtype=self.inv_dtype,
            symmetry_aware=self.symmetry_aware,
            tdc=self.tdc,
        )
        layer_type: type[KFACBaseLayer]
        if compute_method == ComputeMethod.EIGEN:
            layer_type = KFACEigenLayer
            layer_kwargs['prediv_eigenvalues'] = compute_eigenvalue_outer_product
        elif compute_method == ComputeMethod.INVERSE:
            layer_type = KFACInverseLayer
        else:  # pragma: no cover
            raise AssertionError(f'Unknown compute_method={compute_method}')

        kfac_layers = register_modules(
            model,
            kfac_layer_type=layer_type,
            skip_layers=self.skip_layers,
            **layer_kwargs,
        )
        self.register_embeddings = register_embeddings
        if register_embeddings:
            kfac_layers = _add_embeddings(
                model, kfac_layers, compute_method, self.skip_layers, layer_kwargs,
            )
        for name, layer in kfac_layers.values():
            logger.log(loglevel, f'Registered name="{name}": {layer!r}')

        if cost_model not in ('auto', 'flops', 'measured'):
            raise ValueError(f'unknown cost_model {cost_model!r}')
        if cost_model == 'auto':
            # the reference's n^3 placement (kfac/preconditioner.py:266-281);
            # the latency model of parallel/costmodel.py stays opt-in
            # ('measured') until its table is regenerated on the GPU with the
            # current solver tiers (profiles/solver_table_mi355x.json)
            cost_model = 'flops'
        self.cost_model = cost_model
        if assignment_strategy == AssignmentStrategy.COMPUTE and cost_model == 'measured':
            from distributed_kfac_pytorch_amd.parallel.costmodel import solver_ms as cost
        elif assignment_strategy == AssignmentStrategy.COMPUTE:
            def cost(n: int) -> float:
                return float(n) ** 3
        elif assignment_strategy == AssignmentStrategy.MEMORY:
            def cost(n: int) -> float:
                return float(n) ** 2
        else:  # pragma: no cover
            raise AssertionError(f'Unknown assignment_strategy={assignment_strategy}')
        work = {
            name: {
                'A': cost(layer.module.a_factor_shape[0]),
                'G': cost(layer.module.g_factor_shape[0]),
            }
            for name, layer in kfac_layers.values()
        }
        distributed = dist.is_available() and dist.is_initialized()
        assignment = KAISAAssignment(
            work,
            local_rank=get_rank(),
            world_size=size,
            grad_worker_fraction=frac,
            group_func=_cached_new_group if distributed else (lambda ranks: None),
            colocate_factors=colocate_factors,
        )
        logger.log(loglevel, f'KFAC layer assignments: {assignment}')

        defaults = {
            'allreduce_bucket_cap_mb': self.allreduce_bucket_cap_mb,
            'allreduce_method': self.allreduce_method,
            'assignment_strategy': self.assignment_strategy,
            'colocate_factors': self.colocate_factors,
            'compute_eigenvalue_outer_product': self.compute_eigenvalue_outer_product,
            'compute_method': self.compute_method,
            'distributed_strategy': self.distributed_strategy,
            'grad_worker_fraction': self.grad_worker_fraction,
            'grad_scaler': self.grad_scaler is not None,
            'factor_dtype': self.factor_dtype,
            'inv_dtype': self.inv_dtype,
            'skip_layers': self.skip_layers,
            'symmetry_aware': self.symmetry_aware,
            'register_embeddings': self.register_embeddings,
            'cost_model': self.cost_model,
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
