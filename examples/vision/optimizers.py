"""Optimizer / K-FAC / schedule factory for the vision examples
(reference ``examples/vision/optimizers.py:15-113``).

Behavioural notes vs the reference:

* The K-FAC step-interval and damping schedules are *milestone* lambdas:
  ``LambdaParamScheduler`` multiplies the current value by ``lambda(epoch)``
  on every call (reference ``kfac/scheduler.py:118-166``), so the lambda
  returns ``alpha`` exactly at a milestone epoch and 1 otherwise.  The
  reference passes cumulative factors, which compound after the first
  milestone; this gives the documented schedule.
* ``--kfac-kl-clip <= 0`` disables clipping (``kl_clip=None``).
"""
from __future__ import annotations

import argparse
from typing import Callable

import torch
import torch.optim as optim

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.utils.training import create_lr_schedule


def strategy_from_args(args: argparse.Namespace) -> kfac.enums.DistributedStrategy | float:
    if args.kfac_strategy == 'comm-opt':
        return kfac.enums.DistributedStrategy.COMM_OPT
    if args.kfac_strategy == 'mem-opt':
        return kfac.enums.DistributedStrategy.MEM_OPT
    if args.kfac_strategy == 'hybrid-opt':
        return args.kfac_grad_worker_fraction
    raise ValueError(f'Unknown K-FAC strategy: {args.kfac_strategy}')


def milestone_lambda(alpha: float, epochs: list[int] | None) -> Callable[[int], float]:
    """Per-call multiplier: ``alpha`` at each milestone epoch, else 1."""
    marks = set(epochs or [])

    def scale(epoch: int) -> float:
        return alpha if epoch in marks else 1.0

    return scale


def build_preconditioner(
    model: torch.nn.Module,
    optimizer: optim.Optimizer,
    args: argparse.Namespace,
) -> kfac.KFACPreconditioner | None:
    if args.kfac_inv_update_steps <= 0:
        return None
    return kfac.KFACPreconditioner(
        model,
        factor_update_steps=args.kfac_factor_update_steps,
        inv_update_steps=args.kfac_inv_update_steps,
        damping=args.kfac_damping,
        factor_decay=args.kfac_factor_decay,
        kl_clip=args.kfac_kl_clip if args.kfac_kl_clip > 0 else None,
        lr=lambda step: optimizer.param_groups[0]['lr'],
        accumulation_steps=getattr(args, 'batches_per_allreduce', 1),
        allreduce_bucket_cap_mb=args.kfac_bucket_cap_mb,
        colocate_factors=args.kfac_colocate_factors,
        compute_method=(
            kfac.enums.ComputeMethod.INVERSE if args.kfac_inv_method
            else kfac.enums.ComputeMethod.EIGEN
        ),
        grad_worker_fraction=strategy_from_args(args),
        symmetry_aware=args.kfac_symmetry_aware,
        grad_scaler=getattr(args, 'grad_scaler', None),
        skip_layers=args.kfac_skip_layers,
        register_embeddings=getattr(args, 'kfac_register_embeddings', False),
    )


def get_optimizer(
    model: torch.nn.Module,
    args: argparse.Namespace,
) -> tuple[
    optim.Optimizer,
    kfac.KFACPreconditioner | None,
    tuple[optim.lr_scheduler.LambdaLR, kfac.scheduler.LambdaParamScheduler | None],
]:
    """SGD(momentum, wd) + warmup/step LR + optional K-FAC and its scheduler."""
    optimizer = optim.SGD(
        model.parameters(),
        lr=args.base_lr,
        momentum=args.momentum,
        weight_decay=args.weight_decay,
    )
    lrs = create_lr_schedule(args.world_size, args.warmup_epochs, args.lr_decay)
    lr_scheduler = optim.lr_scheduler.LambdaLR(optimizer, lrs)
    preconditioner = build_preconditioner(model, optimizer, args)
    kfac_scheduler = None
    if preconditioner is not None:
        steps = milestone_lambda(args.kfac_update_steps_alpha, args.kfac_update_steps_decay)
        kfac_scheduler = kfac.scheduler.LambdaParamScheduler(
            preconditioner,
            damping_lambda=milestone_lambda(args.kfac_damping_alpha, args.kfac_damping_decay),
            factor_update_steps_lambda=steps,
            inv_update_steps_lambda=steps,
        )
    return optimizer, preconditioner, (lr_scheduler, kfac_scheduler)
