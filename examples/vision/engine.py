"""Train / evaluate loops for the vision examples
(reference ``examples/vision/engine.py:15-155``).

Per optimizer step (``batches_per_allreduce`` micro-batches):
forward under autocast (bf16 by default on MI355X; fp16 + GradScaler with
``--fp16``) -> backward (DDP ``no_sync`` on all but the last micro-batch)
-> ``scaler.unscale_`` -> ``preconditioner.step()`` -> ``optimizer.step()``.

MI355X-specific choices: inputs are moved with ``non_blocking`` copies from
pinned memory and converted to channels_last on the device; loss/accuracy
are accumulated on the device and only reduced across ranks when the
progress bar is refreshed (every ``log_interval`` steps) instead of a
synchronous all-reduce every step (reference ``examples/utils.py:65-88``).
"""
from __future__ import annotations

import argparse
import contextlib
import math
from typing import Any

import torch
from tqdm import tqdm

from distributed_kfac_pytorch_amd.utils.training import accuracy
from distributed_kfac_pytorch_amd.utils.training import Metric


def _autocast(args: argparse.Namespace) -> Any:
    if getattr(args, 'amp_dtype', None) is None:
        return contextlib.nullcontext()
    return torch.autocast(args.device.type, dtype=args.amp_dtype)


def _to_device(data: torch.Tensor, target: torch.Tensor, args: argparse.Namespace
               ) -> tuple[torch.Tensor, torch.Tensor]:
    data = data.to(args.device, non_blocking=True)
    target = target.to(args.device, non_blocking=True)
    if getattr(args, 'channels_last', False) and data.dim() == 4:
        data = data.contiguous(memory_format=torch.channels_last)
    return data, target


class _GraphedSteps:
    """Whole-step HIP-graph runner for ``train`` (``--graphs``): static input
    buffers, the loss and accuracy produced inside the captured step
    (``distributed_kfac_pytorch_amd.graphs.GraphedTrainStep``; graph-safe
    strided convolutions, one step stream).  Batches of another shape (the
    last partial batch) take the eager path."""

    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer,
                 preconditioner: Any, loss_func: torch.nn.Module,
                 data: torch.Tensor, target: torch.Tensor, args: argparse.Namespace) -> None:
        from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep

        self.x = torch.empty_like(data)
        self.y = torch.empty_like(target)
        self.acc = torch.zeros((), device=data.device)
        # captured with the autocast weight cache off (it cannot be replayed)
        amp = getattr(args, 'amp_dtype', None)

        def fb() -> torch.Tensor:
            with torch.autocast(data.device.type, dtype=amp or torch.float32,
                                enabled=amp is not None, cache_enabled=False):
                output = model(self.x)
                loss = loss_func(output, self.y)
            with torch.no_grad():
                self.acc.copy_(accuracy(output, self.y))
            loss.backward()
            return loss

        # under bf16 autocast every 1x1 conv runs as GEMMs in the graphs
        # (MIOpen's tuned bf16 backward-weights solvers read outside them)
        self.runner = GraphedTrainStep(fb, optimizer, preconditioner, model=model,
                                       conv_mode='gemm' if amp is not None else None)

    def fits(self, data: torch.Tensor, target: torch.Tensor) -> bool:
        return data.shape == self.x.shape and data.stride() == self.x.stride() and \
            target.shape == self.y.shape

    def __call__(self, data: torch.Tensor, target: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        self.x.copy_(data)
        self.y.copy_(target)
        loss = self.runner()
        return loss.float(), self.acc


def _graphs_usable(args: argparse.Namespace) -> bool:
    return (bool(getattr(args, 'graphs', False)) and args.device.type == 'cuda'
            and max(1, args.batches_per_allreduce) == 1
            and getattr(args, 'grad_scaler', None) is None)


def train(
    epoch: int,
    model: torch.nn.Module,
    optimizer: torch.optim.Optimizer,
    preconditioner: Any,
    loss_func: torch.nn.Module,
    train_sampler: Any,
    train_loader: torch.utils.data.DataLoader,
    args: argparse.Namespace,
) -> dict[str, float]:
    model.train()
    if train_sampler is not None and hasattr(train_sampler, 'set_epoch'):
        train_sampler.set_epoch(epoch)
    train_loss = Metric('train_loss', args.device)
    train_accuracy = Metric('train_accuracy', args.device)
    scaler = getattr(args, 'grad_scaler', None)
    accum = max(1, args.batches_per_allreduce)
    log_interval = max(1, getattr(args, 'log_interval', 10))
    max_steps = getattr(args, 'max_steps_per_epoch', None)
    n_batches = len(train_loader)
    total = math.ceil(n_batches / accum)
    if max_steps:
        total = min(total, max_steps)
    step_loss = torch.zeros((), device=args.device)
    step_acc = torch.zeros((), device=args.device)
    mini_step = 0
    steps = 0
    with tqdm(total=total, bar_format='{l_bar}{bar:10}{r_bar}',
              desc=f'Epoch {epoch:3d}/{args.epochs:3d}', disable=not args.verbose) as t:
        for batch_idx, (data, target) in enumerate(train_loader):
            data, target = _to_device(data, target, args)
            if _graphs_usable(args):
                graphed = getattr(args, '_graphed_steps', None)
                if graphed is None:
                    graphed = _GraphedSteps(model, optimizer, preconditioner, loss_func,
                                            data, target, args)
                    args._graphed_steps = graphed
                if graphed.fits(data, target):
                    loss_v, acc_v = graphed(data, target)
                    train_loss.update(loss_v)
                    train_accuracy.update(acc_v)
                    steps += 1
                    t.update(1)
                    if steps % log_interval == 0 or steps == total:
                        t.set_postfix_str(
                            f'loss: {train_loss.avg:.4f}, acc: {100 * train_accuracy.avg:.2f}%, '
                            f'lr: {optimizer.param_groups[0]["lr"]:.4f}',
                        )
                    if max_steps and steps >= max_steps:
                        break
                    continue
            mini_step += 1
            last = mini_step % accum == 0 or batch_idx + 1 == n_batches
            sync_ctx = (
                model.no_sync() if (not last and hasattr(model, 'no_sync'))
                else contextlib.nullcontext()
            )
            with sync_ctx:
                with _autocast(args):
                    output = model(data)
                    loss = loss_func(output, target)
                with torch.no_grad():
                    step_loss += loss.detach().float()
                    step_acc += accuracy(output, target)
                loss = loss / accum
                if scaler is not None:
                    scaler.scale(loss).backward()
                else:
                    loss.backward()
            if not last:
                continue
            if preconditioner is not None:
                if scaler is not None:
                    scaler.unscale_(optimizer)
                preconditioner.step()
            if scaler is not None:
                scaler.step(optimizer)
                scaler.update()
            else:
                optimizer.step()
            optimizer.zero_grad(set_to_none=False)
            train_loss.update(step_loss / mini_step)
            train_accuracy.update(step_acc / mini_step)
            step_loss.zero_()
            step_acc.zero_()
            mini_step = 0
            steps += 1
            t.update(1)
            if steps % log_interval == 0 or steps == total:
                t.set_postfix_str(
                    f'loss: {train_loss.avg:.4f}, acc: {100 * train_accuracy.avg:.2f}%, '
                    f'lr: {optimizer.param_groups[0]["lr"]:.4f}',
                )
            if max_steps and steps >= max_steps:
                break
    out = {'train/loss': train_loss.avg, 'train/accuracy': train_accuracy.avg,
           'train/lr': optimizer.param_groups[0]['lr']}
    graphed = getattr(args, '_graphed_steps', None)
    if graphed is not None:
        out['train/graph_replays'] = float(graphed.runner.replays)
    writer = getattr(args, 'log_writer', None)
    if writer is not None:
        for k, v in out.items():
            writer.add_scalar(k, v, epoch)
    return out


def test(
    epoch: int,
    model: torch.nn.Module,
    loss_func: torch.nn.Module,
    val_loader: torch.utils.data.DataLoader,
    args: argparse.Namespace,
) -> dict[str, float]:
    model.eval()
    val_loss = Metric('val_loss', args.device)
    val_accuracy = Metric('val_accuracy', args.device)
    max_steps = getattr(args, 'max_steps_per_epoch', None)
    with torch.no_grad(), tqdm(total=len(val_loader), bar_format='{l_bar}{bar:10}|{postfix}',
                               desc='             ', disable=not args.verbose) as t:
        for i, (data, target) in enumerate(val_loader):
            data, target = _to_device(data, target, args)
            with _autocast(args):
                output = model(data)
            val_loss.update(loss_func(output.float(), target))
            val_accuracy.update(accuracy(output, target))
            t.update(1)
            if max_steps and i + 1 >= max_steps:
                break
        t.set_postfix_str(
            f'val_loss: {val_loss.avg:.4f}, val_acc: {100 * val_accuracy.avg:.2f}%',
            refresh=False,
        )
    out = {'val/loss': val_loss.avg, 'val/accuracy': val_accuracy.avg}
    writer = getattr(args, 'log_writer', None)
    if writer is not None:
        for k, v in out.items():
            writer.add_scalar(k, v, epoch)
    return out
