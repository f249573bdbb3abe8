"""Train / evaluate loops for the language-model example (reference
``examples/language/engine.py:15-117``): forward, token cross-entropy,
``clip_grad_norm_(0.5)`` *before* ``preconditioner.step()`` (as the
reference does), then SGD.  Runs under bf16 autocast on the GPU; the model
is batch-first with a causal mask sized by the sequence length (the
reference builds it from the batch dimension).
"""
from __future__ import annotations

import contextlib
import math
from typing import Any

import torch
from tqdm import tqdm

from distributed_kfac_pytorch_amd.utils.training import Metric


def _autocast(device: torch.device, amp_dtype: torch.dtype | None) -> Any:
    if amp_dtype is None:
        return contextlib.nullcontext()
    return torch.autocast(device.type, dtype=amp_dtype)


def train(model: torch.nn.Module, *, criterion: torch.nn.Module,
          optimizer: torch.optim.Optimizer, preconditioner: Any,
          dataloader: torch.utils.data.DataLoader, epoch: int, epochs: int,
          device: torch.device, amp_dtype: torch.dtype | None = None,
          clip: float = 0.5, verbose: bool = True, max_steps: int | None = None) -> float:
    model.train()
    train_loss = Metric('train_loss', device)
    total = len(dataloader) if not max_steps else min(len(dataloader), max_steps)
    with tqdm(total=total, bar_format='{l_bar}{bar:8}{r_bar}',
              desc=f'Epoch {epoch:2d}/{epochs:2d}', disable=not verbose) as t:
        for i, (data, target) in enumerate(dataloader):
            data = data.to(device, non_blocking=True)
            target = target.to(device, non_blocking=True).reshape(-1)
            optimizer.zero_grad(set_to_none=False)
            with _autocast(device, amp_dtype):
                output = model(data)
            loss = criterion(output.float().reshape(-1, output.shape[-1]), target)
            loss.backward()
            if clip > 0:
                torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
            if preconditioner is not None:
                preconditioner.step()
            optimizer.step()
            train_loss.update(loss.detach())
            t.update(1)
            if (i + 1) % 20 == 0 or i + 1 == total:
                avg = train_loss.avg
                t.set_postfix_str(f'loss: {avg:.2f}, ppl: {math.exp(min(avg, 50)):.2f}')
            if max_steps and i + 1 >= max_steps:
                break
    return train_loss.avg


def evaluate(model: torch.nn.Module, *, criterion: torch.nn.Module,
             dataloader: torch.utils.data.DataLoader, device: torch.device,
             amp_dtype: torch.dtype | None = None, prefix: str = 'Validation',
             verbose: bool = True, max_steps: int | None = None) -> float:
    model.eval()
    loss_m = Metric('eval_loss', device)
    with torch.no_grad():
        for i, (data, target) in enumerate(dataloader):
            data = data.to(device, non_blocking=True)
            target = target.to(device, non_blocking=True).reshape(-1)
            with _autocast(device, amp_dtype):
                output = model(data)
            loss_m.update(criterion(output.float().reshape(-1, output.shape[-1]), target))
            if max_steps and i + 1 >= max_steps:
                break
    avg = loss_m.avg
    if verbose:
        print(f'{prefix} loss: {avg:.4f}, ppl: {math.exp(min(avg, 50)):.2f}', flush=True)
    return avg
