"""Multi-rank training end to end (reference tests/training_test.py): a
TinyModel under DDP + K-FAC must reduce its loss on a fixed batch, for COMM-OPT
and HYBRID-OPT on 1, 2 and 4 gloo ranks, and all ranks must stay in sync."""
from __future__ import annotations

import pytest
import torch
import torch.distributed as dist

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models.tiny import TinyModel
from tests.harness import run_distributed


def _train(grad_worker_fraction: float, method: str, symmetry_aware: bool) -> None:
    torch.manual_seed(42)
    model = TinyModel()
    distributed = dist.is_initialized()
    if distributed:
        model = torch.nn.parallel.DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    pre = kfac.KFACPreconditioner(
        model,
        factor_update_steps=1,
        inv_update_steps=2,
        grad_worker_fraction=grad_worker_fraction,
        compute_method=method,
        symmetry_aware=symmetry_aware,
        allreduce_bucket_cap_mb=0.001,
    )
    rank = dist.get_rank() if distributed else 0
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(32, 10, generator=g)
    y = torch.randint(0, 10, (32,), generator=g)
    losses = []
    for _ in range(20):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        pre.step()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses
    if distributed:
        # parameters identical on every rank
        for p in model.parameters():
            q = p.detach().clone()
            dist.broadcast(q, src=0)
            assert torch.allclose(q, p.detach(), atol=1e-6)
    # checkpoint keys carry the DDP prefix, like the reference
    names = list(pre.state_dict()['layers'])
    prefix = 'module.' if distributed else ''
    assert names == [f'{prefix}linear1', f'{prefix}linear2']


def test_training_single_process():
    _train(1.0, 'eigen', False)


@pytest.mark.parametrize(
    'world,frac,method,sym',
    [
        (1, 0.0, 'eigen', False),
        (2, 0.5, 'eigen', False),
        (2, 0.5, 'inverse', True),
        (4, 0.5, 'eigen', True),
        (4, 0.25, 'inverse', False),
        (4, 1.0, 'eigen', False),
    ],
)
def test_training_distributed(world, frac, method, sym):
    run_distributed(_train, world, frac, method, sym)
