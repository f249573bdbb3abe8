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


def _params_after(frac: float, method: str) -> list:
    torch.manual_seed(7)
    model = torch.nn.parallel.DistributedDataParallel(TinyModel())
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    pre = kfac.KFACPreconditioner(model, factor_update_steps=1, inv_update_steps=2,
                                  grad_worker_fraction=frac, compute_method=method,
                                  allreduce_bucket_cap_mb=0.0005)
    g = torch.Generator().manual_seed(dist.get_rank())
    x = torch.randn(16, 10, generator=g)
    y = torch.randint(0, 10, (16,), generator=g)
    for _ in range(6):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
        opt.step()
    return [p.detach().clone() for p in model.parameters()]


def _exchange_matches_local(method: str) -> None:
    # HYBRID / MEM-OPT: receivers take the grad worker's preconditioned
    # gradient through the per-group exchange; COMM-OPT computes it on every
    # rank.  Same eigenbases (one inverse worker each), same bits.
    local = _params_after(1.0, method)
    for frac in (0.5, 1.0 / dist.get_world_size()):
        got = _params_after(frac, method)
        for a, b in zip(got, local):
            assert torch.equal(a, b), (frac, float((a - b).abs().max()))


@pytest.mark.parametrize('world,method', [(2, 'eigen'), (4, 'eigen'), (4, 'inverse')])
def test_gradient_exchange_matches_comm_opt(world, method):
    run_distributed(_exchange_matches_local, world, method)
