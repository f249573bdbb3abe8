"""Factor updates on the side stream vs inline, two ranks on one GPU.

On RCCL process groups the forward / backward hooks issue each factor's
SYRK + EMA + all-reduce on a side HIP stream that overlaps the rest of the
pass (``base_preconditioner.BaseKFACPreconditioner._on_factor_stream``; the
reference issues them inline from its hooks,
``kfac/base_preconditioner.py:435-477``).  gloo turns the side stream off by
default, so ``KFAC_FACTOR_STREAM=1`` forces it here: two gloo ranks sharing
cuda:0 run the same training twice -- inline, then on the side stream -- and
every factor, eigenbasis and gradient must match to the bit.
"""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return int(s.getsockname()[1])


def _rank_main(rank: int, world: int, port: int) -> None:
    import torch.distributed as dist

    import distributed_kfac_pytorch_amd as kfac
    from tests.test_packed_factors import _Net

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.deterministic = True

    def run(mode: str) -> tuple:
        os.environ['KFAC_FACTOR_STREAM'] = mode
        torch.manual_seed(0)
        model = torch.nn.parallel.DistributedDataParallel(_Net().to(dev))
        opt = torch.optim.SGD(model.parameters(), lr=0.05)
        pre = kfac.KFACPreconditioner(model, factor_update_steps=2, inv_update_steps=4,
                                      allreduce_bucket_cap_mb=0.01)
        g = torch.Generator().manual_seed(rank)
        grads, used = [], 0
        for _ in range(9):
            x = torch.randn(8, 3, 8, 8, generator=g).to(dev)
            y = torch.randint(0, 10, (8,), generator=g).to(dev)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(model(x), y).backward()
            used += len(pre._factor_forked)
            pre.step()
            grads.append([p.grad.clone() for p in model.parameters()])
            opt.step()
        fac = {n: (l.a_factor.clone(), l.g_factor.clone(), l.qa.clone(), l.qg.clone())
               for n, l in pre._layers.values()}
        return grads, fac, used

    inline = run('0')
    side = run('1')
    assert inline[2] == 0 and side[2] > 0, (inline[2], side[2])
    for gi, gs in zip(inline[0], side[0]):
        for a, b in zip(gi, gs):
            assert torch.equal(a, b)
    for name, ts in inline[1].items():
        for a, b in zip(ts, side[1][name]):
            assert torch.equal(a, b), name
    dist.barrier()
    dist.destroy_process_group()


def test_factor_side_stream_matches_inline_two_ranks():
    mp.spawn(_rank_main, args=(2, _port()), nprocs=2, join=True)
