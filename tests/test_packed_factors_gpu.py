"""Packed-factor all-reduce on the GPU: two gloo ranks sharing cuda:0.

The factor-update SYRK writes the packed triangle straight into the
persistent all-reduce buffer (csrc/syrk.hip packed epilogue); gradients and
factors after several factor / second-order updates must match the dense
pack / all-reduce / unpack path.  Spawned ranks (the pytest process has
already initialised HIP, so forking is not an option).
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


def _rank_main(rank: int, world: int, port: int, method: str) -> None:
    import torch.distributed as dist

    import distributed_kfac_pytorch_amd as kfac
    from tests.test_packed_factors import _Net

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    dev = torch.device('cuda', 0)
    # the two runs are compared element-wise: MIOpen's default backward-
    # weights kernels accumulate with atomics (run-to-run noise that the
    # INVERSE preconditioner amplifies past the tolerance on some boxes)
    torch.backends.cudnn.deterministic = True

    def run(mode: str) -> tuple:
        os.environ['KFAC_PACKED_FACTORS'] = mode
        torch.manual_seed(0)
        model = torch.nn.parallel.DistributedDataParallel(_Net().to(dev))
        opt = torch.optim.SGD(model.parameters(), lr=0.05)
        pre = kfac.KFACPreconditioner(model, factor_update_steps=2, inv_update_steps=4,
                                      compute_method=method, allreduce_bucket_cap_mb=0.01)
        g = torch.Generator().manual_seed(rank)
        grads = []
        for _ in range(9):
            x = torch.randn(8, 3, 8, 8, generator=g).to(dev)
            y = torch.randint(0, 10, (8,), generator=g).to(dev)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(model(x), y).backward()
            pre.step()
            grads.append([p.grad.clone() for p in model.parameters()])
            opt.step()
        homes = sum(1 for _, l in pre._layers.values() for h in l._homes.values() if h)
        fac = {n: (l.a_factor.clone(), l.g_factor.clone()) for n, l in pre._layers.values()}
        return grads, fac, homes

    dense = run('0')
    packed = run('auto')  # GPU: packed by default
    assert dense[2] == 0 and packed[2] == 8, (dense[2], packed[2])
    for gd, gp in zip(dense[0], packed[0]):
        for a, b in zip(gd, gp):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
    for name, (ad, gd) in dense[1].items():
        torch.testing.assert_close(ad, packed[1][name][0], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(gd, packed[1][name][1], rtol=1e-5, atol=1e-7)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
def test_packed_factor_allreduce_two_ranks_one_gpu(method):
    mp.spawn(_rank_main, args=(2, _port(), method), nprocs=2, join=True)
