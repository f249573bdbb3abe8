"""Lazy join of the factor side stream (single process).

``step()`` of a factor-update step waits only for the A-factor SYRKs and
leaves the G-factor SYRKs of the backward hooks running on the side stream
(``BaseKFACPreconditioner._lazy_factor_join``); every reader of the factors
joins first.  The same training -- inline factor updates, side stream with a
full join, side stream with the lazy join -- must give bit-identical
gradients, factors and eigenbases, while the caller overwrites its input
batch in place right after each step (the hazard the A-side wait covers).
"""
from __future__ import annotations

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(stream: str, join: str, segment: str = '8') -> tuple:
    import distributed_kfac_pytorch_amd as kfac
    from tests.test_packed_factors import _Net

    old = {k: os.environ.get(k) for k in ('KFAC_FACTOR_STREAM', 'KFAC_FACTOR_JOIN',
                                         'KFAC_FACTOR_SEGMENT')}
    os.environ['KFAC_FACTOR_STREAM'] = stream
    os.environ['KFAC_FACTOR_JOIN'] = join
    os.environ['KFAC_FACTOR_SEGMENT'] = segment
    try:
        dev = torch.device('cuda', 0)
        torch.manual_seed(0)
        model = _Net().to(dev)
        opt = torch.optim.SGD(model.parameters(), lr=0.05)
        pre = kfac.KFACPreconditioner(model, factor_update_steps=2, inv_update_steps=4)
        g = torch.Generator().manual_seed(3)
        x = torch.empty(8, 3, 8, 8, device=dev)
        y = torch.empty(8, dtype=torch.long, device=dev)
        pending, grads = 0, []
        for _ in range(11):
            x.copy_(torch.randn(8, 3, 8, 8, generator=g))
            y.copy_(torch.randint(0, 10, (8,), generator=g))
            opt.zero_grad()
            torch.nn.functional.cross_entropy(model(x), y).backward()
            pre.step()
            pending += len(pre._factor_forked)
            # the next batch lands in the same buffer at once
            x.copy_(torch.randn(8, 3, 8, 8, generator=g))
            grads.append([p.grad.clone() for p in model.parameters()])
            opt.step()
        pre.sync_factors()
        fac = {n: (l.a_factor.clone(), l.g_factor.clone(), l.qa.clone(), l.qg.clone())
               for n, l in pre._layers.values()}
        return grads, fac, pending
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize('segment', ['1', '2', '8'])
def test_lazy_factor_join_matches_inline(segment: str) -> None:
    """... for every side-stream segment size (hook work launched one
    layer at a time, in pairs, or a whole pass at once)."""
    torch.backends.cudnn.deterministic = True
    inline = _run('0', 'lazy')
    full = _run('1', 'full', segment)
    lazy = _run('1', 'lazy', segment)
    assert inline[2] == 0 and full[2] == 0
    assert lazy[2] > 0, 'no factor work was left pending by step()'
    for other in (full, lazy):
        for gi, go in zip(inline[0], other[0]):
            for a, b in zip(gi, go):
                assert torch.equal(a, b)
        for name, ts in inline[1].items():
            for a, b in zip(ts, other[1][name]):
                assert torch.equal(a, b), name
