"""Latency-aware KAISA cost model (parallel/costmodel.py) on CPU."""
from __future__ import annotations

import torch

from distributed_kfac_pytorch_amd.parallel import costmodel
from distributed_kfac_pytorch_amd.preconditioner import KFACPreconditioner


def test_solver_ms_interpolates_and_is_monotone() -> None:
    t = costmodel.SOLVER_MS
    for n, ms in t.items():
        assert costmodel.solver_ms(n) == ms
    sizes = list(range(1, 6000, 37))
    vals = [costmodel.solver_ms(n) for n in sizes]
    assert all(b >= a for a, b in zip(vals, vals[1:]))
    # strictly between neighbouring table points
    keys = sorted(t)
    for lo, hi in zip(keys, keys[1:]):
        if hi - lo > 1:
            mid = (lo + hi) // 2
            assert t[lo] <= costmodel.solver_ms(mid) <= t[hi]


def test_latency_model_is_not_cubic() -> None:
    # the native chain is latency bound: a 1152 factor costs far more than
    # (1152/4608)^3 of a 4608 one
    r = costmodel.solver_ms(1152) / costmodel.solver_ms(4608)
    assert r > 4 * (1152 / 4608) ** 3


def test_model_factor_sizes() -> None:
    rn = costmodel.model_factor_sizes('resnet50')
    assert len(rn) == 54
    dims = sorted({d for _, a, g in rn for d in (a, g)})
    assert max(dims) == 4608 and 147 in dims and 2049 in dims and 1000 in dims
    neox = costmodel.model_factor_sizes('gpt_neox_125m')
    assert len(neox) == 48 and max(g for _, _, g in neox) == 3072


def test_plan_balances_predicted_ms() -> None:
    sizes = costmodel.model_factor_sizes('resnet50')
    total = sum(costmodel.solver_ms(a) + costmodel.solver_ms(g) for _, a, g in sizes)
    one = costmodel.plan(sizes, 1)
    assert abs(one['max_ms'] - total) < 1e-6 * total
    for world in (2, 4, 8):
        m = costmodel.plan(sizes, world, cost='measured')
        f = costmodel.plan(sizes, world, cost='flops')
        assert sum(len(p) for p in m['factors_per_rank']) == 2 * len(sizes)
        assert abs(sum(m['predicted_ms']) - total) < 1e-6 * total
        # balancing predicted ms is never worse than balancing flops
        assert m['max_ms'] <= f['max_ms'] * 1.0001
        # and within LPT's bound of the ideal split
        biggest = max(costmodel.solver_ms(max(a, g)) * 2 for _, a, g in sizes)
        assert m['max_ms'] <= total / world + biggest


def test_preconditioner_cost_model_selection() -> None:
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    p = KFACPreconditioner(model)
    assert p.cost_model == 'flops'  # CPU model: the reference's n^3
    p = KFACPreconditioner(model, cost_model='measured')
    assert p.cost_model == 'measured'
    assert 'cost_model' in repr(p)
    try:
        KFACPreconditioner(model, cost_model='bogus')
    except ValueError:
        pass
    else:  # pragma: no cover
        raise AssertionError('bogus cost model accepted')
