"""Latency-aware cost model for KAISA's second-order work placement.

The reference balances the per-rank eigendecomposition work on ``n^3`` of
each factor dimension (``kfac/preconditioner.py:266-281``).  On MI355X the
native eigensolver (csrc/sytrd.hip one-stage Householder chain, csrc/tridiag.hip
divide and conquer, blocked back-transform) is not flop-bound: every factor
pays a per-column chain of dependent launches (about n kernel pairs), so a
1152 factor costs far more than (1152/4608)^3 of a 4608 one, and a rank that
owns one large factor still waits for its whole chain.  ``n^3`` mis-balances
exactly the N = 8 case the refresh is amortised over.

``solver_ms(n)`` interpolates a MEASURED single-factor refresh time table
(log-log between measured sizes; ``tools/solver_table.py`` regenerates it and
``profiles/solver_table_mi355x.json`` holds the run the defaults come from).
``KFACPreconditioner(assignment_strategy='compute')`` uses it as the factor
cost on CUDA models with the eigen method (``cost_model='auto'``), so the
LPT placement (``parallel/assignment.py``, unchanged) balances predicted
milliseconds instead of flops.  ``plan()`` prints the predicted per-rank
refresh for a model at any world size without a GPU.
"""
from __future__ import annotations

import bisect
import math
from typing import Any

# single-factor refresh on one MI355X, ms (tools/solver_table.py).  Sizes
# <= 128 run in the one-workgroup LDS Jacobi tier (all together in one
# launch); above that the native chain.
SOLVER_MS: dict[int, float] = {
    64: 0.3, 128: 0.5,
    129: 4.0, 256: 7.0, 512: 13.0, 768: 19.0, 1024: 25.0, 1536: 37.0,
    2048: 50.0, 2304: 56.0, 3072: 80.0, 4096: 110.0, 4608: 125.0,
}


def solver_ms(n: int, table: dict[int, float] | None = None) -> float:
    """Predicted refresh milliseconds of one ``n x n`` factor."""
    t = table or SOLVER_MS
    keys = sorted(t)
    if n <= keys[0]:
        return t[keys[0]] * max(n, 1) / keys[0]
    if n >= keys[-1]:
        # beyond the table the bandwidth term dominates: n^3 growth
        return t[keys[-1]] * (n / keys[-1]) ** 3
    i = bisect.bisect_left(keys, n)
    if keys[i] == n:
        return t[n]
    lo, hi = keys[i - 1], keys[i]
    f = (math.log(n) - math.log(lo)) / (math.log(hi) - math.log(lo))
    return math.exp(math.log(t[lo]) + f * (math.log(t[hi]) - math.log(t[lo])))


def flops_cost(n: int) -> float:
    """The reference's COMPUTE cost (``kfac/preconditioner.py:266-281``)."""
    return float(n) ** 3


def model_factor_sizes(name: str) -> list[tuple[str, int, int]]:
    """``[(layer, A dim, G dim)]`` of a benchmark model, without building it
    on a device (ResNet-50 from the in-tree definition on the meta device;
    GPT-NeoX-125M from its architecture: hidden 768, 12 layers)."""
    if name == 'resnet50':
        import torch

        from distributed_kfac_pytorch_amd.models.resnet import resnet50

        with torch.device('meta'):
            model = resnet50()
        out = []
        for lname, m in model.named_modules():
            if isinstance(m, torch.nn.Conv2d):
                kh, kw = m.kernel_size
                a = m.in_channels * kh * kw + int(m.bias is not None)
                out.append((lname, a, m.out_channels))
            elif isinstance(m, torch.nn.Linear):
                out.append((lname, m.in_features + int(m.bias is not None), m.out_features))
        return out
    if name == 'gpt_neox_125m':
        h, layers = 768, 12
        out = []
        for i in range(layers):
            out += [(f'layers.{i}.attention.query_key_value', h + 1, 3 * h),
                    (f'layers.{i}.attention.dense', h + 1, h),
                    (f'layers.{i}.mlp.dense_h_to_4h', h + 1, 4 * h),
                    (f'layers.{i}.mlp.dense_4h_to_h', 4 * h + 1, h)]
        return out
    raise ValueError(f'unknown model {name!r}')


def plan(sizes: list[tuple[str, int, int]], world: int, grad_worker_fraction: float = 0.5,
         cost: str = 'measured', colocate_factors: bool = True) -> dict[str, Any]:
    """KAISA placement of ``sizes`` on ``world`` ranks (no process groups)
    and each rank's predicted refresh milliseconds."""
    from distributed_kfac_pytorch_amd.parallel.assignment import KAISAAssignment

    fn = solver_ms if cost == 'measured' else flops_cost
    work = {name: {'A': fn(a), 'G': fn(g)} for name, a, g in sizes}
    frac = grad_worker_fraction if world > 1 else 1.0
    asg = KAISAAssignment(work, local_rank=0, world_size=world,
                          grad_worker_fraction=max(frac, 1.0 / world),
                          group_func=lambda ranks: None,
                          colocate_factors=colocate_factors)
    per: list[list[int]] = [[] for _ in range(world)]
    dims = {name: {'A': a, 'G': g} for name, a, g in sizes}
    for name in asg.get_layers():
        for f in asg.get_factors(name):
            per[asg.inv_worker(name, f)].append(dims[name][f])
    pred = [sum(solver_ms(n) for n in ns) for ns in per]
    return {'world': world, 'cost': cost, 'factors_per_rank': per,
            'predicted_ms': pred, 'max_ms': max(pred) if pred else 0.0}
