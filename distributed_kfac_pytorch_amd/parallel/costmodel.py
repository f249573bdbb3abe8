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
import json
import math
import os
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


# ---------------------------------------------------------------------------
# Refresh-time model of a whole factor SET (what one rank decomposes per
# refresh), mirroring ops.linalg.eigh_many's schedule instead of summing
# single factors:
#
# * n <= 128: one LDS Jacobi launch per size bucket, on a side lane
#   (overlaps the chains: only its own time when nothing else runs);
# * two-stage buckets (ops.linalg.twostage_sizes): per bucket
#   ts_a * count * n^3 / 1e9 + ts_b * n;
# * the rest: one-stage Householder chains, split at KFAC_SYTRD_SPLIT.  A
#   chain advances all its members one column per launch pair, so it costs
#   L per column of its LARGEST member plus the bytes its symv steps stream
#   (4 * sum over members and columns of the trailing square (n - k - 1)^2)
#   at bandwidth BW.  Each symv launch is sized to fill the chip, so
#   concurrent chains time-share it: their column latencies ADD, and all
#   chains' bytes share one BW;
# * the tail of the largest bucket (divide and conquer + blocked
#   back-transform), tail_a * count * n^2 / 1e6 + tail_b * count * n^3 / 1e9,
#   is exposed after the chains (smaller buckets' tails overlap them).
#
# T = sum_chains L * N_c + bytes / BW + tail(largest) (+ two-stage buckets,
# + Jacobi when it is all there is).  Parameters are fitted to measured
# refreshes by tools/fit_costmodel.py and stored with the measurements in
# profiles/solver_table_mi355x.json ("fit"); the defaults below are that fit.
# ---------------------------------------------------------------------------

REFRESH_PARAMS: dict[str, float] = {
    'L_us': 13.9, 'bw_tbs': 5.9, 'tail_a': 0.25, 'tail_b': 0.06,
    'jacobi_ms': 1.3, 'ts_a': 1.0, 'ts_b': 0.02,
}

_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      'profiles', 'solver_table_mi355x.json')


def load_params(path: str | None = None) -> dict[str, float]:
    """The fitted refresh-model parameters (``fit`` of the measured table),
    or ``REFRESH_PARAMS`` when the table is absent."""
    try:
        with open(path or _TABLE) as f:
            fit = json.load(f).get('fit')
        if fit:
            return {**REFRESH_PARAMS, **{k: float(v) for k, v in fit.items() if k in REFRESH_PARAMS}}
    except (OSError, ValueError):
        pass
    return dict(REFRESH_PARAMS)


def _split_cuts() -> list[int]:
    return sorted((int(c) for c in os.environ.get('KFAC_SYTRD_SPLIT', '4000,1000').split(',')
                   if c), reverse=True)


def refresh_terms(sizes: list[int], params: dict[str, float] | None = None) -> dict[str, float]:
    """Per-term predicted milliseconds of one eigen refresh of ``sizes``
    (see the model above)."""
    from distributed_kfac_pytorch_amd.ops.linalg import JACOBI_MAX_N
    from distributed_kfac_pytorch_amd.ops.linalg import twostage_sizes

    p = params or load_params()
    counts: dict[int, int] = {}
    for n in sizes:
        counts[int(n)] = counts.get(int(n), 0) + 1
    ts = twostage_sizes({n: c for n, c in counts.items() if n > JACOBI_MAX_N})
    jac = [n for n in counts if n <= JACOBI_MAX_N]
    chain_sizes = {n: c for n, c in counts.items() if n > JACOBI_MAX_N and n not in ts}
    groups: list[dict[int, int]] = []
    left = dict(chain_sizes)
    for cut in _split_cuts():
        groups.append({n: c for n, c in left.items() if n >= cut})
        left = {n: c for n, c in left.items() if n < cut}
    groups.append(left)
    groups = [g for g in groups if g]
    lat = sum(p['L_us'] * 1e-3 * (max(g) - 1) for g in groups)
    byts = 0.0
    for n, c in chain_sizes.items():
        m = n - 1  # trailing squares (n-1)^2 ... 1^2
        byts += 4.0 * c * m * (m + 1) * (2 * m + 1) / 6.0
    bw = byts / (p['bw_tbs'] * 1e12) * 1e3
    tail = 0.0
    if chain_sizes:
        n = max(chain_sizes)
        c = chain_sizes[n]
        tail = p['tail_a'] * c * n * n / 1e6 + p['tail_b'] * c * n ** 3 / 1e9
    two = sum(p['ts_a'] * counts[n] * n ** 3 / 1e9 + p['ts_b'] * n for n in ts)
    jacobi = p['jacobi_ms'] * len(jac)
    return {'latency': lat, 'bandwidth': bw, 'tail': tail, 'twostage': two, 'jacobi': jacobi}


def refresh_ms(sizes: list[int], params: dict[str, float] | None = None) -> float:
    """Predicted milliseconds of one eigen refresh of the factor set
    ``sizes`` on one MI355X (ops.linalg.eigh_many)."""
    t = refresh_terms(sizes, params)
    main = t['latency'] + t['bandwidth'] + t['tail'] + t['twostage']
    return max(main, t['jacobi']) if main > 0 else t['jacobi']


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
    # each rank's refresh is one eigh_many over its set: the set model, not
    # a sum of single factors
    pred = [refresh_ms(ns) if ns else 0.0 for ns in per]
    return {'world': world, 'cost': cost, 'factors_per_rank': per,
            'predicted_ms': pred, 'max_ms': max(pred) if pred else 0.0}
