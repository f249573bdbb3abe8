"""Latency-aware cost model for KAISA's second-order work placement.

The reference balances the per-rank eigendecomposition work on ``n^3`` of
each factor dimension (``kfac/preconditioner.py:266-281``).  On MI355X the
native eigensolver (csrc/sytrd.hip one-stage Householder chain, csrc/tridiag.hip
divide and conquer, blocked back-transform) is not flop-bound: every factor
pays a per-column chain of dependent launches (about n kernel pairs), so a
1152 factor costs far more than (1152/4608)^3 of a 4608 one, and a rank that
owns one large factor still waits for its whole chain.  ``n^3`` mis-balances
exactly the N = 8 case the refresh is amortised over.

``refresh_ms(sizes)`` predicts the refresh of a whole factor SET -- one
rank's ``ops.linalg.eigh_many`` call -- from a model of that schedule (below)
whose parameters are fitted to measured refreshes (``tools/solver_table.py``
measures, ``tools/fit_costmodel.py`` fits; ``profiles/solver_table_mi355x.json``
holds both).  ``solver_ms(n)`` is its single-factor value, the factor cost
of ``KFACPreconditioner(assignment_strategy='compute', cost_model='measured')``
(opt-in; ``'auto'`` keeps the reference's ``n^3``), so the LPT placement
(``parallel/assignment.py``, unchanged) balances predicted milliseconds.
``plan()`` prints each rank's predicted refresh at any world size without a
GPU.
"""
from __future__ import annotations

import json
import os
from typing import Any

import numpy as np

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
#   chain advances all its members one column per launch pair: column k
#   costs L0 (the col step and the launch gaps) plus the symv step, which
#   streams the members' trailing squares, b_k = 4 * sum (n - k - 1)^2
#   bytes, and takes max(L1 + L2 * (n_max - k) / 1000, b_k / BW): a latency
#   floor that grows with the launch's grid, or bandwidth, BW = bw_mall
#   while b_k fits the 256 MB Infinity Cache and bw_hbm above;
# * chains run concurrently on their own lanes: the slowest sets the pace,
#   and every other chain adds its bytes (shared bandwidth) and a fraction
#   nu of its column latency (its kernels take CU slots between the
#   critical chain's);
# * a fixed base per call plus bucket_ms per size bucket (its tail's
#   launches and joins), and the largest bucket's tail (divide and
#   conquer + back-transform, tail_b * count * n^3 / 1e9) after the chains.
#
# Parameters are fitted to measured refreshes by tools/fit_costmodel.py and
# stored with the measurements in profiles/solver_table_mi355x.json
# ("fit"); REFRESH_PARAMS are the fallback when that file is absent.
# ---------------------------------------------------------------------------

REFRESH_PARAMS: dict[str, float] = {
    'L0_us': 8.0, 'L1_us': 8.0, 'L2_us': 1.0, 'nu': 0.2, 'bw_mall_tbs': 6.0, 'bw_hbm_tbs': 3.0,
    'base_ms': 1.5, 'bucket_ms': 0.5,
    'tail_b': 0.05, 'jacobi_ms': 1.3, 'ts_a': 0.5, 'ts_b': 0.01,
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


_PARAMS: dict[str, float] | None = None


def _params() -> dict[str, float]:
    global _PARAMS
    if _PARAMS is None:
        _PARAMS = load_params()
    return _PARAMS


def _split_cuts() -> list[int]:
    return sorted((int(c) for c in os.environ.get('KFAC_SYTRD_SPLIT', '4000,1000').split(',')
                   if c), reverse=True)


def refresh_terms(sizes: list[int], params: dict[str, float] | None = None) -> dict[str, float]:
    """Per-term predicted milliseconds of one eigen refresh of ``sizes``
    (see the model above)."""
    from distributed_kfac_pytorch_amd.ops.linalg import JACOBI_MAX_N
    from distributed_kfac_pytorch_amd.ops.linalg import twostage_sizes

    p = params or _params()
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
    chains = []
    mall = 256.0 * 2 ** 20
    for g in groups:
        top = max(g)
        k = np.arange(top - 1, dtype=np.float64)
        b = np.zeros_like(k)
        for n, c in g.items():
            r = np.clip(n - k - 1, 0, None)
            b += 4.0 * c * r * r
        bw = np.where(b <= mall, p['bw_mall_tbs'], p['bw_hbm_tbs']) * 1e12
        floor = (p['L1_us'] + p['L2_us'] * (top - k) / 1000.0) * 1e-6
        symv = np.maximum(floor, b / bw)
        lat = p['L0_us'] * 1e-3 * (top - 1)
        chains.append((lat, float(symv.sum()) * 1e3))
    crit = max(range(len(chains)), key=lambda i: sum(chains[i])) if chains else -1
    lat = chains[crit][0] if chains else 0.0
    bwt = chains[crit][1] if chains else 0.0
    share = sum(p['nu'] * (l + b) for i, (l, b) in enumerate(chains) if i != crit)
    tail = 0.0
    if chain_sizes:
        n = max(chain_sizes)
        tail = p['tail_b'] * chain_sizes[n] * n ** 3 / 1e9
    two = sum(p['ts_a'] * counts[n] * n ** 3 / 1e9 + p['ts_b'] * n for n in ts)
    jacobi = p['jacobi_ms'] * len(jac)
    base = (p['base_ms'] + p['bucket_ms'] * len(chain_sizes)) if (chains or ts) else 0.0
    return {'latency': lat, 'bandwidth': bwt, 'other_chains': share, 'tail': tail,
            'twostage': two, 'jacobi': jacobi, 'base': base}


def refresh_ms(sizes: list[int], params: dict[str, float] | None = None) -> float:
    """Predicted milliseconds of one eigen refresh of the factor set
    ``sizes`` on one MI355X (ops.linalg.eigh_many)."""
    t = refresh_terms(sizes, params)
    main = (t['latency'] + t['bandwidth'] + t['other_chains'] + t['tail'] + t['twostage']
            + t['base'])
    return max(main, t['jacobi'])


def solver_ms(n: int, params: dict[str, float] | None = None) -> float:
    """Predicted refresh milliseconds of one ``n x n`` factor alone (the KAISA
    COMPUTE cost of ``cost_model='measured'``)."""
    return refresh_ms([int(n)], params)


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
