"""Fit the factor-set refresh model of parallel/costmodel.py to a measured
solver table (tools/solver_table.py output) and store the fit in it.

    python tools/fit_costmodel.py profiles/solver_table_mi355x.json [--write]

Every measurement is a factor SET timed as one ``eigh_many`` call: single
sizes, same-size batches, and each rank's set under the KAISA assignment at
N = 1/2/4/8 for ResNet-50 and GPT-NeoX-125M.  The parameters minimise the
squared log error over all of them (scipy least squares, positive
parameters); the table keeps the measurements, the fit and each set's
prediction so tests/test_costmodel.py can check the model against them.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np
from scipy.optimize import least_squares

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.parallel import costmodel  # noqa: E402


def measured_sets(table: dict) -> list[tuple[str, list[int], float]]:
    """``(label, sizes, ms)`` of every measurement in the table."""
    out = []
    for n, ms in table.get('single_ms', {}).items():
        out.append((f'1x{n}', [int(n)], float(ms)))
    for key, ms in table.get('batch_ms', {}).items():
        k, n = key.split('x')
        out.append((key, [int(n)] * int(k), float(ms)))
    for key, v in table.get('rank_ms', {}).items():
        per = v.get('sizes')
        if per is None:  # older tables: the assignment is deterministic
            model, world = key.split('/N')
            per = costmodel.plan(costmodel.model_factor_sizes(model), int(world),
                                 grad_worker_fraction=0.5)['factors_per_rank']
        for r, ms in enumerate(v['measured_ms']):
            if ms > 0:
                out.append((f'{key}/r{r}', [int(n) for n in per[r]], float(ms)))
    return out


def fit(sets: list[tuple[str, list[int], float]]) -> dict[str, float]:
    names = list(costmodel.REFRESH_PARAMS)
    x0 = np.log([costmodel.REFRESH_PARAMS[k] for k in names])

    def resid(x: np.ndarray) -> np.ndarray:
        p = dict(zip(names, np.exp(x)))
        return np.array([math.log(max(costmodel.refresh_ms(s, p), 1e-3) / ms)
                         for _, s, ms in sets])

    # a few starting points (the latency / bandwidth split has local minima)
    best = None
    rng = np.random.default_rng(0)
    for trial in range(24):
        start = x0 if trial == 0 else x0 + rng.normal(0.0, 0.8, size=x0.shape)
        r = least_squares(resid, start, method='trf')
        if best is None or r.cost < best.cost:
            best = r
    return {k: float(round(v, 5)) for k, v in zip(names, np.exp(best.x))}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('table')
    ap.add_argument('--write', action='store_true')
    args = ap.parse_args()
    with open(args.table) as f:
        table = json.load(f)
    sets = measured_sets(table)
    params = fit(sets)
    pred = {}
    worst = 0.0
    for label, s, ms in sets:
        p = costmodel.refresh_ms(s, params)
        pred[label] = {'measured_ms': ms, 'predicted_ms': round(p, 2)}
        worst = max(worst, abs(p / ms - 1))
        print(f'{label:28s} measured {ms:8.1f}  predicted {p:8.1f}  {100 * (p / ms - 1):+6.1f}%')
    print(json.dumps({'fit': params, 'worst_rel_err': round(worst, 3)}))
    if args.write:
        table['fit'] = params
        table['fit_predictions'] = pred
        with open(args.table, 'w') as f:
            json.dump(table, f, indent=1)


if __name__ == '__main__':
    main()
