"""Time ``ops.linalg.eigh_many`` on K-FAC-like factors and check accuracy.

    python tools/eigh_probe.py --sizes 4608 --count 1 [--reps 3] [--mix resnet50]

Factors are ``X X^T / k + 1e-4 I`` with ``k = n / 2`` columns (rank-deficient
spectrum, as K-FAC activation covariances); accuracy against float64
``torch.linalg.eigh`` for the first factor of each size.  One JSON line per
configuration; ``last_stats['tiers']`` says which solver ran each bucket.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402

RESNET50 = {64: 12, 128: 12, 147: 1, 256: 26, 512: 19, 576: 3, 1000: 1,
            1024: 14, 1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}


def factor(n: int, dev: torch.device, seed: int) -> torch.Tensor:
    g = torch.Generator(device='cpu').manual_seed(seed)
    k = max(1, n // 2)
    x = torch.randn(n, k, generator=g, dtype=torch.float64)
    x = x * torch.logspace(0, -3, k, dtype=torch.float64)  # decaying spectrum
    a = x @ x.T / k + 1e-4 * torch.eye(n, dtype=torch.float64)
    return a.to(torch.float32).to(dev)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='4608')
    ap.add_argument('--count', type=int, default=1)
    ap.add_argument('--mix', default='')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--no-acc', action='store_true')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    if args.mix == 'resnet50':
        sizes = dict(RESNET50)
    else:
        sizes = {int(s): args.count for s in args.sizes.split(',')}
    mats = []
    for n, c in sizes.items():
        for j in range(c):
            mats.append(factor(n, dev, 1000 * n + j))
    torch.cuda.synchronize()
    times = []
    for r in range(args.reps + 1):
        linalg.last_stats.clear()
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = linalg.eigh_many(mats)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t) * 1e3)
    rec = {'sizes': sizes, 'ms_cold': round(times[0], 2),
           'ms': [round(t, 2) for t in times[1:]],
           'ms_min': round(min(times[1:]), 2) if len(times) > 1 else None,
           'tiers': sorted(set(map(tuple, linalg.last_stats.get('tiers', []))))}
    if not args.no_acc:
        acc = {}
        seen = set()
        for m, (w, v) in zip(mats, res):
            n = m.shape[0]
            if n in seen:
                continue
            seen.add(n)
            a = m.double()
            wr = torch.linalg.eigvalsh(a)
            vd = v.double()
            resid = float((a @ vd - vd * w.double()).norm() / a.norm())
            orth = float((vd.T @ vd - torch.eye(n, dtype=torch.float64, device=dev)).abs().max())
            err = float((w.double() - wr).abs().max() / wr.abs().max())
            acc[n] = {'eval_err': err, 'resid': resid, 'orth': orth}
        rec['acc'] = acc
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
