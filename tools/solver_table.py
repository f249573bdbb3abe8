"""Measure the native eigensolver's refresh time per factor size (and per
batch), the table behind the latency-aware KAISA cost model
(parallel/costmodel.py), and the refresh time of each rank's factor set
under the KAISA assignment at N = 2 / 4 / 8 for ResNet-50 and GPT-NeoX-125M.

    python tools/solver_table.py > profiles/solver_table_mi355x.json
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402
from distributed_kfac_pytorch_amd.parallel import costmodel  # noqa: E402


def factor(n: int, seed: int, dev: torch.device) -> torch.Tensor:
    g = torch.Generator(device='cpu').manual_seed(seed)
    x = torch.randn(max(8, n // 3), n, generator=g)
    a = 0.57 * torch.eye(n) + 0.43 * (x.T @ x) / x.shape[0]
    return a.to(dev)


def timed(mats: list[torch.Tensor], reps: int = 3) -> float:
    linalg.eigh_many([m.clone() for m in mats])  # warm: allocator, handles
    torch.cuda.synchronize()
    best = float('inf')
    for _ in range(reps):
        ms = [m.clone() for m in mats]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        linalg.eigh_many(ms)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    return best


def main() -> None:
    dev = torch.device('cuda')
    out: dict = {'single_ms': {}, 'batch_ms': {}, 'rank_ms': {}}
    for n in (129, 256, 512, 768, 1024, 1536, 2048, 2304, 3072, 4096, 4608):
        out['single_ms'][n] = round(timed([factor(n, n, dev)]), 2)
        print(json.dumps({'n': n, 'ms': out['single_ms'][n]}), file=sys.stderr, flush=True)
    for n, k in ((1152, 4), (2304, 6), (4608, 3), (3072, 12)):
        out['batch_ms'][f'{k}x{n}'] = round(timed([factor(n, n + i, dev) for i in range(k)], 2), 2)
    for model in ('resnet50', 'gpt_neox_125m'):
        sizes = costmodel.model_factor_sizes(model)
        for world in (1, 2, 4, 8):
            plan = costmodel.plan(sizes, world, grad_worker_fraction=0.5)
            per = []
            for r in range(world):
                ns = plan['factors_per_rank'][r]
                mats = [factor(n, 100 + i, dev) for i, n in enumerate(ns)]
                per.append(round(timed(mats, reps=2), 1) if mats else 0.0)
                del mats
                torch.cuda.empty_cache()
            out['rank_ms'][f'{model}/N{world}'] = {
                'measured_ms': per, 'predicted_ms': [round(v, 1) for v in plan['predicted_ms']],
                'sizes': plan['factors_per_rank']}
            print(json.dumps({model: world, 'measured': per,
                              'predicted': plan['predicted_ms']}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
