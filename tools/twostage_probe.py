"""GPU probe of the two-stage eigensolver: accuracy against float64 eigh and
per-stage time for K-FAC-like factors of the ResNet-50 / GPT-NeoX sizes.

    python tools/twostage_probe.py [--sizes 129,577,2304,4608] [--batch 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.ops import twostage  # noqa: E402


def factor(n: int, batch: int, seed: int, dev: torch.device) -> torch.Tensor:
    """EMA-like K-FAC factor: X^T X / m of m < n random rows (rank deficient)
    plus a smaller full-rank part."""
    g = torch.Generator(device='cpu').manual_seed(seed)
    out = []
    for _ in range(batch):
        m = max(8, n // 2)
        x = torch.randn(m, n, generator=g, dtype=torch.float64)
        f = x.T @ x / m + 1e-3 * torch.eye(n, dtype=torch.float64)
        out.append(f)
    return torch.stack(out).to(dev, torch.float32)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='129,147,256,577,1000,1152,2049,2304,4608')
    ap.add_argument('--batch', type=int, default=1)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda')
    for n in [int(s) for s in args.sizes.split(',')]:
        a = factor(n, args.batch, n, dev)
        twostage.eigh_twostage(a)  # warm-up
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            w, x, err, _ = twostage.eigh_twostage(a)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        w, x, err, ms = twostage.eigh_twostage(a, timed=True)  # warm per-stage times
        ad = a.double()
        w64 = torch.linalg.eigvalsh(ad)
        xd, wd = x.double(), w.double()
        nrm = torch.linalg.matrix_norm(ad).clamp_min(1e-30)
        res = torch.linalg.matrix_norm(ad @ xd - xd * wd.unsqueeze(1)) / nrm
        eye = torch.eye(n, dtype=torch.float64, device=dev)
        orth = torch.linalg.matrix_norm(xd.transpose(1, 2) @ xd - eye)
        rec = {
            'n': n, 'batch': args.batch, 'err': int(err.max().item()),
            'finite': bool(torch.isfinite(x).all() and torch.isfinite(w).all()),
            'eig_maxrel': float(((wd - w64).abs().amax(1) / w64.abs().amax(1)).max()),
            'resid_rel': float(res.max()), 'orth': float(orth.max()),
            'ms': round(best, 3), 'stage_ms': [round(float(t), 3) for t in ms],
        }
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
