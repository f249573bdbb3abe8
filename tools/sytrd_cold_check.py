"""Diagnostic: run ONLY the native tridiagonalisation (no stedc) on the
step-0 (cold) ResNet-50 factors and report, per matrix, whether d / e / tau
are finite and in range.  JSON lines."""
from __future__ import annotations

import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from refresh_probe import snapshot  # noqa: E402

from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402


def main() -> None:
    mats, _ = snapshot(0)
    by = defaultdict(list)
    for m in mats:
        by[m.shape[0]].append(m)
    lib = native()
    keys = sorted(n for n in by if n >= 512)
    stacks = [torch.stack(by[n]).contiguous() for n in keys]
    print(json.dumps({'finite_inputs': [bool(torch.isfinite(s).all()) for s in stacks],
                      'sizes': keys}), flush=True)
    flat = lib.sytrd_reduce([s.clone() for s in stacks])
    torch.cuda.synchronize()
    for j, n in enumerate(keys):
        d, e, tau = flat[3 * j:3 * j + 3]
        for b in range(d.shape[0]):
            row = {'n': n, 'b': b, 'd_fin': bool(torch.isfinite(d[b]).all()),
                   'e_fin': bool(torch.isfinite(e[b]).all()),
                   'tau_fin': bool(torch.isfinite(tau[b]).all()),
                   'tau_min': float(tau[b, :n - 1].min()), 'tau_max': float(tau[b, :n - 1].max()),
                   'tau0': int((tau[b, :n - 1] == 0).sum()),
                   'e_absmax': float(e[b, :n - 1].abs().max()),
                   'd_absmax': float(d[b].abs().max()),
                   'fro': float(stacks[j][b].norm())}
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
