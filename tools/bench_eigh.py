"""Time the eigensolver paths on the ResNet-50 K-FAC factor size mix.

For every distinct factor dimension n (with its multiplicity in ResNet-50):
  * torch.linalg.eigh one matrix at a time
  * torch.linalg.eigh batched over the same-size factors
  * the native batched Jacobi kernel (n <= 128)
Prints one JSON line per size and a total.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402

SIZES = {64: 12, 128: 12, 147: 1, 256: 26, 512: 19, 576: 3, 1000: 1,
         1024: 14, 1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main() -> None:
    dev = torch.device('cuda')
    tot_single = tot_batched = tot_best = 0.0
    for n, cnt in SIZES.items():
        x = torch.randn(cnt, n, 2 * n, device=dev)
        a = (x @ x.transpose(1, 2)) / (2 * n) + 1e-3 * torch.eye(n, device=dev)
        reps = 1 if n >= 2048 else 2
        single = timed(lambda: [torch.linalg.eigh(a[i]) for i in range(cnt)], reps)
        batched = timed(lambda: torch.linalg.eigh(a), reps)
        row = {'n': n, 'count': cnt, 'single_ms': round(single, 2),
               'batched_ms': round(batched, 2)}
        best = min(single, batched)
        if n <= linalg.jacobi_max_n():
            jac = timed(lambda: native().jacobi_eigh(a.contiguous(), 15, 1e-7), reps)
            row['jacobi_ms'] = round(jac, 2)
            best = min(best, jac)
        tot_single += single
        tot_batched += batched
        tot_best += best
        print(json.dumps(row), flush=True)
    print(json.dumps({'total_single_ms': round(tot_single, 1),
                      'total_batched_ms': round(tot_batched, 1),
                      'total_best_ms': round(tot_best, 1)}), flush=True)


if __name__ == '__main__':
    main()
