"""Time the native sytrd tier stages on the ResNet-50 factor mix (n >= 512):
sytrd_reduce alone, then stedc + ormtr per bucket.  JSON lines."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402

SIZES = {512: 19, 576: 3, 1000: 1, 1024: 14, 1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}


def main() -> None:
    dev = torch.device('cuda')
    lib = native()
    only = os.environ.get('ONLY')
    sizes = {int(only): SIZES[int(only)]} if only else SIZES
    base = {}
    for n, c in sizes.items():
        x = torch.randn(c, n, 2 * n, device=dev)
        base[n] = (x @ x.transpose(1, 2)) / (2 * n) + 1e-3 * torch.eye(n, device=dev)
    for rep in range(3):
        stacks = [base[n].clone() for n in sizes]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        flat = lib.sytrd_reduce(stacks)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        row = {'rep': rep, 'sizes': list(sizes), 'sytrd_host_ms': round((t1 - t0) * 1e3, 1),
               'sytrd_ms': round((t2 - t0) * 1e3, 1)}
        for j, n in enumerate(sizes):
            d, e, tau = flat[3 * j:3 * j + 3]
            t3 = time.perf_counter()
            lib.tridiag_eigvecs(stacks[j], d, e, tau)
            torch.cuda.synchronize()
            row[f'tri_{n}x{sizes[n]}_ms'] = round((time.perf_counter() - t3) * 1e3, 1)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
