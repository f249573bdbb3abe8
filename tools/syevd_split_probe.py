"""syevd on 3 x 4608 factors: one strided-batched call vs three sequential
single-matrix calls (a 4608^2 fp32 factor is 85 MB: one fits the 256 MB
Infinity Cache, three do not -- the one-stage tridiagonalisation re-reads
the trailing matrix for every column)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402

lib = _native.native()
for n in (4608, 2304, 2048):
    cnt = 3 if n == 4608 else 6
    x = torch.randn(cnt, n, n // 3, device='cuda')
    a = (x @ x.transpose(1, 2) / n + 1e-3 * torch.eye(n, device='cuda')).contiguous()

    def batched():
        return lib.rocsolver_eigh(a.clone(), 0, 100, 1e-7)

    def split():
        return [lib.rocsolver_eigh(a[i:i + 1].clone(), 0, 100, 1e-7) for i in range(cnt)]

    for name, fn in (('batched', batched), ('split', split)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        print(json.dumps({'n': n, 'count': cnt, 'mode': name,
                          'ms': round((time.perf_counter() - t0) / 2 * 1e3, 1)}), flush=True)
