"""Run the native rocSOLVER syevd on one n x n SPD matrix a few times
(rocprofv3 target: per-kernel breakdown of the large-factor eigensolver)."""
from __future__ import annotations

import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4608
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
x = torch.randn(1, n, 2 * n, device='cuda')
a = (x @ x.transpose(1, 2)) / (2 * n) + 1e-3 * torch.eye(n, device='cuda')
lib = native()
for i in range(reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    lib.rocsolver_eigh(a.clone(), 0, 100, 1e-7)
    torch.cuda.synchronize()
    print(f'n={n} rep={i} syevd {1e3 * (time.perf_counter() - t):.1f} ms', flush=True)
