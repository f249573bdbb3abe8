"""PMC workload: the native tridiagonalisation alone (no rocSOLVER, which
faults under counter collection): 3 x 4608 and 6 x 2304 SPD factors, two
reductions each."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402


def main() -> None:
    dev = torch.device('cuda')
    lib = native()
    torch.manual_seed(0)
    base = []
    for n, c in ((4608, 3), (2304, 6)):
        x = torch.randn(c, n, n // 2, device=dev)
        base.append((x @ x.transpose(1, 2)) / n + 1e-3 * torch.eye(n, device=dev))
    for _ in range(2):
        lib.sytrd_reduce([b.clone() for b in base])
    torch.cuda.synchronize()
    print('ok')


if __name__ == '__main__':
    main()
