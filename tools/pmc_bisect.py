"""One eigensolver stage at a time, for finding which one makes
``rocprofv3 --pmc`` crash (rounds 3-4: every counter pass over the
eigensolver probes segfaulted, even from one host thread).

    rocprofv3 --pmc SQ_WAVES -- python3 tools/pmc_bisect.py <stage> [--n N]

stages: matmul (control: a torch GEMM), jacobi (LDS Jacobi tier, n = 64),
sytrd (native tridiagonalisation only, default stream), sytrd_hi (the same
on a high-priority stream), dc (native divide and conquer of a random
tridiagonal), applyq (blocked back-transform), eigh (the whole default tier).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402


def spd(n: int, dev: torch.device) -> torch.Tensor:
    x = torch.randn(n, n // 2 + 1, device=dev)
    return (x @ x.T) / n + 1e-3 * torch.eye(n, device=dev)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('stage')
    ap.add_argument('--n', type=int, default=512)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    lib = native()
    n = args.n
    if args.stage == 'matmul':
        a = torch.randn(1024, 1024, device=dev)
        (a @ a).sum().item()
    elif args.stage == 'jacobi':
        linalg.eigh_many([spd(64, dev)])
    elif args.stage in ('sytrd', 'sytrd_hi'):
        a = spd(n, dev).unsqueeze(0).contiguous()
        if args.stage == 'sytrd_hi':
            lo, hi = torch.cuda.Stream.priority_range()
            s = torch.cuda.Stream(device=dev, priority=hi)
            with torch.cuda.stream(s):
                lib.sytrd_reduce([a])
            s.synchronize()
        else:
            lib.sytrd_reduce([a])
    elif args.stage == 'dc':
        d = torch.randn(1, n, device=dev)
        e = torch.randn(1, n - 1, device=dev)
        lib.tridiag_eigh_dc(d, e)
    elif args.stage == 'applyq':
        a = spd(n, dev).unsqueeze(0).contiguous()
        out = lib.sytrd_reduce([a])
        tau = out[2]
        z = torch.eye(n, device=dev).unsqueeze(0)
        torch.cuda.synchronize()
        linalg.apply_q_blocked(a, tau, z)
    elif args.stage == 'eigh':
        linalg.eigh_many([spd(n, dev)])
    else:
        raise SystemExit(f'unknown stage {args.stage}')
    torch.cuda.synchronize()
    print('ok', args.stage, flush=True)


if __name__ == '__main__':
    main()
