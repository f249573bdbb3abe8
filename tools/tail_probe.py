"""Time the tail of the native large-n eigensolver tier per size bucket:
rocSOLVER stedc alone, stedc + rocSOLVER ormtr (tridiag_eigvecs), and
stedc + the blocked UT back-transform (ops.linalg.apply_q_blocked), with the
reconstruction / orthogonality error of each.  JSON lines."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402
from distributed_kfac_pytorch_amd.ops.linalg import apply_q_blocked  # noqa: E402

SIZES = {512: 19, 1024: 14, 2048: 6, 2304: 6, 4608: 3}


def timed(fn):  # type: ignore[no-untyped-def]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return out, round((time.perf_counter() - t0) * 1e3, 2)


def err(a: torch.Tensor, w: torch.Tensor, x: torch.Tensor) -> tuple[float, float]:
    a, w, x = a.double(), w.double(), x.double()
    r = (a @ x - x * w.unsqueeze(1)).flatten(1).norm(dim=1) / a.flatten(1).norm(dim=1)
    eye = torch.eye(a.shape[-1], device=a.device, dtype=a.dtype)
    o = (x.transpose(1, 2) @ x - eye).flatten(1).norm(dim=1) / a.shape[-1] ** 0.5
    return float(r.max()), float(o.max())


def main() -> None:
    dev = torch.device('cuda')
    lib = native()
    only = os.environ.get('ONLY')
    sizes = {int(only): SIZES[int(only)]} if only else SIZES
    for n, c in sizes.items():
        torch.manual_seed(n)
        x = torch.randn(c, n, n // 3 + 8, device=dev)
        a = (x @ x.transpose(1, 2)) / n + 1e-4 * torch.eye(n, device=dev)
        for rep in range(2):
            red = a.clone()
            (d, e, tau), t_chain = timed(lambda: lib.sytrd_reduce([red]))
            row = {'n': n, 'cnt': c, 'rep': rep, 'chain_ms': t_chain}
            (w0, z0), row['stedc_ms'] = timed(lambda: lib.tridiag_stedc(d.clone(), e.clone()))
            (w1, x1), row['stedc_ormtr_ms'] = timed(
                lambda: lib.tridiag_eigvecs(red.clone(), d.clone(), e.clone(), tau))
            row['rocsolver_resid'], row['rocsolver_orth'] = err(a, w1, x1)
            for nb in (128, 256, 512):
                x2, row[f'applyq{nb}_ms'] = timed(lambda: apply_q_blocked(red, tau, z0, nb=nb))
                row[f'applyq{nb}_resid'], row[f'applyq{nb}_orth'] = err(a, w0, x2)
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
