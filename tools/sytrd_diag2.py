"""Diagnostic: orthogonality of Q formed (fp64, host) from the reflectors of
the native tridiagonalisation, and the reconstruction, per matrix, for the
sytrd-tier test's mixed sizes (KFAC_SYTRD_FUSED selects the kernel mode)."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402


def form_q(refl: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
    n = refl.shape[0]
    v = torch.triu(refl, diagonal=2)
    idx = torch.arange(n - 1)
    v[idx, idx + 1] = 1.0
    q = torch.eye(n, dtype=torch.float64)
    for k in range(n - 2, -1, -1):
        q = q - float(tau[k]) * torch.outer(v[k], v[k] @ q)
    return q


def main() -> None:
    dev = torch.device('cuda')
    torch.manual_seed(7)
    sizes = (65, 96, 97, 130, 257)
    mats = []
    for j, n in enumerate(sizes):
        rows = n // 3 if j % 2 else 2 * n
        x = torch.randn(n, rows, device=dev)
        mats.append(x @ x.t() / rows + 1e-3 * torch.eye(n, device=dev))
    stacks = [m.unsqueeze(0).contiguous().clone() for m in mats]
    flat = native().sytrd_reduce(stacks)
    torch.cuda.synchronize()
    for s, (n, m) in enumerate(zip(sizes, mats)):
        d, e, tau = (t[0].double().cpu() for t in flat[3 * s:3 * s + 3])
        refl = stacks[s][0].double().cpu()
        q = form_q(refl, tau)
        t = torch.diag(d) + torch.diag(e[:n - 1], 1) + torch.diag(e[:n - 1], -1)
        orth = float((q.t() @ q - torch.eye(n, dtype=torch.float64)).abs().max())
        rec = float((q @ t @ q.t() - m.double().cpu()).abs().max())
        ev = torch.linalg.eigvalsh(t)
        ref = torch.linalg.eigvalsh(m.double().cpu())
        print(json.dumps({'mode': os.environ.get('KFAC_SYTRD_FUSED', '1'), 'n': n,
                          'orth': orth, 'recon': rec,
                          'eig_err': float((ev - ref).abs().max()),
                          'tau_range': [float(tau[:n - 1].min()), float(tau[:n - 1].max())]}),
              flush=True)


if __name__ == '__main__':
    main()
