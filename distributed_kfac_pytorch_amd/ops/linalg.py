"""Second-order linear algebra: batched symmetric eigensolver and SPD inverse.

``eigh_many(mats)`` decomposes a list of symmetric fp32 matrices of mixed
sizes in as few launches as possible:

* n <= ``jacobi_max_n()`` (128): one batched launch per size of the
  LDS-resident parallel Jacobi kernel (csrc/eigh_jacobi.hip), one matrix per
  workgroup, no host synchronisation.
* larger n: same-size matrices are stacked and sent through
  ``torch.linalg.eigh`` as one batched call (rocSOLVER), so the per-call
  latency and the host sync torch does to check ``info`` are paid once per
  size bucket instead of once per factor.

Results match ``torch.linalg.eigh``: ascending eigenvalues, eigenvectors in
columns.  Eigenvectors are unique only up to sign (and rotation inside
degenerate eigenspaces); K-FAC only uses them through ``Q f(D) Q^T``, which
is invariant to that freedom.
"""
from __future__ import annotations

import os
from collections import defaultdict

import torch

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native

JACOBI_SWEEPS = int(os.environ.get('KFAC_JACOBI_SWEEPS', '15'))
JACOBI_TOL = float(os.environ.get('KFAC_JACOBI_TOL', '1e-7'))


def jacobi_max_n() -> int:
    lib = native()
    return int(lib.jacobi_max_n()) if lib is not None else 0


def eigh_many(
    mats: list[torch.Tensor],
) -> list[tuple[torch.Tensor, torch.Tensor]]:
    """Eigendecompose each symmetric matrix; returns ``[(evals, evecs)]``."""
    out: list[tuple[torch.Tensor, torch.Tensor] | None] = [None] * len(mats)
    buckets: dict[tuple[int, torch.device], list[int]] = defaultdict(list)
    for i, m in enumerate(mats):
        buckets[(m.shape[0], m.device)].append(i)
    jmax = None
    for (n, dev), idxs in buckets.items():
        stack = torch.stack([mats[i].to(torch.float32) for i in idxs])
        if dev.type == 'cuda' and use_native(stack):
            if jmax is None:
                jmax = jacobi_max_n()
            if n <= jmax:
                evals, evecs = native().jacobi_eigh(
                    stack.contiguous(),
                    JACOBI_SWEEPS,
                    JACOBI_TOL,
                )
            else:
                evals, evecs = torch.linalg.eigh(stack)
        else:
            evals, evecs = torch.linalg.eigh(stack)
        for k, i in enumerate(idxs):
            out[i] = (evals[k], evecs[k])
    return [o for o in out if o is not None]


def eigh(mat: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Single-matrix convenience wrapper around ``eigh_many``."""
    return eigh_many([mat])[0]


def damped_inverse(mat: torch.Tensor, damping: float) -> torch.Tensor:
    """``(mat + damping*I)^-1`` computed in fp32 (reference inverse.py:
    185-212).  The damped factor is SPD, so a Cholesky factorisation plus
    ``cholesky_inverse`` replaces the general LU inverse (half the flops, no
    pivoting); if the factorisation fails (indefinite input) it falls back
    to ``torch.linalg.inv`` (checked on CPU only; on the GPU the check
    would be a host sync)."""
    a = mat.to(torch.float32)
    a = a + damping * torch.eye(a.shape[0], dtype=a.dtype, device=a.device)
    chol, info = torch.linalg.cholesky_ex(a)
    if a.is_cuda:
        # No host sync on the GPU path: a damped K-FAC factor is SPD by
        # construction (PSD running average + damping * I).
        return torch.cholesky_inverse(chol)
    if int(info) != 0:
        return torch.linalg.inv(a)
    return torch.cholesky_inverse(chol)
