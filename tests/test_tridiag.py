"""Tridiagonal divide and conquer (K-HIP-3 last stage).

CPU: the float64 reference (ops/tridiag.py) against LAPACK through
``torch.linalg.eigh``.  GPU: the native batched solver (csrc/tridiag.hip)
against float64 ``torch.linalg.eigh`` of the same tridiagonals, at the sizes
of the ResNet-50 / GPT-NeoX factors.
"""
from __future__ import annotations

import pytest
import torch

from distributed_kfac_pytorch_amd.ops import tridiag


def _dense(d: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    return torch.diag_embed(d) + torch.diag_embed(e, 1) + torch.diag_embed(e, -1)


def _check(w: torch.Tensor, z: torch.Tensor, d: torch.Tensor, e: torch.Tensor, tol: float):
    a = _dense(d.double(), e.double())
    wr = torch.linalg.eigvalsh(a)
    nrm = torch.linalg.matrix_norm(a, ord=2, keepdim=False).reshape(-1, 1)
    w, z = w.double(), z.double()
    assert (w - wr).abs().div(nrm).max() <= tol
    eye = torch.eye(d.shape[-1], dtype=torch.float64)
    assert (z.transpose(-1, -2) @ z - eye).abs().max() <= tol * 10
    res = (a @ z - z * w.unsqueeze(-2)).norm(dim=(-2, -1)) / nrm.reshape(-1)
    assert res.max() <= tol * 10


def _cases(n: int, seed: int = 0) -> list[tuple[torch.Tensor, torch.Tensor]]:
    g = torch.Generator().manual_seed(seed + n)
    out = [(torch.randn(n, generator=g), torch.randn(n - 1, generator=g))]
    # a tight cluster (identity-dominated EMA factor) and decoupled blocks
    d = torch.ones(n) + 1e-7 * torch.randn(n, generator=g)
    e = 1e-6 * torch.randn(n - 1, generator=g)
    if n > 8:
        e[n // 3] = 0.0
    out.append((d, e))
    # PSD factor-like spectrum: tridiagonal of a Householder reduction
    x = torch.randn(n, max(2, n // 4), generator=g, dtype=torch.float64)
    a = x @ x.T / x.shape[1] + 0.5 * torch.eye(n, dtype=torch.float64)
    q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    from scipy.linalg import hessenberg
    h = torch.from_numpy(hessenberg((q @ a @ q.T).numpy()))
    out.append((torch.diagonal(h).float().clone(), torch.diagonal(h, 1).float().clone()))
    return out


@pytest.mark.parametrize('n', [1, 2, 5, 64, 65, 100, 130])
def test_reference_matches_lapack(n: int) -> None:
    for d, e in _cases(n):
        w, z = tridiag.tridiag_eigh_reference(d, e)
        _check(w.unsqueeze(0), z.unsqueeze(0), d.unsqueeze(0), e.unsqueeze(0), 1e-6)


def test_plan_padding() -> None:
    for n in (65, 129, 147, 577, 1000, 1152, 2049, 2304, 3073, 4608):
        leaf, levels, n_pad = tridiag.dc_plan(n)
        assert leaf <= tridiag.LEAF_MAX and n_pad == leaf << levels >= n
        assert n_pad - n <= max(1, n // 32)
    assert tridiag.dc_plan(4608) == (36, 7, 4608)


@pytest.mark.gpu
@pytest.mark.parametrize('n', [2, 5, 64, 65, 129, 577, 1152, 2304, 4608])
def test_native_dc_matches_float64(cuda, n: int) -> None:
    from distributed_kfac_pytorch_amd.ops import _native

    lib = _native.native()
    assert tuple(lib.tridiag_dc_plan(n)) == tridiag.dc_plan(n)
    cases = _cases(n) if n <= 1152 else _cases(n)[::2]
    d = torch.stack([c[0] for c in cases])
    e = torch.stack([c[1] for c in cases])
    w, z = lib.tridiag_eigh_dc(d.to(cuda), e.to(cuda))
    torch.cuda.synchronize()
    assert w.shape == d.shape and z.shape == (d.shape[0], n, n)
    assert bool(torch.isfinite(w).all()) and bool(torch.isfinite(z).all())
    _check(w.cpu(), z.cpu(), d, e, 2e-6 * max(1.0, (n / 64) ** 0.5))
