"""Blocked UT back-transform of the tridiagonalisation (ops.linalg.
apply_q_blocked) on the CPU: reflectors from LAPACK ssytrd (scipy) in the
native kernel's layout (reflector k in row k), eigenvectors of T from
scipy; X = Q Z must diagonalise A and be orthonormal, for block widths that
do and do not divide n - 1."""
from __future__ import annotations

import numpy as np
import pytest
import scipy.linalg as sl
import torch
from scipy.linalg import lapack

from distributed_kfac_pytorch_amd.ops.linalg import apply_q_blocked


@pytest.mark.parametrize('n,nb', [(2, 512), (5, 2), (37, 8), (300, 64), (700, 256), (600, 512)])
def test_apply_q_blocked_matches_lapack(n: int, nb: int) -> None:
    rng = np.random.default_rng(n)
    x = rng.standard_normal((n, n // 2 + 1)).astype(np.float32)
    a = (x @ x.T / n).astype(np.float32)
    c, d, e, tau, info = lapack.ssytrd(a, lower=1)
    assert info == 0
    w, z = sl.eigh_tridiagonal(d.astype(np.float64), e[: n - 1].astype(np.float64))
    red = torch.tensor(np.ascontiguousarray(c.T))[None]
    t = torch.zeros(1, n)
    t[0, : n - 1] = torch.tensor(tau[: n - 1].astype(np.float32))
    xq = apply_q_blocked(red, t, torch.tensor(z.astype(np.float32))[None], nb=nb)[0].double().numpy()
    a64 = a.astype(np.float64)
    assert np.linalg.norm(a64 @ xq - xq * w) / np.linalg.norm(a64) < 1e-5
    assert np.abs(xq.T @ xq - np.eye(n)).max() < 1e-5


def test_apply_q_blocked_zero_tau_is_identity_reflector() -> None:
    """tau = 0 (nothing to annihilate) must contribute H = I whatever is
    stored in the reflector row."""
    n = 6
    red = torch.randn(1, n, n)
    tau = torch.zeros(1, n)
    z = torch.eye(n)[None]
    assert torch.allclose(apply_q_blocked(red, tau, z, nb=4), z)
