"""CPU (float64) checks of the two-stage eigensolver's algorithms
(ops/twostage.py): the exact stage / schedule / blocking choices the HIP
kernels implement (csrc/sy2sb.hip, sb2st.hip, bt2.hip) against LAPACK."""
from __future__ import annotations

import pytest
import torch

from distributed_kfac_pytorch_amd.ops import twostage as ts


def _sym(n: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    m = torch.randn(n, n, generator=g, dtype=torch.float64)
    return m + m.T


@pytest.mark.parametrize('n,b', [(40, 4), (67, 16), (100, 16), (53, 8)])
def test_stage1_band_and_reconstruction(n: int, b: int) -> None:
    a = _sym(n, n)
    band, panels = ts.sy2sb_reference(a, b)
    idx = torch.arange(n)
    outside = (idx[:, None] - idx[None, :]).abs() > b
    assert band[outside].abs().max() < 1e-12
    q = ts.q1_apply_reference(panels, torch.eye(n, dtype=torch.float64), b)
    assert torch.allclose(q @ band @ q.T, a, atol=1e-11)


@pytest.mark.parametrize('n,b', [(60, 4), (90, 8), (70, 16)])
def test_stage2_pipeline_order_is_exact(n: int, b: int) -> None:
    a = _sym(n, 3 * n)
    band, _ = ts.sy2sb_reference(a, b)
    d0, e0, r0 = ts.sb2st_reference(band, b)
    d1, e1, r1 = ts.sb2st_reference(band, b, order='pipeline', seed=n)
    # the lag-3 dependency rule reproduces the sequential sweeps bit for bit
    assert torch.equal(d0, d1) and torch.equal(e0, e1)
    assert set(r0) == set(r1)


@pytest.mark.parametrize('n,b', [(70, 16), (61, 4)])
def test_bt2_step_schedule_matches_dense_product(n: int, b: int) -> None:
    a = _sym(n, 5 * n)
    band, _ = ts.sy2sb_reference(a, b)
    d, e, refl = ts.sb2st_reference(band, b)
    q2 = torch.eye(n, dtype=torch.float64)
    for (j, k) in sorted(refl):
        st, v, tau = refl[(j, k)]
        h = torch.eye(n, dtype=torch.float64)
        h[st:st + len(v), st:st + len(v)] -= tau * torch.outer(v, v)
        q2 = q2 @ h
    t = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    assert torch.allclose(q2 @ t @ q2.T, band, atol=1e-10)
    z = torch.randn(n, n, dtype=torch.float64)
    assert torch.allclose(ts.bt2_reference(refl, z, n, b), q2 @ z, atol=1e-12)


@pytest.mark.parametrize('n', [50, 97])
def test_full_pipeline_matches_lapack(n: int) -> None:
    a = _sym(n, 7 * n)
    w, x = ts.eigh_reference(a, 16, order='pipeline')
    w0 = torch.linalg.eigvalsh(a)
    assert torch.allclose(w, w0, atol=1e-10)
    assert torch.allclose(x @ torch.diag(w) @ x.T, a, atol=1e-10)
    assert torch.allclose(x.T @ x, torch.eye(n, dtype=torch.float64), atol=1e-12)
