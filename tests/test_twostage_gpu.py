"""GPU checks of the native two-stage eigensolver (csrc/sy2sb.hip,
sb2st.hip, bt2.hip, twostage_host.cpp) against float64 eigh, at the sizes of
the ResNet-50 / GPT-NeoX factors (reference: torch.linalg.eigh in
kfac/layers/eigen.py:294-347)."""
from __future__ import annotations

import pytest
import torch

from distributed_kfac_pytorch_amd.ops import twostage

pytestmark = pytest.mark.gpu


def _factor(n: int, batch: int, seed: int, dev: torch.device) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(batch):
        m = max(8, n // 2)  # rank deficient, like a young K-FAC factor
        x = torch.randn(m, n, generator=g, dtype=torch.float64)
        out.append(x.T @ x / m + 1e-3 * torch.eye(n, dtype=torch.float64))
    return torch.stack(out).to(dev, torch.float32)


def _check(a: torch.Tensor, w: torch.Tensor, x: torch.Tensor, tol: float = 2e-5) -> None:
    assert torch.isfinite(w).all() and torch.isfinite(x).all()
    ad, xd, wd = a.double(), x.double(), w.double()
    w64 = torch.linalg.eigvalsh(ad)
    scale = w64.abs().amax(1)
    assert float(((wd - w64).abs().amax(1) / scale).max()) <= tol
    res = torch.linalg.matrix_norm(ad @ xd - xd * wd.unsqueeze(1)) / torch.linalg.matrix_norm(ad)
    assert float(res.max()) <= tol
    n = a.shape[-1]
    eye = torch.eye(n, dtype=torch.float64, device=a.device)
    assert float((xd.transpose(1, 2) @ xd - eye).abs().max()) <= tol


@pytest.mark.parametrize('n', [129, 147, 577, 1000, 1152, 2049, 2304, 4608])
def test_twostage_matches_float64(cuda, n: int) -> None:
    a = _factor(n, 1, n, cuda)
    w, x, err, _ = twostage.eigh_twostage(a)
    assert int(err.max().item()) == 0
    _check(a, w, x)


def test_twostage_batch_mixed_spectra(cuda) -> None:
    # a batch with a zero matrix, a diagonal one and a random factor
    n = 300
    a = _factor(n, 3, 11, cuda)
    a[0].zero_()
    a[1] = torch.diag(torch.linspace(0.0, 1.0, n, device=cuda))
    w, x, err, _ = twostage.eigh_twostage(a)
    assert int(err.max().item()) == 0
    assert torch.isfinite(w).all() and torch.isfinite(x).all()
    _check(a[2:], w[2:], x[2:])
    assert float(w[0].abs().max()) == 0.0
