"""CPU tests of the eigensolver front-end plan (ops/linalg.py)."""
from __future__ import annotations

import torch

from distributed_kfac_pytorch_amd.ops import linalg


def _spd(n: int) -> torch.Tensor:
    x = torch.randn(n, 3 * n, dtype=torch.float64)
    return (x @ x.T / (3 * n)).float()


def test_eigh_many_cpu_matches_torch() -> None:
    torch.manual_seed(1)
    mats = [_spd(n) for n in (5, 40, 40, 90)]
    for m, (d, q) in zip(mats, linalg.eigh_many(mats)):
        torch.testing.assert_close(d, torch.linalg.eigvalsh(m), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close((q * d) @ q.T, m, rtol=1e-4, atol=1e-5)
