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


def test_twostage_bucket_rule():
    """Two-stage by bucket population: GPT-NeoX-125M's large buckets qualify,
    ResNet-50's step-100 mix stays on the one-stage chains."""
    from distributed_kfac_pytorch_amd.ops import linalg
    neox = {768: 24, 769: 36, 2304: 12, 3072: 12, 3073: 12}
    resnet = {64: 12, 128: 12, 147: 1, 256: 26, 512: 19, 576: 3, 1000: 1, 1024: 14,
              1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}
    assert linalg.twostage_sizes(neox) == set(neox)
    assert linalg.twostage_sizes(resnet) == set()


def test_chain_waves_knob(monkeypatch) -> None:
    from distributed_kfac_pytorch_amd.ops.linalg import _chain_waves

    monkeypatch.delenv('KFAC_SYTRD_WAVES', raising=False)
    assert _chain_waves(0) == 0 and _chain_waves(2) == 0  # 0 = the kernel's default
    monkeypatch.setenv('KFAC_SYTRD_WAVES', '6144,2048')
    assert [_chain_waves(g) for g in range(4)] == [6144, 2048, 2048, 2048]
