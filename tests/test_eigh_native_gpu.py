"""The DEFAULT eigensolver tier selection at production factor sizes against
float64 ``torch.linalg.eigh`` (reference: kfac/layers/eigen.py:294-347).

Factors are K-FAC-like: an EMA of sample second moments over an identity
start (decayed), i.e. PSD, with a cluster of eigenvalues near the decayed
identity and a rank-deficient data part.
"""
from __future__ import annotations

import pytest
import torch

from distributed_kfac_pytorch_amd.ops import linalg

pytestmark = pytest.mark.gpu


def _factor(n: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    a = 0.95 ** 11 * torch.eye(n, dtype=torch.float64)
    for _ in range(3):
        x = torch.randn(max(8, n // 3), n, generator=g, dtype=torch.float64)
        x *= torch.rand(n, generator=g, dtype=torch.float64) ** 2  # uneven columns
        a = 0.95 * a + 0.05 * (x.T @ x) / x.shape[0]
    return a


def _check(a64: torch.Tensor, d: torch.Tensor, q: torch.Tensor) -> None:
    d, q = d.double().cpu(), q.double().cpu()
    n = a64.shape[0]
    ref = torch.linalg.eigvalsh(a64)
    nrm = float(torch.linalg.matrix_norm(a64, ord=2))
    assert float((d - ref).abs().max()) <= 1e-5 * nrm
    rec = q @ torch.diag(d) @ q.T
    assert float((rec - a64).norm() / a64.norm()) <= 1e-5
    assert float((q.T @ q - torch.eye(n, dtype=torch.float64)).abs().max()) <= 1e-5


@pytest.mark.parametrize('n', [129, 577, 1152, 2304, 4608])
def test_default_tier_matches_float64(cuda, n: int) -> None:
    a64 = _factor(n, n)
    linalg.last_stats.clear()
    (d, q), = linalg.eigh_many([a64.float().to(cuda)])
    torch.cuda.synchronize()
    tiers = {t[0] for t in linalg.last_stats.get('tiers', [])}
    assert tiers == {'sytrd+dc'}, tiers  # no rocSOLVER eigensolver
    _check(a64, d, q)


def test_mixed_refresh_two_rounds(cuda) -> None:
    """A ResNet-50-like mix (every tier, several chains) twice in a row
    (the second refresh reuses the lanes, streams and chain state)."""
    sizes = [64, 147, 256, 512, 576, 1000, 1152, 2049, 2304, 4608]
    mats64 = [_factor(n, 7 + i) for i, n in enumerate(sizes)]
    mats = [m.float().to(cuda) for m in mats64]
    res = linalg.eigh_many(mats)
    torch.cuda.synchronize()
    for a64, (d, q) in zip(mats64, res):
        _check(a64, d, q)
    res2 = linalg.eigh_many(mats)
    torch.cuda.synchronize()
    for a64, (d, q) in zip(mats64, res2):
        _check(a64, d, q)


_COLD = r'''
import sys, torch
sys.path.insert(0, {root!r})
from tests.test_eigh_native_gpu import _factor, _check
from distributed_kfac_pytorch_amd.ops import linalg
mats64 = [_factor(n, 31 + i) for i, n in enumerate((1000, 2049, 1000))]
res = linalg.eigh_many([m.float().cuda() for m in mats64])
torch.cuda.synchronize()
for a64, (d, q) in zip(mats64, res):
    _check(a64, d, q)
print('ok', sorted({{t[0] for t in linalg.last_stats['tiers']}}))
'''


def test_cold_process_chain_1000_2049() -> None:
    """Round 2 saw one fault of a chain holding n = 1000 and 2049 in a COLD
    bench process (first refresh, fresh allocator and streams); those sizes
    run through the chains on every ResNet-50 refresh since round 3.  Here:
    a fresh process whose first GPU work is exactly that bucket mix."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, '-c', _COLD.format(root=root)], cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert 'ok' in p.stdout and 'sytrd+dc' in p.stdout, p.stdout


_MODES = r'''
import sys, torch
sys.path.insert(0, {root!r})
from tests.test_eigh_native_gpu import _factor, _check
from distributed_kfac_pytorch_amd.ops import linalg
sizes = [147, 256, 256, 512, 576, 577, 1000, 1152, 2049, 2304, 4608, 4608]
mats64 = [_factor(n, 50 + i) for i, n in enumerate(sizes)]
for rnd in range(2):
    res = linalg.eigh_many([m.float().cuda() for m in mats64])
    torch.cuda.synchronize()
    for a64, (d, q) in zip(mats64, res):
        _check(a64, d, q)
print('ok', sorted({{t[0] for t in linalg.last_stats['tiers']}}))
'''


@pytest.mark.parametrize('env', [
    {},                                                          # default chain
    {'KFAC_SYTRD_SU': '8'},                                      # 8 column blocks in flight
])
def test_chain_variants_match_float64(env) -> None:
    """Every Householder-chain variant (csrc/sytrd.hip: symv column blocks in
    flight) on a mix of chain sizes -- including ResNet-50's 256 / 512 / 576
    -- twice in a fresh
    process (the variant is chosen once per process).  (The round-5
    persistent-panel and tile-symv variants, which returned wrong eigenpairs
    at 256 / 512 / 576 with PERSIST_FRAC 0.9 and were slower everywhere, are
    gone.)"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, '-c', _MODES.format(root=root)], cwd=root,
                       capture_output=True, text=True, timeout=240,
                       env={**os.environ, **env})
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert 'ok' in p.stdout and 'sytrd+dc' in p.stdout, p.stdout
