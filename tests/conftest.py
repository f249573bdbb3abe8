"""Test configuration: the ``gpu`` marker and shared fixtures."""
from __future__ import annotations

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config: pytest.Config) -> None:
    config.addinivalue_line(
        'markers',
        'gpu: needs an MI355X (runs the native HIP kernels)',
    )


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from distributed_kfac_pytorch_amd.ops import _native

    if not _native.available():
        raise RuntimeError(f'native extension missing: {_native.load_error()!r}')
    return torch.device('cuda:0')


def pytest_sessionstart(session: pytest.Session) -> None:
    # The multi-process tests fork worker ranks from this process.  A BLAS /
    # OpenMP thread pool created here before a fork leaves the children's
    # pool in an unusable state (they hang in their first LAPACK call), so
    # the parent stays single-threaded.
    import torch

    torch.set_num_threads(1)
