"""Native NHWC max pooling (ops/pool.py, csrc/pool.hip)."""
from __future__ import annotations

import pytest
import torch
from torch import nn

from distributed_kfac_pytorch_amd.ops.pool import MaxPool2dNHWC


def test_maxpool_nhwc_cpu_fallback_matches_torch() -> None:
    """On the CPU (and for any input the kernels do not take) the module is
    ``nn.MaxPool2d``: same output, same gradient, no parameters."""
    torch.manual_seed(0)
    x = torch.randn(2, 8, 13, 11).contiguous(memory_format=torch.channels_last)
    a, b = MaxPool2dNHWC(3, 2, 1), nn.MaxPool2d(3, 2, 1)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = a(xa), b(xb)
    assert torch.equal(ya, yb)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(xa.grad, xb.grad)
    assert not list(a.parameters()) and a.state_dict() == {}


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('shape,k,s,p', [((32, 64, 112, 112), 3, 2, 1), ((3, 16, 9, 11), 3, 2, 1),
                                         ((2, 8, 10, 10), 2, 2, 0), ((2, 24, 15, 13), 5, 3, 2),
                                         ((1, 8, 7, 7), 3, 1, 1)])
def test_maxpool_nhwc_native_matches_torch(cuda, dtype, shape, k, s, p, monkeypatch) -> None:
    """The native kernels run, the output equals torch's bit for bit, the
    input gradient matches torch's (sums of up to ceil(k/s)^2 window
    gradients: fixed order here) and repeats bit for bit -- also with the
    ties a ReLU leaves (zeros: the first maximum in window order wins)."""
    from distributed_kfac_pytorch_amd.ops import _native

    lib = _native.native()
    assert lib is not None, _native.load_error()
    calls = []

    class Spy:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(lib, name)

        def maxpool_nhwc_bwd(self, *a):  # type: ignore[no-untyped-def]
            calls.append('bwd')
            return lib.maxpool_nhwc_bwd(*a)

    monkeypatch.setattr(_native, 'native', lambda: Spy())
    torch.manual_seed(0)
    x = torch.relu(torch.randn(*shape, device=cuda)).to(dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    pool, ref = MaxPool2dNHWC(k, s, p), nn.MaxPool2d(k, s, p)
    grads = []
    for _ in range(2):
        xa = x.clone().requires_grad_(True)
        ya = pool(xa)
        g = torch.randn_like(ya, dtype=torch.float32).to(dtype) if not grads else g
        ya.backward(g)
        grads.append(xa.grad)
    assert calls == ['bwd', 'bwd']
    assert torch.equal(grads[0], grads[1])
    xb = x.clone().requires_grad_(True)
    yb = ref(xb)
    yb.backward(g)
    assert torch.equal(ya, yb)
    assert ya.is_contiguous(memory_format=torch.channels_last)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(grads[0].float(), xb.grad.float(), rtol=tol, atol=tol)
