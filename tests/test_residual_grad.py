"""Identity-shortcut gradient fused into the block's first 1x1 convolution
(ops/conv.py ResidualGradSlot): the same gradients as autograd's sum, in
either backward order, on CPU (addmm) -- the GPU epilogue path is covered by
tests/test_conv.py-style GPU runs of the models."""
from __future__ import annotations

import copy

import pytest
import torch

from distributed_kfac_pytorch_amd.models.resnet import Bottleneck
from distributed_kfac_pytorch_amd.ops import conv as cops


def _block() -> torch.nn.Module:
    torch.manual_seed(0)
    b = Bottleneck(64, 16)  # identity shortcut (64 -> 16 * 4)
    cops.use_gemm_conv1x1(b)
    return b.to(memory_format=torch.channels_last)


def _grads(block: torch.nn.Module, x: torch.Tensor) -> list[torch.Tensor]:
    xa = x.clone().requires_grad_(True)
    y = block(xa)
    y.backward(torch.ones_like(y) * 0.1 + y.detach() * 0.01)
    return [xa.grad] + [p.grad for p in block.parameters()]


@pytest.mark.parametrize('fuse', ['1', '0'])
def test_fused_shortcut_gradient_matches(monkeypatch, fuse):
    x = torch.randn(2, 64, 6, 6).contiguous(memory_format=torch.channels_last)
    base = _block()
    monkeypatch.setenv('KFAC_RESIDUAL_GRAD_FUSE', '0')
    ref = _grads(copy.deepcopy(base), x)
    monkeypatch.setenv('KFAC_RESIDUAL_GRAD_FUSE', fuse)
    seen: list = []
    orig = cops._mm_nn

    def spy(g, w, addend=None):  # type: ignore[no-untyped-def]
        seen.append(addend is not None)
        return orig(g, w, addend)
    monkeypatch.setattr(cops, '_mm_nn', spy)
    got = _grads(copy.deepcopy(base), x)
    # conv1 and conv3 input gradients; conv1's carries the shortcut's
    assert sorted(seen) == ([False, True] if fuse == '1' else [False, False]), seen
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_slot_is_order_independent():
    """The convolution's backward running before the tap's: the tap hands
    its gradient back to autograd (``done``), nothing is lost."""
    slot = cops.ResidualGradSlot()
    x = torch.randn(3, 4, requires_grad=True)
    t = cops.residual_tap(x, slot)
    slot.done = True  # as if conv1's backward had already run
    t.sum().backward()
    torch.testing.assert_close(x.grad, torch.ones(3, 4))
    slot2 = cops.ResidualGradSlot()
    x2 = torch.randn(3, 4, requires_grad=True)
    (cops.residual_tap(x2, slot2) * 2).sum().backward()
    assert x2.grad is None and torch.equal(slot2.g, torch.full((3, 4), 2.0))


def test_block_arms_only_fusable_convs(monkeypatch):
    """A plain nn.Conv2d conv1 (not converted) never takes the slot."""
    torch.manual_seed(0)
    b = Bottleneck(64, 16).to(memory_format=torch.channels_last)
    x = torch.randn(2, 64, 6, 6).contiguous(memory_format=torch.channels_last).requires_grad_()
    b(x).sum().backward()
    assert x.grad is not None and '_dgrad_slot' not in b.conv1.__dict__


@pytest.mark.gpu
def test_fused_shortcut_gradient_gpu(cuda, monkeypatch):
    """On the GPU the shortcut's gradient is added in the native bf16x3
    GEMM's epilogue (csrc/gemm3.hip GemmDesc::D), in place."""
    from distributed_kfac_pytorch_amd.ops._native import native

    assert native() is not None
    torch.manual_seed(0)
    base = Bottleneck(256, 64)
    cops.use_gemm_conv1x1(base)
    cops.use_implicit_gemm_conv(base)
    base = base.to(cuda).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, 28, 28, device=cuda).contiguous(memory_format=torch.channels_last)
    runs = {}
    for fuse in ('0', '1'):
        monkeypatch.setenv('KFAC_RESIDUAL_GRAD_FUSE', fuse)
        runs[fuse] = _grads(copy.deepcopy(base), x)
    for a, b in zip(runs['1'], runs['0']):
        scale = b.abs().max().item()
        assert (a - b).abs().max().item() <= 1e-5 * scale + 1e-7, ((a - b).abs().max(), scale)
