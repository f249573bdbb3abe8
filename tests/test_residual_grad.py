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


def _block(proj: int = 0) -> torch.nn.Module:
    """Identity shortcut (proj 0: 64 -> 16 * 4), or a projection of stride
    ``proj`` (64 -> 32 * 4, the torchvision downsample layout)."""
    torch.manual_seed(0)
    if proj:
        from distributed_kfac_pytorch_amd.ops.bnact import BatchNormAct2d

        ds = torch.nn.Sequential(cops.StridedConv1x1(64, 128, 1, stride=proj, bias=False)
                                 if proj > 1 else torch.nn.Conv2d(64, 128, 1, bias=False),
                                 BatchNormAct2d(128))
        b = Bottleneck(64, 32, stride=proj, downsample=ds)
    else:
        b = Bottleneck(64, 16)
    cops.use_gemm_conv1x1(b)
    return b.to(memory_format=torch.channels_last)


def _grads(block: torch.nn.Module, x: torch.Tensor) -> list[torch.Tensor]:
    xa = x.clone().requires_grad_(True)
    y = block(xa)
    y.backward(torch.ones_like(y) * 0.1 + y.detach() * 0.01)
    return [xa.grad] + [p.grad for p in block.parameters()]


@pytest.mark.parametrize('fuse', ['1', '0'])
@pytest.mark.parametrize('proj', [0, 1, 2])
def test_fused_shortcut_gradient_matches(monkeypatch, fuse, proj):
    x = torch.randn(2, 64, 6, 6).contiguous(memory_format=torch.channels_last)
    base = _block(proj)
    monkeypatch.setenv('KFAC_RESIDUAL_GRAD_FUSE', '0')
    ref = _grads(copy.deepcopy(base), x)
    monkeypatch.setenv('KFAC_RESIDUAL_GRAD_FUSE', fuse)
    seen: list = []
    orig = cops._mm_nn

    def spy(g, w, addend=None):  # type: ignore[no-untyped-def]
        seen.append(addend is not None)
        return orig(g, w, addend)
    monkeypatch.setattr(cops, '_mm_nn', spy)
    handed: list = []

    class Rec(cops.ResidualGradSlot):
        __slots__ = ()

        def __setattr__(self, k, v):  # type: ignore[no-untyped-def]
            if k == 'g' and v is not None:
                handed.append(v.dim())
            super().__setattr__(k, v)
    from distributed_kfac_pytorch_amd.models import resnet as rmod
    monkeypatch.setattr(rmod, 'ResidualGradSlot', Rec)
    got = _grads(copy.deepcopy(base), x)
    # a gradient went through the slot exactly when fusing: the tap's 4-D
    # gradient (identity) or conv1's parked 2-D input gradient (projection)
    assert handed == ([] if fuse == '0' else [4 if proj == 0 else 2]), handed
    # identity: conv1's input gradient carries the shortcut's; stride-1
    # projection: the shortcut conv's carries conv1's; stride 2: the
    # subsample adjoint accumulates (no GEMM addend)
    n_add = 1 if fuse == '1' and proj in (0, 1) else 0
    assert sum(seen) == n_add, seen
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
@pytest.mark.parametrize('proj', [0, 1, 2])
def test_fused_shortcut_gradient_gpu(cuda, monkeypatch, proj):
    """On the GPU the shortcut's gradient is added in the native bf16x3
    GEMM's epilogue (csrc/gemm3.hip GemmDesc::D), in place; a strided
    projection's adjoint accumulates into conv1's gradient
    (csrc/subsample.hip subsample_bwd_acc)."""
    from distributed_kfac_pytorch_amd.ops._native import native
    from distributed_kfac_pytorch_amd.ops.bnact import BatchNormAct2d

    assert native() is not None
    torch.manual_seed(0)
    if proj:
        ds = torch.nn.Sequential(cops.StridedConv1x1(256, 512, 1, stride=proj, bias=False)
                                 if proj > 1 else torch.nn.Conv2d(256, 512, 1, bias=False),
                                 BatchNormAct2d(512))
        base = Bottleneck(256, 128, stride=proj, downsample=ds)
    else:
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
