"""Fused autocast weight casts (ops/cast.py, csrc/cast.hip): same forward
and the same fp32 parameter gradients as autocast's per-tensor casts."""
from __future__ import annotations

import pytest
import torch
from torch import nn

from distributed_kfac_pytorch_amd.ops import cast as cast_ops
from distributed_kfac_pytorch_amd.ops import _native


def _net() -> nn.Module:
    torch.manual_seed(0)
    return nn.Sequential(
        nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.ReLU(),
        nn.Conv2d(16, 24, 3, stride=2, padding=1), nn.ReLU(),
        nn.Flatten(), nn.Linear(24 * 4 * 4, 10),
    )


def _run(model: nn.Module, x: torch.Tensor, dev: str) -> tuple[torch.Tensor, list]:
    model.zero_grad(set_to_none=True)
    with torch.autocast(dev, dtype=torch.bfloat16):
        out = model(x)
    out.float().square().sum().backward()
    return out.detach().float(), [p.grad.clone() for p in model.parameters()]


def _check(dev: str, group_mb: float, channels_last: bool) -> None:
    x = torch.randn(4, 3, 8, 8, device=dev)
    ref = _net().to(dev)
    fused = _net().to(dev)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
        ref = ref.to(memory_format=torch.channels_last)
        fused = fused.to(memory_format=torch.channels_last)
    h = cast_ops.enable_fused_weight_cast(fused, group_mb=group_mb, device_type=dev)
    o1, g1 = _run(ref, x, dev)
    o2, g2 = _run(fused, x, dev)
    assert torch.equal(o1, o2)
    for a, b in zip(g1, g2):
        assert b.dtype == torch.float32 and b.shape == a.shape
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    # the hooks really ran the fused path: its groups cover every weight
    assert sum(len(g) for g in h.groups) == 5
    h.remove()
    o3, g3 = _run(fused, x, dev)
    assert torch.equal(o1, o3)


@pytest.mark.parametrize('group_mb', [25.0, 0.001])
def test_fused_cast_matches_autocast_cpu(group_mb: float) -> None:
    _check('cpu', group_mb, channels_last=False)


def test_fused_cast_groups_follow_backward_order() -> None:
    net = _net()
    h = cast_ops.enable_fused_weight_cast(net, group_mb=0.001, device_type='cpu')
    names = [n for g in h.groups for _, n in g]
    assert names[:2] == ['weight', 'bias']  # the Linear (last module) first
    assert h.groups[0][0][0] is net[5]
    h.remove()


def test_fused_cast_stale_copies_never_used() -> None:
    """A forward that raises leaves its bf16 copies behind; later forwards
    (inside or outside autocast) must not use them."""
    net = _net()
    h = cast_ops.enable_fused_weight_cast(net, device_type='cpu')
    x = torch.randn(2, 3, 8, 8)
    with pytest.raises(RuntimeError):
        with torch.autocast('cpu', dtype=torch.bfloat16):
            net(x[:, :2])  # wrong channel count: the first conv raises
    assert '_fused_cast' in net[0].__dict__  # left behind by the failed forward
    with torch.no_grad():
        net[0].weight.add_(1.0)  # an optimizer update after the failure
    out = net(x)  # outside autocast: plain fp32 forward
    assert out.dtype == torch.float32
    ref = nn.Sequential(*[m for m in _net()])
    ref.load_state_dict(net.state_dict())
    torch.testing.assert_close(out, ref(x))
    with torch.autocast('cpu', dtype=torch.bfloat16):
        o2 = net(x)
        o3 = ref(x)
    assert torch.equal(o2.float(), o3.float())
    h.remove()


@pytest.mark.gpu
@pytest.mark.parametrize('channels_last', [False, True])
@pytest.mark.parametrize('group_mb', [25.0, 0.001])
def test_fused_cast_matches_autocast_gpu(channels_last: bool, group_mb: float) -> None:
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    assert _native.native() is not None, 'native extension must be loaded on a GPU box'
    _check('cuda', group_mb, channels_last)


@pytest.mark.gpu
def test_cast_multi_kernel_gpu() -> None:
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    lib = _native.native()
    assert lib is not None
    torch.manual_seed(1)
    srcs = [torch.randn(n, device='cuda') * 100 for n in (1, 7, 8, 1000, 4097)]
    srcs.append(torch.tensor([float('inf'), -float('inf'), 0.0, -0.0, 1e-40], device='cuda'))
    outs = cast_ops._caster().cast(srcs, torch.bfloat16)
    for s, o in zip(srcs, outs):
        assert torch.equal(o, s.to(torch.bfloat16))
    back = cast_ops._caster().cast(outs, torch.float32)
    for o, b in zip(outs, back):
        assert torch.equal(b, o.float())
