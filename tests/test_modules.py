"""Module helpers, registration and factor utilities (reference
tests/layers/{modules,register,utils}_test.py strategy)."""
from __future__ import annotations

import pytest
import torch

from distributed_kfac_pytorch_amd.layers import register
from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.modules import Conv2dModuleHelper
from distributed_kfac_pytorch_amd.layers.modules import LinearModuleHelper
from distributed_kfac_pytorch_amd.layers.utils import append_bias_ones
from distributed_kfac_pytorch_amd.layers.utils import get_cov
from distributed_kfac_pytorch_amd.layers.utils import reshape_data
from distributed_kfac_pytorch_amd.models.tiny import LeNet
from distributed_kfac_pytorch_amd.models.tiny import TinyModel
from distributed_kfac_pytorch_amd.ops import factors as fops
from distributed_kfac_pytorch_amd.parallel.comm import TorchDistributedCommunicator


# ------------------------------------------------------------------- utils
def test_append_bias_ones():
    x = torch.randn(4, 6)
    y = append_bias_ones(x)
    assert y.shape == (4, 7)
    assert torch.equal(y[:, :6], x) and torch.equal(y[:, 6], torch.ones(4))
    z = append_bias_ones(torch.randn(2, 3, 5))
    assert z.shape == (2, 3, 6)


def test_get_cov_exact():
    a = torch.tensor([[1.0, 2.0], [3.0, 4.0]])
    # a^T a / 2 = [[10, 14], [14, 20]] / 2
    assert torch.equal(get_cov(a), torch.tensor([[5.0, 7.0], [7.0, 10.0]]))
    assert torch.equal(get_cov(a, scale=1), torch.tensor([[10.0, 14.0], [14.0, 20.0]]))
    b = torch.tensor([[1.0, 0.0], [0.0, 1.0]])
    assert torch.equal(get_cov(a, b), torch.tensor([[0.5, 1.5], [1.0, 2.0]]))
    with pytest.raises(ValueError):
        get_cov(torch.ones(3))
    with pytest.raises(ValueError):
        get_cov(torch.ones(2, 2), torch.ones(3, 2))


def test_reshape_data():
    d = reshape_data([torch.ones(2, 3, 4), torch.ones(5, 3, 4)])
    assert d.shape == (7, 3, 4)
    d = reshape_data([torch.ones(2, 3, 4)] * 2, batch_first=False, collapse_dims=True)
    assert d.shape == (2 * 6, 4)


@pytest.mark.parametrize('bias', [False, True])
def test_cov_accumulate_cpu(bias):
    x = torch.randn(50, 7, dtype=torch.float64)
    out = torch.randn(7 + bias, 7 + bias, dtype=torch.float64)
    c0 = out.clone()
    fops.cov_accumulate_(out, x, bias=bias, alpha=0.3, beta=0.5)
    xb = append_bias_ones(x) if bias else x
    assert torch.allclose(out, 0.5 * c0 + 0.3 * xb.t() @ xb)


# ----------------------------------------------------------------- helpers
def test_linear_helper():
    m = torch.nn.Linear(5, 3)
    h = LinearModuleHelper(m)
    assert h.a_factor_shape == (6, 6)
    assert h.g_factor_shape == (3, 3)
    assert h.has_bias() and h.has_symmetric_factors()
    x = torch.randn(4, 2, 5)
    a = h.get_a_factor(x)
    xb = append_bias_ones(x.reshape(-1, 5))
    assert torch.allclose(a, xb.t() @ xb / 8)
    g = torch.randn(4, 2, 3)
    assert torch.allclose(h.get_g_factor(g), g.reshape(-1, 3).t() @ g.reshape(-1, 3) / 8)
    m(x).sum().backward()
    grad = h.get_grad()
    assert grad.shape == (3, 6)
    assert torch.equal(grad[:, :5], m.weight.grad) and torch.equal(grad[:, 5], m.bias.grad)
    new = torch.randn(3, 6)
    h.set_grad(new)
    assert torch.equal(m.weight.grad, new[:, :5]) and torch.equal(m.bias.grad, new[:, 5])
    newer = torch.randn(3, 6)
    h.write_grad(newer, 2.0)
    assert torch.allclose(m.weight.grad, 2 * newer[:, :5])
    assert torch.allclose(m.bias.grad, 2 * newer[:, 5])


def test_accumulate_matches_get():
    m = torch.nn.Linear(5, 3)
    h = LinearModuleHelper(m)
    x = torch.randn(6, 5)
    out = torch.zeros(6, 6)
    h.accumulate_a_factor(x, out, 1.0, 0.0)
    assert torch.allclose(out, h.get_a_factor(x), atol=1e-6)


@pytest.mark.parametrize('bias', [False, True])
@pytest.mark.parametrize('stride,pad', [(1, 0), (2, 1), (1, 2)])
def test_conv_helper_matches_unfold(bias, stride, pad):
    m = torch.nn.Conv2d(3, 4, 3, stride=stride, padding=pad, bias=bias)
    h = Conv2dModuleHelper(m)
    assert h.a_factor_shape == (27 + bias, 27 + bias)
    assert h.g_factor_shape == (4, 4)
    x = torch.randn(2, 3, 9, 8)
    a = h.get_a_factor(x)
    cols = torch.nn.functional.unfold(x, 3, padding=pad, stride=stride)  # [B, C*9, L]
    spatial = cols.shape[-1]
    p = cols.transpose(1, 2).reshape(-1, 27)
    if bias:
        p = append_bias_ones(p)
    p = p / spatial
    assert torch.allclose(a, p.t() @ p / p.shape[0], atol=1e-6)
    y = m(x)
    g = torch.randn_like(y)
    gf = h.get_g_factor(g)
    rows = g.permute(0, 2, 3, 1).reshape(-1, 4) / (y.shape[2] * y.shape[3])
    assert torch.allclose(gf, rows.t() @ rows / rows.shape[0], atol=1e-6)
    y.backward(g)
    assert h.get_grad().shape == (4, 27 + bias)


def test_conv_natural_order_equivalence():
    torch.manual_seed(0)
    m_ref = torch.nn.Conv2d(4, 5, 3, padding=1, bias=True)
    m_nat = torch.nn.Conv2d(4, 5, 3, padding=1, bias=True)
    m_nat.load_state_dict(m_ref.state_dict())
    m_nat = m_nat.to(memory_format=torch.channels_last)
    h_ref, h_nat = Conv2dModuleHelper(m_ref), Conv2dModuleHelper(m_nat)
    assert not h_ref.natural_order and h_nat.natural_order
    x = torch.randn(2, 4, 6, 6)
    a_ref = h_ref.get_a_factor(x)
    a_nat = h_nat.get_a_factor(x.contiguous(memory_format=torch.channels_last))
    assert torch.allclose(h_nat.a_to_reference_order(a_nat), a_ref, atol=1e-6)
    assert torch.allclose(h_nat.a_from_reference_order(a_ref), a_nat, atol=1e-6)
    for mod in (m_ref, m_nat):
        mod(x).sum().backward()
    # gradient views describe the same matrix up to the same column permutation
    g_ref = h_ref.get_grad()
    g_nat = h_nat.get_grad()
    perm = h_nat._perm(torch.device('cpu'))
    assert torch.allclose(g_nat[:, perm], g_ref)
    # write_grad in natural order lands in the right weight entries
    p = torch.randn(5, 37)
    h_nat.write_grad(p, None)
    h_ref.write_grad(p[:, perm], None)
    assert torch.allclose(m_nat.weight.grad, m_ref.weight.grad)
    assert torch.allclose(m_nat.bias.grad, m_ref.bias.grad)


def test_conv_unsupported_configs_are_skipped():
    model = torch.nn.Sequential(
        torch.nn.Conv2d(4, 4, 3, groups=2),
        torch.nn.Conv2d(4, 4, 3, dilation=2),
        torch.nn.Conv2d(4, 4, 3),
    )
    with pytest.warns(UserWarning):
        layers = register.register_modules(
            model, KFACEigenLayer, [], tdc=TorchDistributedCommunicator(),
        )
    assert [n for n, _ in layers.values()] == ['2']


# ---------------------------------------------------------------- register
class NestedTinyModel(torch.nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.tiny = TinyModel()
        self.extra = torch.nn.Linear(10, 10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.extra(self.tiny(x))


def test_flattened_modules_names():
    names = [n for n, _ in register.get_flattened_modules(NestedTinyModel())]
    assert names == [
        'tiny.linear1', 'tiny.activation', 'tiny.linear2', 'tiny.softmax', 'extra',
    ]


def test_requires_grad():
    m = torch.nn.Linear(2, 2)
    assert register.requires_grad(m)
    m.bias.requires_grad = False
    assert not register.requires_grad(m)


def test_get_module_helper_dispatch():
    assert isinstance(register.get_module_helper(torch.nn.Linear(2, 2)), LinearModuleHelper)
    assert isinstance(register.get_module_helper(torch.nn.Conv2d(2, 2, 1)), Conv2dModuleHelper)
    assert register.get_module_helper(torch.nn.Conv3d(2, 2, 1)) is None
    assert register.get_module_helper(torch.nn.ReLU()) is None


@pytest.mark.parametrize(
    'skip,expected',
    [
        ([], 5),
        (['conv'], 3),
        (['Conv2d'], 3),
        (['fc1'], 4),
        (['fc'], 2),
        (['Linear', 'conv1'], 1),
        (['^conv2$'], 4),
    ],
)
def test_register_counts(skip, expected):
    layers = register.register_modules(
        LeNet(), KFACEigenLayer, skip, tdc=TorchDistributedCommunicator(),
    )
    assert len(layers) == expected


def test_any_match():
    assert register.any_match('layer1.conv', ['conv'])
    assert not register.any_match('layer1.conv', ['Conv'])
    assert register.any_match('abc', ['^a', 'zzz'])
    assert not register.any_match('abc', [])
