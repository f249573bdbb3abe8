"""Preconditioner API, runtime and checkpoint behaviour (reference
tests/{preconditioner,base_preconditioner}_test.py strategy)."""
from __future__ import annotations

import logging
import warnings

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.base_preconditioner import BaseKFACPreconditioner
from distributed_kfac_pytorch_amd.enums import ComputeMethod
from distributed_kfac_pytorch_amd.enums import DistributedStrategy
from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.inverse import KFACInverseLayer
from distributed_kfac_pytorch_amd.layers.register import register_modules
from distributed_kfac_pytorch_amd.models.tiny import LeNet
from distributed_kfac_pytorch_amd.models.tiny import TinyModel
from distributed_kfac_pytorch_amd.parallel.comm import TorchDistributedCommunicator
from distributed_kfac_pytorch_amd.preconditioner import resolve_grad_worker_fraction
from tests.fakes import LazyAssignment
from tests.harness import distributed_test


def _base(model, layer_type=KFACEigenLayer, broadcast=False, **kw):
    tdc = TorchDistributedCommunicator()
    layers = register_modules(model, layer_type, [], tdc=tdc)
    return BaseKFACPreconditioner(
        layers, assignment=LazyAssignment(broadcast=broadcast), tdc=tdc, **kw,
    )


# ---------------------------------------------------------------- validation
@pytest.mark.parametrize(
    'kw',
    [
        dict(factor_update_steps=0),
        dict(inv_update_steps=-1),
        dict(damping=0.0),
        dict(factor_decay=0.0),
        dict(factor_decay=1.1),
        dict(kl_clip=0.0),
        dict(lr=-1.0),
        dict(accumulation_steps=0),
    ],
)
def test_base_validation(kw):
    with pytest.raises(ValueError):
        _base(TinyModel(), **kw)


def test_base_warns_on_non_multiple_steps():
    with pytest.warns(UserWarning):
        _base(TinyModel(), factor_update_steps=3, inv_update_steps=10)


def test_callable_hyperparameters():
    p = _base(
        TinyModel(),
        factor_update_steps=lambda s: 2,
        inv_update_steps=lambda s: 4,
        damping=lambda s: 0.1 * (s + 1),
        factor_decay=lambda s: 0.5,
        kl_clip=lambda s: 0.01,
        lr=lambda s: 0.2,
    )
    assert p.factor_update_steps == 2 and p.inv_update_steps == 4
    assert p.damping == pytest.approx(0.1)
    p._steps = 4
    assert p.damping == pytest.approx(0.5)
    assert p.factor_decay == 0.5 and p.kl_clip == 0.01 and p.lr == 0.2
    sd = p.state_dict()
    for k in ('factor_update_steps', 'inv_update_steps', 'damping', 'factor_decay', 'kl_clip', 'lr'):
        assert k not in sd


def test_repr_sorted():
    p = kfac.KFACPreconditioner(TinyModel())
    lines = [ln.strip() for ln in repr(p).splitlines()[1:-1]]
    keys = [ln.split('=')[0] for ln in lines]
    assert keys == sorted(keys)
    assert 'compute_method=ComputeMethod.EIGEN,' in lines


def _train(model, precond, steps=3, accumulation=1, x_shape=(8, 10), classes=10, eval_mode=False):
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    torch.manual_seed(0)
    for _ in range(steps):
        opt.zero_grad()
        for _ in range(accumulation):
            x = torch.randn(*x_shape)
            y = torch.randint(0, classes, (x_shape[0],))
            out = model(x)
            torch.nn.functional.cross_entropy(out, y).backward()
        precond.step()
        opt.step()


@pytest.mark.parametrize('layer_type', [KFACEigenLayer, KFACInverseLayer])
@pytest.mark.parametrize(
    'kw',
    [
        dict(accumulation_steps=1, update_factors_in_hook=True),
        dict(accumulation_steps=3, update_factors_in_hook=True),
        dict(accumulation_steps=2, update_factors_in_hook=False),
    ],
)
def test_base_e2e(layer_type, kw):
    model = LeNet()
    p = _base(model, layer_type=layer_type, factor_update_steps=1, inv_update_steps=2, **kw)
    grads_before = None
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    x = torch.randn(4, 1, 28, 28)
    y = torch.randint(0, 10, (4,))
    for step in range(3):
        opt.zero_grad()
        for _ in range(kw['accumulation_steps']):
            torch.nn.functional.cross_entropy(model(x), y).backward()
        grads_before = [q.grad.clone() for q in model.parameters()]
        p.step()
        changed = [not torch.equal(a, q.grad) for a, q in zip(grads_before, model.parameters())]
        assert all(changed)
        opt.step()
    assert p.steps == 3
    mem = p.memory_usage()
    assert mem['total'] == sum(v for k, v in mem.items() if k != 'total')
    assert mem['a_factors'] > 0 and mem['a_inverses'] > 0
    # state dict round trip recomputes inverses
    sd = p.state_dict()
    model2 = LeNet()
    p2 = _base(model2, layer_type=layer_type, factor_update_steps=1, inv_update_steps=2, **kw)
    p2.load_state_dict(sd, compute_inverses=True)
    assert p2.steps == 3
    for (_, l1), (_, l2) in zip(p._layers.values(), p2._layers.values()):
        assert torch.allclose(l1.a_factor, l2.a_factor)
        if layer_type is KFACEigenLayer:
            assert l2.qa is not None
        else:
            assert l2.a_inv is not None


def test_hooks_skipped_in_eval():
    model = TinyModel()
    p = _base(model)
    model.eval()
    model(torch.randn(2, 10)).sum().backward()
    for _, layer in p._layers.values():
        assert layer.a_factor is None and layer._a_batch is None
        assert layer.g_factor is None and layer._g_batch is None


def test_factor_update_steps_gate_hooks():
    model = TinyModel()
    p = _base(model, factor_update_steps=2, inv_update_steps=2)
    _train(model, p, steps=1)
    first = [l.a_factor.clone() for _, l in p._layers.values()]
    _train(model, p, steps=1)  # step 1: no factor update
    for f, (_, l) in zip(first, p._layers.values()):
        assert torch.equal(f, l.a_factor)


def test_state_dict_contents():
    model = TinyModel()
    p = kfac.KFACPreconditioner(model, lr=0.2, damping=0.01)
    sd = p.state_dict(include_factors=False)
    assert sd == {
        'steps': 0,
        'factor_update_steps': 1,
        'inv_update_steps': 1,
        'damping': 0.01,
        'factor_decay': 0.95,
        'kl_clip': 0.001,
        'lr': 0.2,
    }
    _train(model, p, steps=2)
    sd = p.state_dict()
    assert sorted(sd) == sorted(
        ['damping', 'factor_decay', 'factor_update_steps', 'inv_update_steps', 'kl_clip', 'layers', 'lr', 'steps'],
    )
    assert {k: (v['A'].shape, v['G'].shape) for k, v in sd['layers'].items()} == {
        'linear1': ((10, 10), (20, 20)),
        'linear2': ((21, 21), (10, 10)),
    }
    # not saved: accumulation / hook flags / defaults
    for k in ('accumulation_steps', 'update_factors_in_hook', 'defaults'):
        assert k not in sd
    p2 = kfac.KFACPreconditioner(TinyModel())
    with pytest.warns(UserWarning):
        p2.load_state_dict({'steps': 5})
    assert p2.steps == 5
    bad = dict(sd)
    bad['layers'] = {'linear1': sd['layers']['linear1']}
    with pytest.raises(ValueError):
        p2.load_state_dict(bad)


def test_kl_clip_none_and_empty():
    model = TinyModel()
    p = kfac.KFACPreconditioner(model, kl_clip=None)
    _train(model, p, steps=2)
    empty = _base(torch.nn.Sequential(torch.nn.ReLU()))
    assert empty._compute_grad_scale() == 1.0


def test_device_scale_matches_python_scale():
    model = TinyModel()
    p = kfac.KFACPreconditioner(model, lr=0.5, kl_clip=1e-4)
    x = torch.randn(8, 10)
    torch.nn.functional.cross_entropy(model(x), torch.randint(0, 10, (8,))).backward()
    ordered = list(reversed(list(p._layers.values())))
    p._compute_second_order(ordered)
    for _, layer in ordered:
        layer.preconditioned_grad(p.damping)
    ref = p._compute_grad_scale()
    dev = p._device_grad_scale(ordered, p.kl_clip)
    assert float(dev) == pytest.approx(ref, rel=1e-6)


# -------------------------------------------------------- KFACPreconditioner
def test_preconditioner_validation():
    with pytest.raises(ValueError):
        kfac.KFACPreconditioner(TinyModel(), allreduce_bucket_cap_mb=-1)
    with pytest.raises(ValueError):
        kfac.KFACPreconditioner(
            TinyModel(), compute_eigenvalue_outer_product=True, colocate_factors=False,
        )
    with pytest.raises(KeyError):
        kfac.KFACPreconditioner(TinyModel(), compute_method='nope')
    p = kfac.KFACPreconditioner(TinyModel(), compute_method='inverse',
                                assignment_strategy='memory')
    assert p.compute_method == ComputeMethod.INVERSE
    assert all(isinstance(l, KFACInverseLayer) for _, l in p._layers.values())
    p = kfac.KFACPreconditioner(TinyModel(), allreduce_bucket_cap_mb=0)
    assert p.allreduce_method == kfac.AllreduceMethod.ALLREDUCE


@pytest.mark.parametrize(
    'world,value,expected',
    [
        (1, DistributedStrategy.COMM_OPT, (1.0, DistributedStrategy.COMM_OPT)),
        (4, DistributedStrategy.MEM_OPT, (0.25, DistributedStrategy.MEM_OPT)),
        (4, DistributedStrategy.HYBRID_OPT, (0.5, DistributedStrategy.HYBRID_OPT)),
        (4, 0, (0.25, DistributedStrategy.MEM_OPT)),
        (4, 0.25, (0.25, DistributedStrategy.MEM_OPT)),
        (4, 0.5, (0.5, DistributedStrategy.HYBRID_OPT)),
        (4, 1, (1.0, DistributedStrategy.COMM_OPT)),
    ],
)
def test_grad_worker_fraction_mapping(world, value, expected):
    assert resolve_grad_worker_fraction(value, world) == expected


def test_grad_worker_fraction_invalid():
    with pytest.raises(ValueError):
        resolve_grad_worker_fraction(0.33, 8)
    with pytest.raises(ValueError):
        resolve_grad_worker_fraction(1.5, 8)


@distributed_test(4)
def _strategy_world4():
    for value, strat in (
        (DistributedStrategy.COMM_OPT, DistributedStrategy.COMM_OPT),
        (0.5, DistributedStrategy.HYBRID_OPT),
        (0.25, DistributedStrategy.MEM_OPT),
    ):
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            p = kfac.KFACPreconditioner(TinyModel(), grad_worker_fraction=value,
                                        colocate_factors=True)
        assert p.distributed_strategy == strat
    with pytest.warns(UserWarning):
        p = kfac.KFACPreconditioner(
            TinyModel(), grad_worker_fraction=DistributedStrategy.MEM_OPT,
            colocate_factors=False, compute_eigenvalue_outer_product=False,
        )
    assert p.colocate_factors


def test_strategy_world4():
    _strategy_world4()


def test_log_records(caplog):
    with caplog.at_level(logging.INFO):
        kfac.KFACPreconditioner(TinyModel(), loglevel=logging.INFO)
    msgs = [r.getMessage() for r in caplog.records]
    assert any('Registered name="linear1"' in m for m in msgs)
    assert any('KFAC layer assignments' in m for m in msgs)


def test_skip_layers():
    p = kfac.KFACPreconditioner(LeNet(), skip_layers=['conv'])
    assert [n for n, _ in p._layers.values()] == ['fc1', 'fc2', 'fc3']


def test_lazy_factor_join_decision(monkeypatch):
    """``step()`` leaves the G-factor SYRKs running only on single-process
    steps that do not refresh the second-order state
    (``BaseKFACPreconditioner._lazy_factor_join``; GPU behaviour in
    tests/test_factor_lazy_join_gpu.py)."""
    model = TinyModel()
    pre = kfac.KFACPreconditioner(model, factor_update_steps=2, inv_update_steps=4)
    monkeypatch.delenv('KFAC_FACTOR_JOIN', raising=False)
    pre._steps = 0  # inverse step: full join
    assert not pre._lazy_factor_join()
    pre._steps = 2  # factor step, no refresh
    assert pre._lazy_factor_join()
    monkeypatch.setenv('KFAC_FACTOR_JOIN', 'full')
    assert not pre._lazy_factor_join()
    monkeypatch.setenv('KFAC_FACTOR_JOIN', 'lazy')
    pre._accumulation_steps = 2
    assert not pre._lazy_factor_join()
