"""Scheduler, hyperparameter schedules and tracing (reference
tests/{scheduler,hyperparams,tracing}_test.py strategy)."""
from __future__ import annotations

import time

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd import tracing
from distributed_kfac_pytorch_amd.hyperparams import exp_decay_factor_averaging
from distributed_kfac_pytorch_amd.models.tiny import TinyModel
from distributed_kfac_pytorch_amd.scheduler import LambdaParamScheduler
from tests.harness import distributed_test


def test_exp_decay_values():
    f = exp_decay_factor_averaging()
    assert f(0) == 0.0 and f(1) == 0.0
    assert f(2) == 0.5
    assert f(4) == 0.75
    assert f(100) == 0.95
    g = exp_decay_factor_averaging(0.5)
    assert g(10) == 0.5
    vals = [f(k) for k in range(1, 50)]
    assert vals == sorted(vals)


def test_exp_decay_errors():
    with pytest.raises(ValueError):
        exp_decay_factor_averaging(0)
    with pytest.raises(ValueError):
        exp_decay_factor_averaging()(-1)


def test_scheduler_rejects_callables():
    p = kfac.KFACPreconditioner(TinyModel(), damping=lambda s: 0.1)
    with pytest.raises(ValueError):
        LambdaParamScheduler(p, damping_lambda=lambda s: 0.5)
    for name in ('factor_update_steps', 'inv_update_steps', 'factor_decay', 'kl_clip', 'lr'):
        p = kfac.KFACPreconditioner(TinyModel(), **{name: (lambda s: 1)})
        with pytest.raises(ValueError):
            LambdaParamScheduler(p, **{f'{name}_lambda': lambda s: 2})


def test_scheduler_compounds():
    p = kfac.KFACPreconditioner(
        TinyModel(), factor_update_steps=1, inv_update_steps=3, damping=1.0,
        factor_decay=0.5, kl_clip=1.0, lr=1.0,
    )
    s = LambdaParamScheduler(
        p,
        factor_update_steps_lambda=lambda k: 2,
        inv_update_steps_lambda=lambda k: 1.5,
        damping_lambda=lambda k: 2,
        factor_decay_lambda=lambda k: 1,
        kl_clip_lambda=lambda k: 0.5,
        lr_lambda=lambda k: 3,
    )
    for i in range(1, 4):
        s.step()
        assert p.factor_update_steps == 2 ** i
        assert p.damping == 2 ** i
        assert p.kl_clip == 0.5 ** i
        assert p.lr == 3 ** i
        assert p.factor_decay == 0.5
    assert p.inv_update_steps == int(int(int(3 * 1.5) * 1.5) * 1.5)


def test_scheduler_step_override():
    p = kfac.KFACPreconditioner(TinyModel(), damping=1.0)
    seen = []
    s = LambdaParamScheduler(p, damping_lambda=lambda k: seen.append(k) or 1.0)
    s.step()
    s.step(step=7)
    assert seen == [0, 7]


def test_trace_average_sum_history():
    tracing.clear_trace()

    @tracing.trace()
    def f(t):
        time.sleep(t)

    f(0.01)
    f(0.03)
    avg = tracing.get_trace()['f']
    tot = tracing.get_trace(average=False)['f']
    assert 0.015 < avg < 0.1 and tot == pytest.approx(2 * avg)
    last = tracing.get_trace(max_history=1)['f']
    assert last >= 0.025
    tracing.log_trace()
    tracing.clear_trace()
    assert tracing.get_trace() == {}


@distributed_test(2)
def _trace_sync():
    tracing.clear_trace()

    @tracing.trace(sync=True)
    def g():
        return 5

    assert g() == 5
    assert 'g' in tracing.get_trace()


def test_trace_sync():
    _trace_sync()


def test_phase_timer_cpu():
    t = tracing.PhaseTimer()
    with t.phase('a'):
        time.sleep(0.002)
    with t.phase('a'):
        pass
    s = t.summary()
    assert s['a'] > 1.0
    assert t.counts() == {'a': 2}
    assert t.summary(average=True)['a'] == pytest.approx(s['a'] / 2)
    t.reset()
    assert t.summary() == {}


def test_global_phase_timing_in_step():
    timer = tracing.enable_phase_timing(True)
    try:
        model = TinyModel()
        p = kfac.KFACPreconditioner(model)
        out = model(torch.randn(4, 10))
        out.sum().backward()
        p.step()
        names = set(timer.summary())
        assert {'factor_a', 'factor_g', 'inverse', 'precondition', 'apply'} <= names
    finally:
        tracing.enable_phase_timing(False)
    assert tracing.phase_timer() is None
