"""Numerical parity with the reference, pinned by golden fixtures.

``tests/data/ref_fixtures.pt`` was produced once by running the upstream
``kfac_pytorch`` 0.4.1 package on the CPU (``tools/make_ref_fixtures.py``):
a small conv net (conv with bias, conv without bias, linear) trained for 4
steps with every compute method x eigenvalue-outer-product combination.
This framework must reproduce, at fp32 precision, the preconditioned
gradients of every step, the checkpoint factors (in the reference's column
order) and the checkpoint keys -- including the ``module.`` prefix under
DDP.  Reference semantics: ``kfac/base_preconditioner.py:213-380``,
``kfac/layers/base.py:129-164``.  Loaded with ``weights_only=True``.
"""
from __future__ import annotations

import os

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from tests.harness import run_distributed

FIXTURES = os.path.join(os.path.dirname(__file__), 'data', 'ref_fixtures.pt')


def _fixtures() -> dict:
    return torch.load(FIXTURES, weights_only=True)


def _make_model() -> torch.nn.Module:
    torch.manual_seed(0)
    return torch.nn.Sequential(
        torch.nn.Conv2d(3, 8, 3, padding=1, stride=2),
        torch.nn.ReLU(),
        torch.nn.Conv2d(8, 8, 3, bias=False),
        torch.nn.Flatten(),
        torch.nn.Linear(8 * 5 * 5, 10),
    )


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.double() - b.double()).abs().max()) / max(float(b.double().abs().max()), 1e-30)


@pytest.mark.parametrize('run', ['eigen-prediv1', 'eigen-prediv0', 'inverse-prediv1',
                                 'inverse-prediv0'])
def test_matches_reference_fixtures(run):
    fx = _fixtures()
    ref = fx['runs'][run]
    method, prediv = run.split('-')
    model = _make_model()
    pre = kfac.KFACPreconditioner(
        model, compute_method=method, compute_eigenvalue_outer_product=prediv.endswith('1'),
        **fx['kwargs'],
    )
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for step, (x, y, grads) in enumerate(zip(ref['x'], ref['y'], ref['grads'])):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
        for p, g in zip(model.parameters(), grads):
            assert _rel(p.grad, g) < 1e-5, (run, step, _rel(p.grad, g))
        opt.step()
    sd = pre.state_dict()
    assert sorted(sd.keys()) == ref['state_keys']
    assert sorted(sd['layers']) == sorted(ref['factors'])
    for name, f in ref['factors'].items():
        assert _rel(sd['layers'][name]['A'], f['A']) < 1e-6, (name, "A")
        assert _rel(sd['layers'][name]['G'], f['G']) < 1e-6, (name, "G")


def _ddp_keys(expected: list) -> None:
    model = torch.nn.parallel.DistributedDataParallel(_make_model())
    pre = kfac.KFACPreconditioner(model, **_fixtures()['kwargs'])
    torch.nn.functional.cross_entropy(
        model(torch.randn(4, 3, 14, 14)), torch.zeros(4, dtype=torch.long)).backward()
    pre.step()
    assert sorted(pre.state_dict()['layers']) == expected


def test_ddp_checkpoint_keys_match_reference():
    run_distributed(_ddp_keys, 1, _fixtures()['ddp_layer_keys'])
