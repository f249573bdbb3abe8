"""GraphedTrainStep: whole-step HIP graph replay must train exactly like the
eager loop (same K-FAC schedule, same parameters), and fall back to eager
execution where graphs do not apply."""
from __future__ import annotations

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep


def _setup(device: torch.device, seed: int = 0):
    torch.manual_seed(seed)
    model = torch.nn.Sequential(
        torch.nn.Conv2d(3, 16, 3, padding=1),
        torch.nn.ReLU(),
        torch.nn.Conv2d(16, 16, 3, stride=2, padding=1, bias=False),
        torch.nn.ReLU(),
        torch.nn.Flatten(),
        torch.nn.Linear(16 * 8 * 8, 10),
    ).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    pre = kfac.KFACPreconditioner(
        model, factor_update_steps=2, inv_update_steps=6, damping=0.01,
        lr=lambda s: opt.param_groups[0]['lr'],
    )
    x = torch.randn(8, 3, 16, 16, device=device)
    y = torch.randint(0, 10, (8,), device=device)

    def fb() -> torch.Tensor:
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        return loss

    return model, opt, pre, fb


def test_runner_eager_when_disabled() -> None:
    model, opt, pre, fb = _setup(torch.device('cpu'))
    runner = GraphedTrainStep(fb, opt, pre, enabled=False)
    ref_model, ref_opt, ref_pre, ref_fb = _setup(torch.device('cpu'))
    for _ in range(7):
        runner()
        ref_opt.zero_grad(set_to_none=False)
        ref_fb()
        ref_pre.step()
        ref_opt.step()
    assert runner.replays == 0 and runner.eager_steps == 7
    assert pre.steps == ref_pre.steps == 7
    for a, b in zip(model.parameters(), ref_model.parameters()):
        torch.testing.assert_close(a, b)


def test_step_kinds() -> None:
    _, opt, pre, fb = _setup(torch.device('cpu'))
    runner = GraphedTrainStep(fb, opt, pre, enabled=False)
    kinds = []
    for _ in range(7):
        kinds.append(runner.kind())
        runner()
    assert kinds == ['inverse', 'plain', 'factor', 'plain', 'factor', 'plain', 'inverse']
    assert runner._next_step_of('factor') == 8
    assert runner._next_step_of('plain') == 7


def _train_eager(device: torch.device, steps: int):
    model, opt, pre, fb = _setup(device)
    losses = []
    for _ in range(steps):
        opt.zero_grad(set_to_none=False)
        losses.append(float(fb()))
        pre.step()
        opt.step()
    return model, pre, losses


def _max_diff(ma, pa, mb, pb) -> tuple[float, float]:
    dp = max(float((a - b).abs().max()) for a, b in zip(ma.parameters(), mb.parameters()))
    df = max(
        max(float((la.a_factor - lb.a_factor).abs().max()),
            float((la.g_factor - lb.g_factor).abs().max()))
        for (_, la), (_, lb) in zip(pa._layers.values(), pb._layers.values())
    )
    return dp, df


@pytest.mark.gpu
def test_graph_replay_matches_eager(cuda) -> None:
    steps = 14
    model, opt, pre, fb = _setup(cuda)
    runner = GraphedTrainStep(fb, opt, pre)
    losses = [float(runner()) for _ in range(steps)]
    torch.cuda.synchronize()
    assert runner.captures == 2, runner.captures
    assert runner.replays >= 8, runner.replays
    assert pre.steps == steps
    # two eager runs give the run-to-run noise floor (split-K SYRK uses
    # float atomics, so factors are not bitwise reproducible)
    ma, pa, la = _train_eager(cuda, steps)
    mb, pb, lb = _train_eager(cuda, steps)
    assert pa.steps == steps
    for a, b in zip(losses, la):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (losses, la)
    noise_p, noise_f = _max_diff(ma, pa, mb, pb)
    dp, df = _max_diff(model, pre, ma, pa)
    assert dp <= 20 * noise_p + 1e-5, (dp, noise_p)
    assert df <= 20 * noise_f + 1e-6, (df, noise_f)
