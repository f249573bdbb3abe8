"""GraphedTrainStep: whole-step HIP graph replay must train exactly like the
eager loop (same K-FAC schedule, same parameters), and fall back to eager
execution where graphs do not apply."""
from __future__ import annotations

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep
from distributed_kfac_pytorch_amd.graphs import verify_ratio
from distributed_kfac_pytorch_amd.graphs import verify_tolerance


def _setup(device: torch.device, seed: int = 0, method: str = 'eigen'):
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
        lr=lambda s: opt.param_groups[0]['lr'], compute_method=method,
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


def test_verify_tolerance() -> None:
    """The capture-time check's per-tensor tolerance: strict for a
    deterministic step, floored at the step's noise for a noisy one,
    capped so O(1) corruption never passes, NaN noise fails everything."""
    det = verify_tolerance(torch.zeros(5, dtype=torch.float64))
    assert torch.allclose(det, torch.full_like(det, 1e-3))
    # bf16 step: a tensor whose single eager pair agreed to 1e-4 may still
    # differ by the 4.6 % seen across replays and eager steps
    noisy = verify_tolerance(torch.tensor([1e-4, 0.02, 0.09], dtype=torch.float64))
    assert noisy[0] > 0.12 and noisy[1] > 0.2
    assert torch.all(noisy < 0.7)
    # a model whose noise exceeds 25 %: the floor stops at 25 %, so a
    # quiet tensor off by 100 % still fails
    big = verify_tolerance(torch.tensor([0.0, 0.6], dtype=torch.float64))
    assert float(big[0]) == pytest.approx(0.251)
    assert torch.isnan(verify_tolerance(torch.tensor([0.0, float('nan')]))).all()


def test_verify_ratio_strict() -> None:
    """A bit-reproducible eager step (all noise zero) makes the check
    strict: any nonzero replay distance fails, zero passes; otherwise the
    distance is measured against the tolerance and non-finite fails."""
    tol = verify_tolerance(torch.zeros(3, dtype=torch.float64))
    d = torch.tensor([0.0, 1e-7, 0.0], dtype=torch.float64)
    assert float(verify_ratio(d, tol, False).max()) < 1.0
    strict = verify_ratio(d, tol, True)
    assert strict[0] == 0 and strict[2] == 0 and torch.isinf(strict[1])
    assert float(verify_ratio(torch.zeros(3, dtype=torch.float64), tol, True).max()) == 0.0
    assert torch.isinf(verify_ratio(torch.tensor([float('nan')]), tol[:1], False)).all()
    assert torch.isinf(verify_ratio(torch.tensor([float('nan')]), tol[:1], True)).all()


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


@pytest.fixture
def deterministic():
    """MIOpen's default convolution backward is not bitwise reproducible;
    with deterministic kernels every K-FAC kernel here is (fixed-order
    split-K SYRK and KL-clip reductions), so graph replay and eager
    execution must agree exactly."""
    old = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    yield
    torch.backends.cudnn.deterministic = old


def _eager_runner(device: torch.device, method: str = 'eigen', step_graphs: bool = True,
                  set_to_none: bool = False):
    model, opt, pre, fb = _setup(device, method=method)
    if step_graphs:
        from distributed_kfac_pytorch_amd.base_preconditioner import StepGraphs

        pre._graphs = StepGraphs()  # opt-in (KFAC_GRAPHS=1)
    else:
        pre._graphs = None

    def run() -> float:
        opt.zero_grad(set_to_none=set_to_none)
        loss = float(fb())
        pre.step()
        opt.step()
        return loss
    return model, opt, pre, run


def _state_diff(ma, oa, pa, mb, ob, pb) -> float:
    """Largest relative difference over parameters, momentum buffers and
    K-FAC factors."""
    worst = 0.0

    def rel(a: torch.Tensor, b: torch.Tensor) -> float:
        d = float((a.double() - b.double()).abs().max())
        return d / max(float(b.double().abs().max()), 1e-30)

    for a, b in zip(ma.parameters(), mb.parameters()):
        worst = max(worst, rel(a, b))
        worst = max(worst, rel(oa.state[a]['momentum_buffer'], ob.state[b]['momentum_buffer']))
    for (_, la), (_, lb) in zip(pa._layers.values(), pb._layers.values()):
        worst = max(worst, rel(la.a_factor, lb.a_factor), rel(la.g_factor, lb.g_factor))
    return worst


@pytest.mark.gpu
@pytest.mark.parametrize('method', ['eigen', 'inverse'])
@pytest.mark.parametrize('kinds', [('plain',), ('plain', 'factor')])
def test_graph_replay_matches_eager(cuda, deterministic, method, kinds) -> None:
    """Whole-step graph replay vs eager steps, compared after EVERY step
    over 20 steps (3 second-order updates: the eigenbases / inverses are
    reinstalled in place under the captured graphs); plain steps replayed
    with factor steps eager (the default) or both replayed."""
    steps = 20
    model, opt, pre, fb = _setup(cuda, method=method)
    runner = GraphedTrainStep(fb, opt, pre, kinds=kinds)
    mb, ob, pb, run_b = _eager_runner(cuda, method)
    for i in range(steps):
        la = float(runner())
        lb = run_b()
        torch.cuda.synchronize()
        assert abs(la - lb) <= 1e-6 * max(1.0, abs(lb)), (i, la, lb)
        d = _state_diff(model, opt, pre, mb, ob, pb)
        assert d <= 1e-6, (i, runner.kind(), d)
    assert runner.captures == len(kinds), runner.captures
    assert runner.replays >= (14 if 'factor' in kinds else 9), runner.replays
    assert pre.steps == pb.steps == steps


@pytest.mark.gpu
def test_step_graphs_match_plain_eager(cuda, deterministic) -> None:
    """The precondition-phase graphs (StepGraphs) vs fully eager K-FAC."""
    ma, oa, pa, run_a = _eager_runner(cuda, step_graphs=True)
    mb, ob, pb, run_b = _eager_runner(cuda, step_graphs=False)
    for i in range(14):
        run_a()
        run_b()
        torch.cuda.synchronize()
        assert _state_diff(ma, oa, pa, mb, ob, pb) <= 1e-6, i
    assert pa._graphs.replays >= 6


@pytest.mark.gpu
def test_table_rekey_every_step_matches(cuda, deterministic) -> None:
    """zero_grad(set_to_none=True) gives the gradients new addresses every
    step, so the descriptor tables are rebuilt and their pinned staging
    buffers recycled continuously while the host runs ahead of the GPU (no
    sync inside the loop).  The result must equal the persistent-gradient
    run bit for bit: a staging buffer is never rewritten before its queued
    H2D copy has run."""
    ma, oa, pa, run_a = _eager_runner(cuda, step_graphs=False, set_to_none=True)
    mb, ob, pb, run_b = _eager_runner(cuda, step_graphs=False, set_to_none=False)
    for _ in range(40):
        run_a()
    for _ in range(40):
        run_b()
    torch.cuda.synchronize()
    assert _state_diff(ma, oa, pa, mb, ob, pb) <= 1e-6


def test_graph_safe_conv_modes_cpu() -> None:
    """``GraphedTrainStep``'s conv conversion (``conv_mode``) on CPU: the
    model's and K-FAC's registered 1x1 convolutions, same parameters."""
    from distributed_kfac_pytorch_amd.graphs import _graph_safe
    from distributed_kfac_pytorch_amd.ops.conv import GemmConv1x1
    from distributed_kfac_pytorch_amd.ops.conv import StridedConv1x1

    def net() -> torch.nn.Module:
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 1, stride=2), torch.nn.ReLU(),
                                   torch.nn.Conv2d(8, 8, 1), torch.nn.Conv2d(8, 4, 3))

    m = net()
    x = torch.randn(2, 3, 8, 8).contiguous(memory_format=torch.channels_last)
    ref = m(x)
    assert _graph_safe(m, None, 'strided') == 1
    assert type(m[0]) is StridedConv1x1 and type(m[2]) is torch.nn.Conv2d
    torch.testing.assert_close(m(x), ref)
    m = net().to(memory_format=torch.channels_last)
    pre = kfac.KFACPreconditioner(m)
    assert _graph_safe(m, pre, 'gemm') == 2  # the model's two 1x1 convs
    assert type(m[0]) is GemmConv1x1 and type(m[2]) is GemmConv1x1
    assert type(m[3]) is torch.nn.Conv2d
    torch.testing.assert_close(m(x), ref, rtol=1e-5, atol=1e-6)


def test_close_releases_graphs_and_drain_is_safe_without_gpu() -> None:
    """``GraphedTrainStep.close()`` drops every graph (call it before
    ``destroy_process_group``); ``drain_collectives`` is a no-op without a
    GPU or a process group."""
    from distributed_kfac_pytorch_amd.graphs import drain_collectives

    drain_collectives()
    _, opt, pre, fb = _setup(torch.device('cpu'))
    runner = GraphedTrainStep(fb, opt, pre, enabled=False)
    runner()
    runner.graphs['plain'] = object()  # stand-in for a captured graph
    runner.close()
    assert not runner.graphs and not runner.enabled
    runner()  # still steps, eagerly
    assert runner.eager_steps == 2


@pytest.mark.gpu
def test_verify_leaves_factors_bit_identical(cuda, deterministic) -> None:
    """The capture-time check runs eager steps (one of them a factor step,
    whose G-factor SYRKs may still be running on the factor side stream when
    ``step()`` returns) and restores the saved state after each: the factors
    after the check and the following factor / plain steps must be bit for
    bit those of the same run with the check off (restore()
    ordered after the side stream's work)."""
    runs = []
    for verify in (True, False):
        model, opt, pre, fb = _setup(cuda, method='eigen')
        runner = GraphedTrainStep(fb, opt, pre, kinds=('plain', 'factor'), verify=verify)
        for _ in range(14):
            runner()
        pre.sync_factors()
        torch.cuda.synchronize()
        assert runner.captures == 2, runner.captures
        runs.append([t.clone() for _, l in pre._layers.values() for t in (l.a_factor, l.g_factor)]
                    + [p.detach().clone() for p in model.parameters()])
    for a, b in zip(*runs):
        assert torch.equal(a, b)
