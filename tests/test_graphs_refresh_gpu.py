"""Whole-step HIP graphs across eigen refreshes at production shape.

Round 2 found that ``GraphedTrainStep`` replays after an eager second-order
refresh produced NaN in every K-FAC layer on the ResNet-50 bench config
(profiles/graph_replay_nonfinite_r2.txt), while the toy-model parity test
(tests/test_graphs.py) passed.  The cause: the runner kept the captured
loss -- and through its autograd graph every parameter's AccumulateGrad
node, bound to the capture's side stream -- alive, so the eager refresh
step accumulated its gradients on that foreign stream from buffers the
producing stream had already recycled.

This test runs the configuration that failed: ResNet-50 (every eigensolver
tier: n <= 128 Jacobi, mid sizes, 2304 / 4608 large-n factors), fused BN,
bf16 autocast, channels_last, fused weight casts and the factor side stream,
with three refreshes inside the replay window.  The graph run goes first
(parameters checked for finiteness after every step, snapshots after each
refresh), then an eager twin from the same weights and data; with
deterministic MIOpen the two agree to the bit (round 3).  The twin runs
AFTER the graph run: interleaving a second model's eager steps between
replays perturbed the replays (profiles/graph_replay_r3_investigation.txt),
while runs with no foreign work between replays -- eager factor / refresh
steps of the same model included -- matched exactly.
"""
from __future__ import annotations

import copy

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep
from distributed_kfac_pytorch_amd.models.resnet import resnet50
from distributed_kfac_pytorch_amd.ops.cast import enable_fused_weight_cast

pytestmark = pytest.mark.gpu


def _build(base: torch.nn.Module, cuda: torch.device, graphs: bool, kinds=('plain',)):
    model = copy.deepcopy(base).to(cuda).to(memory_format=torch.channels_last)
    enable_fused_weight_cast(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-5)
    pre = kfac.KFACPreconditioner(
        model, factor_update_steps=2, inv_update_steps=8, damping=0.001,
        kl_clip=0.001, lr=lambda s: opt.param_groups[0]['lr'],
        grad_worker_fraction=0.5,
    )
    x = torch.empty(8, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.empty(8, dtype=torch.long, device=cuda)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)

    def fb() -> torch.Tensor:
        with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=not graphs):
            loss = crit(model(x), y)
        loss.backward()
        return loss

    if graphs:
        runner = GraphedTrainStep(fb, opt, pre, warmup=1, enabled=True, kinds=kinds)
    else:
        def runner() -> torch.Tensor:
            opt.zero_grad(set_to_none=False)
            loss = fb()
            pre.step()
            opt.step()
            return loss.detach()
    return model, pre, x, y, runner


@pytest.mark.parametrize('kinds', [('plain',), ('plain', 'factor')])
def test_graph_replay_matches_eager_across_refreshes(cuda, kinds) -> None:
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        torch.manual_seed(0)
        base = resnet50(num_classes=10)
        gen = torch.Generator(device='cpu').manual_seed(1)
        pool = [(torch.randn(8, 3, 64, 64, generator=gen),
                 torch.randint(0, 10, (8,), generator=gen)) for _ in range(4)]
        steps = 26  # refreshes at steps 0, 8, 16, 24
        marks = (1, 9, 17, 25)  # the step after each refresh
        snaps: list[dict] = []
        for graphs in (True, False):
            m, pre, xs, ys, run = _build(base, cuda, graphs, kinds)
            got: dict = {}
            for i in range(steps):
                x, y = pool[i % len(pool)]
                xs.copy_(x)
                ys.copy_(y)
                run()
                if graphs:
                    torch.cuda.synchronize()
                    fin = all(bool(torch.isfinite(p).all()) for p in m.parameters())
                    assert fin, f'non-finite parameters after step {i} (graph replay)'
                if i in marks:
                    got[i] = [p.detach().float().cpu() for p in m.parameters()]
            assert pre.steps == steps
            if graphs:
                assert isinstance(run, GraphedTrainStep)
                assert run.captures == len(kinds), run.captures
                assert run.replays >= (18 if 'factor' in kinds else 12), run.replays
                # the captured autograd graphs must not outlive their capture
                assert all(o.grad_fn is None for o in run.outputs.values())
            snaps.append(got)
            del m, pre, run
            torch.cuda.synchronize()
        for i in marks:
            num = max(float((a - b).abs().max()) for a, b in zip(snaps[0][i], snaps[1][i]))
            den = max(float(b.abs().max()) for b in snaps[1][i])
            assert num <= 1e-3 * den, (i, num / den)
    finally:
        torch.backends.cudnn.deterministic = det
