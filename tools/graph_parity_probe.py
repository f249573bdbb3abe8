"""Step-by-step parity of whole-step HIP-graph replay against eager steps.

Runs the same small conv net twice in lockstep -- once through
``GraphedTrainStep`` (captured plain/factor graphs, eager inverse steps) and
once eagerly -- and after every step prints one JSON line with the largest
absolute difference of each piece of state: parameters, momentum buffers,
K-FAC factors, second-order state (eigenbases / inverses) and the loss.
The first non-zero column names the phase where the two paths part.

    python tools/graph_parity_probe.py [--method eigen|inverse] [--steps 14]

Environment toggles (``KFAC_FACTOR_STREAM``, ``KFAC_GRAPHS``, ...) apply to
both runs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep  # noqa: E402


def setup(device: torch.device, method: str, seed: int = 0):  # type: ignore[no-untyped-def]
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


def _d(a: torch.Tensor | None, b: torch.Tensor | None) -> float:
    if a is None or b is None:
        return -1.0 if (a is None) != (b is None) else 0.0
    return float((a.float() - b.float()).abs().max())


def diffs(ma, oa, pa, mb, ob, pb) -> dict:  # type: ignore[no-untyped-def]
    out = {
        'param': max(_d(a, b) for a, b in zip(ma.parameters(), mb.parameters())),
        'momentum': max(
            _d(oa.state[a].get('momentum_buffer'), ob.state[b].get('momentum_buffer'))
            for a, b in zip(ma.parameters(), mb.parameters())
        ),
    }
    la = [l for _, l in pa._layers.values()]
    lb = [l for _, l in pb._layers.values()]
    out['a_factor'] = max(_d(x.a_factor, y.a_factor) for x, y in zip(la, lb))
    out['g_factor'] = max(_d(x.g_factor, y.g_factor) for x, y in zip(la, lb))
    for attr in ('qa', 'qg', 'dgda', 'a_inv', 'g_inv'):
        if hasattr(la[0], attr):
            out[attr] = max(_d(getattr(x, attr), getattr(y, attr)) for x, y in zip(la, lb))
    return out


def precond_error(pre) -> float:  # type: ignore[no-untyped-def]
    """Largest relative error, over layers, of the installed eigen
    preconditioner Qg((Qg^T V Qa) * dGdA)Qa^T against float64 math on the
    layer's own factors (random V)."""
    worst = 0.0
    for _, l in pre._layers.values():
        if getattr(l, 'dgda', None) is None:
            continue
        a = l.a_factor.double().cpu()
        g = l.g_factor.double().cpu()
        da, qa = torch.linalg.eigh(a)
        dg, qg = torch.linalg.eigh(g)
        damp = pre.damping
        v = torch.randn(g.shape[0], a.shape[0], dtype=torch.float64)
        ex = qg @ ((qg.t() @ v @ qa) / (torch.outer(dg.clamp(min=0), da.clamp(min=0)) + damp)) @ qa.t()
        Qa, Qg, S = l.qa.double().cpu(), l.qg.double().cpu(), l.dgda.double().cpu()
        got = Qg @ ((Qg.t() @ v @ Qa) * S) @ Qa.t()
        worst = max(worst, float((got - ex).abs().max() / ex.abs().max()))
    return worst


def make(dev: torch.device, method: str, mode: str):  # type: ignore[no-untyped-def]
    """mode: graph (GraphedTrainStep) | step (StepGraphs eager) | eager."""
    m, o, p, f = setup(dev, method)
    if mode == 'eager':
        p._graphs = None
    if mode == 'graph':
        r = GraphedTrainStep(f, o, p)
        return m, o, p, lambda: float(r()), r

    def run() -> float:
        o.zero_grad(set_to_none=False)
        v = float(f())
        p.step()
        o.step()
        return v
    return m, o, p, run, None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--method', default='eigen')
    ap.add_argument('--steps', type=int, default=14)
    ap.add_argument('--a', default='graph', help='graph | step | eager')
    ap.add_argument('--b', default='step', help='graph | step | eager')
    ap.add_argument('--deterministic', action='store_true',
                    help='torch.backends.cudnn.deterministic (MIOpen)')
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = args.deterministic
    dev = torch.device('cuda')
    ma, oa, pa, sa, runner = make(dev, args.method, args.a)
    mb, ob, pb, sb, _ = make(dev, args.method, args.b)
    for i in range(args.steps):
        kind = runner.kind() if runner is not None else ('inverse' if pa.steps % 6 == 0 else '')
        la = sa()
        lb = sb()
        torch.cuda.synchronize()
        rec = {'step': i, 'kind': kind, 'loss': abs(la - lb)}
        rec.update(diffs(ma, oa, pa, mb, ob, pb))
        if args.method == 'eigen' and pa.steps % 6 == 1:
            rec['err_a'] = precond_error(pa)
            rec['err_b'] = precond_error(pb)
        rec['replays'] = runner.replays if runner is not None else 0
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
