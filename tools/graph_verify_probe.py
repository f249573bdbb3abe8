"""Sample the capture-time check's noise floor many times (diagnostic).

``GraphedTrainStep._verify`` compares three replays against two eager steps
from one saved state, with a per-tensor tolerance derived from ONE eager
pair.  When a run drops its graphs, this tool tells whether the replays are
really further from the eager step than eager steps are from each other
(a graph hazard), or the single eager pair under-sampled the noise of a
tensor whose kernels use atomics.

It runs any training CLI (``examples/*.py``) with ``_verify`` wrapped: after
the normal check, from the same saved state, ``N`` eager steps and ``N``
replays (half of them after an eager step of the other kind) are taken and,
per tensor, the largest relative distance eager-eager, replay-eager and
replay-replay is printed (top tensors by replay/eager ratio) as JSON lines
on stderr, prefixed ``[probe]``.

    python tools/graph_verify_probe.py [-n 6] -- examples/torch_imagenet_resnet.py ...
"""
from __future__ import annotations

import json
import os
import runpy
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd import graphs  # noqa: E402


def _rel(xs: list, ys: list) -> torch.Tensor:
    num = torch.stack([torch.linalg.vector_norm((x - y).double()) for x, y in zip(xs, ys)])
    den = torch.stack([torch.linalg.vector_norm(y.double()) for y in ys])
    return num / den.clamp_min(1e-300)


def probe(self: graphs.GraphedTrainStep, kind: str, n: int) -> None:
    p = self.preconditioner
    state = self._state(kind)
    with torch.no_grad():
        saved = [t.detach().clone() for t in state]
    rng = torch.cuda.get_rng_state()
    steps = p._steps if p is not None else 0
    at = self._next_step_of(kind) if p is not None else 0
    other = None
    if p is not None:
        other = self._next_step_of('factor' if kind == 'plain' else 'plain')
    params = self._params()
    names = {id(q): name for name, q in self.model.named_parameters()} if self.model else {}

    def restore() -> None:
        with torch.no_grad():
            for t, s0 in zip(state, saved):
                t.copy_(s0)
        torch.cuda.set_rng_state(rng)

    def grads(gs: list) -> list:
        return [g.detach().clone() if g is not None else torch.zeros_like(q)
                for g, q in zip(gs, params)]

    def eager(step_at: int) -> list:
        restore()
        if p is not None:
            p._steps = step_at
        self._eager_step()
        if p is not None:
            p._steps = steps
            p._mini_steps = defaultdict(int)
            p._mini_steps_g = defaultdict(int)
        return grads([q.grad for q in params])

    def replay() -> list:
        restore()
        self.graphs[kind].replay()
        return grads(self.grads[kind])

    ev = [eager(at) for _ in range(n)]
    rv = []
    for i in range(n):
        if i % 2 and other is not None:
            eager(other)
        rv.append(replay())
    restore()
    if p is not None:
        p._steps = steps
    torch.cuda.synchronize()
    ee = torch.stack([_rel(e, ev[0]) for e in ev[1:]]).amax(0)
    re = torch.stack([_rel(r, ev[0]) for r in rv]).amax(0)
    rr = torch.stack([_rel(r, rv[0]) for r in rv[1:]]).amax(0)
    ratio = re / (ee + 1e-7)
    order = torch.argsort(ratio, descending=True)[:12].tolist()
    out = {'kind': kind, 'n': n, 'eager_max': float(ee.max()), 'replay_max': float(re.max()),
           'replay_replay_max': float(rr.max()), 'top': [
               {'i': i, 'name': names.get(id(params[i]), str(i)), 'ee': float(ee[i]),
                're': float(re[i]), 'rr': float(rr[i])} for i in order]}
    print('[probe] ' + json.dumps(out), file=sys.stderr, flush=True)


def main() -> None:
    argv = sys.argv[1:]
    n = 6
    if argv[:1] == ['-n']:
        n = int(argv[1])
        argv = argv[2:]
    if argv[:1] == ['--']:
        argv = argv[1:]
    orig = graphs.GraphedTrainStep._verify

    def wrapped(self: graphs.GraphedTrainStep, kind: str) -> bool:
        ok = orig(self, kind)
        print('[probe] verify ' + json.dumps({'kind': kind, **self.verify_report[kind]}),
              file=sys.stderr, flush=True)
        probe(self, kind, n)
        return ok

    graphs.GraphedTrainStep._verify = wrapped
    sys.argv = argv
    runpy.run_path(argv[0], run_name='__main__')


if __name__ == '__main__':
    main()
