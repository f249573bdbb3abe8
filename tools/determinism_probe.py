"""Are two EAGER twins of the bench step bit-identical?

    python tools/determinism_probe.py [--steps 24] [--conv1x1 gemm|miopen] [--graphed]
                                      [--db=tuned|--db=fresh] [--det-algos] [--go-on]
                                      [--fp32 [--kxk gemm|miopen]] [--cudnn-det 0|1]

Builds two copies of the bench's ResNet-50 step (batch 32, 224x224, bf16
autocast, fused weight casts, fused SGD, K-FAC factor 2 / inverse 8) from the
same weights and steps them alternately on the same inputs.  After each
backward (before ``pre.step()``) the raw gradients are compared, after each
step the parameters, preconditioned gradients and K-FAC factors: the first
mismatch is reported with the layers involved, in backward order, so a
nondeterministic op shows up as the deepest mismatching layer.  With
``--graphed`` the first copy runs under ``GraphedTrainStep`` (plain steps
replayed) as in ``tests/test_graphs_refresh_gpu.py``.  ``--fp32`` steps the
bench's fp32 headline configuration instead (no autocast; ``--kxk gemm``:
3x3 convolutions on the native implicit GEMM as in the bench); with
``--cudnn-det 0`` MIOpen picks its algorithms as the bench lets it
(``torch.backends.cudnn.deterministic`` off).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db')
# --db tuned: the bench's tuned MIOpen database; --db fresh: an empty one (as
# the test suite sees MIOpen); read before torch initialises MIOpen
_MODE = 'fresh' if '--db=fresh' in sys.argv else 'tuned'
if _MODE == 'tuned' and os.path.isdir(_DB):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', _DB)
elif _MODE == 'fresh':
    import tempfile
    os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='miopen_fresh_')

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_kfac_pytorch_amd.ops.cast import enable_fused_weight_cast  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import use_implicit_gemm_conv  # noqa: E402


def build(base, dev, conv1x1: str, graphed: bool, fp32: bool = False, kxk: str = 'gemm'):
    model = copy.deepcopy(base).to(dev).to(memory_format=torch.channels_last)
    if conv1x1 == 'gemm':
        use_gemm_conv1x1(model)
    if fp32 and kxk == 'gemm':
        use_implicit_gemm_conv(model)
    if not fp32:
        enable_fused_weight_cast(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
    pre = kfac.KFACPreconditioner(model, factor_update_steps=2, inv_update_steps=8,
                                  damping=0.001, kl_clip=0.001,
                                  lr=lambda s: opt.param_groups[0]['lr'], grad_worker_fraction=0.5)
    x = torch.empty(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.empty(32, dtype=torch.long, device=dev)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    raw: dict = {}

    def fb() -> torch.Tensor:
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=not fp32, cache_enabled=False):
            loss = crit(model(x), y)
        loss.backward()
        if not torch.cuda.is_current_stream_capturing():
            raw['g'] = [p.grad.detach().clone() for p in model.parameters()]
        return loss

    if graphed:
        run = GraphedTrainStep(fb, opt, pre, warmup=1, enabled=True, kinds=('plain',),
                               model=model, conv_mode=conv1x1 if conv1x1 == 'gemm' else None)
    else:
        def run() -> torch.Tensor:
            opt.zero_grad(set_to_none=False)
            loss = fb()
            pre.step()
            opt.step()
            return loss.detach()
    return dict(model=model, pre=pre, x=x, y=y, run=run, raw=raw)


def rel(p: torch.Tensor, q: torch.Tensor) -> float:
    p, q = p.detach().double(), q.detach().double()
    return float((p - q).norm() / q.norm().clamp_min(1e-12))


def factors(m) -> list[torch.Tensor]:
    out = []
    for _, layer in m['pre']._layers.values():
        out += [f for f in (layer.a_factor, layer.g_factor) if f is not None]
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=24)
    ap.add_argument('--conv1x1', choices=('gemm', 'miopen'), default='gemm')
    ap.add_argument('--graphed', action='store_true')
    ap.add_argument('--db', choices=('tuned', 'fresh'), default='tuned')
    ap.add_argument('--go-on', action='store_true', help='keep stepping after a mismatch')
    ap.add_argument('--det-algos', action='store_true',
                    help='torch.use_deterministic_algorithms(True, warn_only=True)')
    ap.add_argument('--fp32', action='store_true', help="the bench's fp32 step (no autocast)")
    ap.add_argument('--kxk', choices=('gemm', 'miopen'), default='gemm')
    ap.add_argument('--cudnn-det', type=int, default=1)
    ap.add_argument('--fwd-check', action='store_true',
                    help='step 0: report the first module (forward order) whose output '
                         'differs between the twins')
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = bool(args.cudnn_det)
    if args.det_algos:
        torch.use_deterministic_algorithms(True, warn_only=True)
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = resnet50()
    names = [n for n, _ in base.named_parameters()]
    gen = torch.Generator(device='cpu').manual_seed(1)
    pool = [(torch.randn(32, 3, 224, 224, generator=gen),
             torch.randint(0, 1000, (32,), generator=gen)) for _ in range(4)]
    A = build(base, dev, args.conv1x1, args.graphed, args.fp32, args.kxk)
    B = build(base, dev, args.conv1x1, False, args.fp32, args.kxk)
    report = {'conv1x1': args.conv1x1, 'graphed': args.graphed, 'steps': args.steps,
              'fp32': args.fp32, 'kxk': args.kxk, 'cudnn_det': args.cudnn_det,
              'db': args.db, 'det_algos': args.det_algos,
              'first_mismatch': None}
    for i in range(args.steps):
        xb, yb = pool[i % len(pool)]
        for m in (A, B):
            m['raw'].clear()
            m['x'].copy_(xb)
            m['y'].copy_(yb)
        outs: dict = {'A': [], 'B': []}
        hooks = []
        if args.fwd_check and i == 0:
            for tag, m in (('A', A), ('B', B)):
                for name, mod in m['model'].named_modules():
                    if name and not list(mod.children()):
                        hooks.append(mod.register_forward_hook(
                            lambda mod_, a_, o_, tag=tag, name=name: outs[tag].append(
                                (name, o_.detach().clone()))))
        A['run']()
        B['run']()
        for h in hooks:
            h.remove()
        if outs['A']:
            first = next(((na, rel(oa, ob)) for (na, oa), (_, ob) in zip(outs['A'], outs['B'])
                          if not torch.equal(oa, ob)), None)
            print(json.dumps({'fwd_modules': len(outs['A']), 'first_fwd_mismatch': first}),
                  flush=True)
        torch.cuda.synchronize()
        rec = {'step': i}
        if 'g' in A['raw'] and 'g' in B['raw']:
            rec['raw_grad'] = [n for n, p, q in zip(names, A['raw']['g'], B['raw']['g'])
                               if not torch.equal(p, q)]
        pa, pb = list(A['model'].parameters()), list(B['model'].parameters())
        rec['param'] = [n for n, p, q in zip(names, pa, pb) if not torch.equal(p, q)]
        rec['grad'] = [n for n, p, q in zip(names, pa, pb) if not torch.equal(p.grad, q.grad)]
        rec['factor'] = [j for j, (p, q) in enumerate(zip(factors(A), factors(B)))
                         if not torch.equal(p, q)]
        bad = any(rec.get(k) for k in ('raw_grad', 'param', 'grad', 'factor'))
        # the twin test's tolerance metrics (tests/test_graphs_refresh_gpu.py)
        kfac_ids = {id(p) for _, layer in A['pre']._layers.values()
                    for p in layer.module.module.parameters()}
        rel_p = rel(torch.cat([p.detach().flatten() for p in pa]),
                    torch.cat([q.detach().flatten() for q in pb]))
        rel_g = sorted(((rel(p.grad, q.grad), n) for n, p, q in zip(names, pa, pb)
                        if id(p) not in kfac_ids), reverse=True)[:3]
        print(json.dumps({'step': i, 'bad': bad, 'rel_param': rel_p,
                          'rel_grad_unpreconditioned_top': rel_g,
                          **{k: len(v) for k, v in rec.items() if isinstance(v, list)}}), flush=True)
        if bad and not args.go_on:
            # deepest first: the backward starts at the last layer
            for k in ('raw_grad', 'param', 'grad'):
                if rec.get(k):
                    rec[k] = {'count': len(rec[k]), 'deepest': rec[k][::-1][:6]}
            if rec['factor']:
                rec['factor'] = {'count': len(rec['factor']), 'indices': rec['factor'][:12]}
            report['first_mismatch'] = rec
            break
    print(json.dumps(report), flush=True)


if __name__ == '__main__':
    main()
