"""Which ingredient of the bf16 twin test goes non-finite under the tuned
MIOpen database?

    python tools/tuned_db_bisect.py [--twin 0|1] [--fused-cast 0|1] [--kfac 0|1]
                                    [--db tuned|fresh] [--steps 8]

The configuration of ``tests/test_graphs_refresh_gpu.py`` (ResNet-50,
224x224, batch 32, bf16 autocast, channels_last, fused SGD, 1x1 convs as
GEMMs, K-FAC factor 2 / inverse 8, ``GraphedTrainStep`` replaying plain
steps) with one ingredient switched at a time: the eager twin stepped in
between, the fused weight casts, K-FAC.  After every step: are the graphed
model's parameters and gradients finite, which gradients are not (backward
order), and the capture-time check's report.  One JSON line per step.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import tempfile

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if '--db=fresh' in sys.argv:
    os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='miopen_fresh_')
else:
    d = tempfile.mkdtemp(prefix='miopen_tuned_')
    for f in os.listdir(os.path.join(_ROOT, 'miopen_db')):
        with open(os.path.join(_ROOT, 'miopen_db', f), 'rb') as src, \
                open(os.path.join(d, f), 'wb') as dst:
            dst.write(src.read())
    os.environ['MIOPEN_USER_DB_PATH'] = d

import torch  # noqa: E402

sys.path.insert(0, _ROOT)

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_kfac_pytorch_amd.ops.cast import enable_fused_weight_cast  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1  # noqa: E402


def build(base, dev, graphs: bool, fused: bool, use_kfac: bool):  # type: ignore[no-untyped-def]
    model = copy.deepcopy(base).to(dev).to(memory_format=torch.channels_last)
    use_gemm_conv1x1(model)
    if fused:
        enable_fused_weight_cast(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
    pre = kfac.KFACPreconditioner(
        model, factor_update_steps=2, inv_update_steps=8, damping=0.001, kl_clip=0.001,
        lr=lambda s: opt.param_groups[0]['lr'], grad_worker_fraction=0.5,
    ) if use_kfac else None
    x = torch.empty(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.empty(32, dtype=torch.long, device=dev)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)

    def fb() -> torch.Tensor:
        with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
            loss = crit(model(x), y)
        loss.backward()
        return loss

    if graphs:
        run = GraphedTrainStep(fb, opt, pre, warmup=1, enabled=True, kinds=('plain',),
                               model=model, conv_mode='gemm')
    else:
        def run() -> torch.Tensor:
            opt.zero_grad(set_to_none=False)
            loss = fb()
            if pre is not None:
                pre.step()
            opt.step()
            return loss.detach()
    return model, x, y, run


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--twin', type=int, default=1)
    ap.add_argument('--fused-cast', type=int, default=1)
    ap.add_argument('--kfac', type=int, default=1)
    ap.add_argument('--steps', type=int, default=8)
    ap.add_argument('--db', default='tuned')
    ap.add_argument('--deterministic', type=int, default=0,
                    help='torch.backends.cudnn.deterministic (the twin test sets it)')
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = bool(args.deterministic)
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(0)
    base = resnet50()
    gen = torch.Generator(device='cpu').manual_seed(1)
    pool = [(torch.randn(32, 3, 224, 224, generator=gen),
             torch.randint(0, 1000, (32,), generator=gen)) for _ in range(4)]
    A = build(base, dev, True, bool(args.fused_cast), bool(args.kfac))
    B = build(base, dev, False, bool(args.fused_cast), bool(args.kfac)) if args.twin else None
    cfg = {'deterministic': args.deterministic, 'twin': args.twin, 'fused_cast': args.fused_cast, 'kfac': args.kfac,
           'db': args.db, 'factor_stream': os.environ.get('KFAC_FACTOR_STREAM', 'auto')}
    first_bad = None
    for i in range(args.steps):
        xs, ys = pool[i % len(pool)]
        for m in (A, B):
            if m is not None:
                m[1].copy_(xs)
                m[2].copy_(ys)
        kind = A[3].kind()
        A[3]()
        if B is not None:
            B[3]()
        torch.cuda.synchronize()
        named = list(A[0].named_parameters())
        bad_p = [n for n, p in named if not bool(torch.isfinite(p).all())]
        bad_g = [n for n, p in reversed(named)
                 if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
        rec = {'step': i, 'kind': kind, 'replays': A[3].replays, 'bad_params': len(bad_p),
               'bad_grads': len(bad_g), 'first_bad_grads': bad_g[:4]}
        if B is not None:
            # the eager twin: is the step itself (not the replay) non-finite?
            rec['twin_bad_params'] = sum(not bool(torch.isfinite(p).all())
                                         for p in B[0].parameters())
            rec['twin_bad_grads'] = [n for n, p in reversed(list(B[0].named_parameters()))
                                     if p.grad is not None
                                     and not bool(torch.isfinite(p.grad).all())][:4]
        print(json.dumps(rec), flush=True)
        if (bad_p or bad_g) and first_bad is None:
            first_bad = i
    print(json.dumps({'config': cfg, 'first_nonfinite_step': first_bad,
                      'verify': A[3].verify_report, 'replays': A[3].replays}), flush=True)


if __name__ == '__main__':
    main()
