"""Second-order refresh on REAL ResNet-50 K-FAC factors.

Trains the bench configuration (ResNet-50, batch 32, synthetic batches,
factor update 10, inverse update 100) up to the step-100 refresh, snapshots
every factor and the eigenbases from the step-0 refresh, then times the
refresh of the whole factor mix (and of each size bucket) with each solver
tier and reports the block-Jacobi sweep counts and the accuracy against
float64.

    python tools/refresh_probe.py [--steps 100]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db')
os.environ.setdefault('MIOPEN_USER_DB_PATH', _DB)

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402


def snapshot(steps: int):  # type: ignore[no-untyped-def]
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5)
    pre = kfac.KFACPreconditioner(
        model, factor_update_steps=10, inv_update_steps=100, damping=0.001,
        lr=lambda s: opt.param_groups[0]['lr'], grad_worker_fraction=0.5,
    )
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    xs = [torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
          for _ in range(8)]
    ys = [torch.randint(0, 1000, (32,), device=dev) for _ in range(8)]
    qs = {}
    for i in range(steps):
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = crit(model(xs[i % 8]), ys[i % 8])
        loss.backward()
        pre.step()
        opt.step()
        if i == 0:
            for name, l in pre._layers.values():
                qs[name] = (l.qa.clone(), l.qg.clone())
    if steps == 0:  # cold: the step-0 factors (no previous basis)
        qs = None
    # factors as they stand at the next refresh: run the step-100 forward /
    # backward (factor hooks fire) without the K-FAC step
    opt.zero_grad()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        loss = crit(model(xs[steps % 8]), ys[steps % 8])
    loss.backward()
    pre._join_factor_streams()
    mats, warm = [], []
    for name, l in pre._layers.values():
        mats += [l.a_factor.float().clone(), l.g_factor.float().clone()]
        warm += [qs[name][0], qs[name][1]] if qs is not None else [None, None]
    return mats, warm


HOST: list = []


def timed(fn, reps: int = 2):  # type: ignore[no-untyped-def]
    fn()
    torch.cuda.synchronize()
    time.sleep(0.2)  # an idle gap that marks the timed reps in kernel traces
    t0 = time.perf_counter()
    HOST.clear()
    for _ in range(reps):
        t1 = time.perf_counter()
        out = fn()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        HOST.append((round((t2 - t1) * 1e3, 1), round((time.perf_counter() - t1) * 1e3, 1)))
    return (time.perf_counter() - t0) / reps * 1e3, out


def accuracy(mats, res) -> dict:  # type: ignore[no-untyped-def]
    worst = {'eval_err': 0.0, 'recon_err': 0.0, 'orth_err': 0.0}
    for m, (d, q) in zip(mats, res):
        if m.shape[0] <= 128:
            continue
        m64 = m.double()
        ref = torch.linalg.eigvalsh(m64)
        sc = float(ref.abs().max())
        rec = q.double() @ torch.diag(d.double()) @ q.double().t()
        eye = torch.eye(m.shape[0], dtype=torch.float64, device=m.device)
        worst['eval_err'] = max(worst['eval_err'], float((d.double() - ref).abs().max()) / sc)
        worst['recon_err'] = max(worst['recon_err'], float((rec - m64).abs().max()) / sc)
        worst['orth_err'] = max(worst['orth_err'],
                                float((q.double().t() @ q.double() - eye).abs().max()))
    return worst


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--per-bucket', type=int, default=1)
    ap.add_argument('--modes', type=int, default=4)
    ap.add_argument('--mode-list', default='',
                    help='comma-separated modes, e.g. auto_warm,sytrd4000_warm (overrides --modes)')
    ap.add_argument('--reps', type=int, default=2)
    ap.add_argument('--no-acc', action='store_true',
                    help='skip the float64 accuracy check (kernel traces)')
    args = ap.parse_args()
    mats, warm = snapshot(args.steps)
    sizes = defaultdict(int)
    for m in mats:
        sizes[m.shape[0]] += 1
    print(json.dumps({'factors': len(mats), 'sizes': dict(sorted(sizes.items()))}), flush=True)

    def run(mode: str):  # type: ignore[no-untyped-def]
        if mode.startswith('default'):
            # the library's default tiers, untouched (default / default_warm)
            w = list(warm) if '_warm' in mode else None
            linalg.last_stats.clear()
            return linalg.eigh_many([m.clone() for m in mats], w)
        os.environ['KFAC_EIGH_BLOCK'] = '0' if mode == 'syevd' else '1'
        os.environ['KFAC_EIGH_LARGE'] = 'block' if mode.startswith('block') else 'syevd'
        if mode.startswith('sytrd'):
            # native batched tridiagonalisation for n >= the number in the name
            os.environ['KFAC_EIGH'] = 'sytrd'
            spec = mode[len('sytrd'):].split('_')[0]  # e.g. 1000x4000-2000
            os.environ['KFAC_SYTRD_MIN_N'] = spec.split('x')[0]
            os.environ['KFAC_SYTRD_SPLIT'] = (spec.split('x')[1].replace('-', ',')
                                              if 'x' in spec else '4000')
        else:
            os.environ['KFAC_EIGH'] = 'auto'
        os.environ['KFAC_EIGH_ORMTR'] = 'rocsolver' if '_ormtr' in mode else 'blocked'
        w = list(warm) if '_warm' in mode else None
        linalg.last_stats.clear()
        return linalg.eigh_many([m.clone() for m in mats], w)

    modes = (args.mode_list.split(',') if args.mode_list else
             ['syevd', 'auto_warm', 'block_warm', 'block_cold'][: args.modes])
    for mode in modes:
        ms, res = timed(lambda: run(mode), args.reps)
        rec = {'mode': mode, 'mix_ms': round(ms, 1), 'host_gpu_ms': list(HOST)}
        if linalg.last_stats.get('accepted'):
            rec['accepted'] = len(linalg.last_stats['accepted']) // 3
        if mode.startswith('block'):
            sw = defaultdict(list)
            for n, s in linalg.last_stats.get('sweeps', []):
                sw[n].append(s)
            rec['sweeps'] = {str(k): v[: len(v) // 2 or 1] for k, v in sorted(sw.items())}
        if not args.no_acc:
            rec.update(accuracy(mats, res))
        print(json.dumps(rec), flush=True)
    if args.per_bucket:
        by = defaultdict(list)
        for i, m in enumerate(mats):
            by[m.shape[0]].append(i)
        for n, idxs in sorted(by.items()):
            if n <= 128:
                continue
            stack = torch.stack([mats[i] for i in idxs])
            wst = torch.stack([warm[i] for i in idxs])
            lib = linalg.native()
            t_s, _ = timed(lambda: lib.rocsolver_eigh(stack.clone(), 0, 100, 1e-7))
            t_w, out = timed(lambda: lib.block_jacobi_eigh(stack, wst, 12, linalg.BJ_TOL,
                                                           linalg.BJ_INNER, linalg.BJ_NOISE, True))
            print(json.dumps({'n': n, 'count': len(idxs), 'syevd_ms': round(t_s, 2),
                              'block_warm_ms': round(t_w, 2),
                              'sweeps': out[2].tolist(),
                              'active': out[3][0].tolist()}), flush=True)


if __name__ == '__main__':
    main()
