"""The bench's eigen refresh in isolation: real K-FAC factors vs the
synthetic probe mix, in one process.

    python tools/refresh_replay.py [--steps 101] [--reps 3]

Trains the bench configuration (ResNet-50, batch 32, 224x224, fp32,
channels_last, fused SGD, K-FAC factor 10 / inverse 100) eagerly for
``--steps`` steps, takes every layer's A and G factor as the refresh sees
them, and times ``ops.linalg.eigh_many`` on clones of them (``reps`` runs,
one untimed first), then on the same number of synthetic factors of the
same sizes (``tools/eigh_probe.py``'s generator).  A gap between the two
isolates the data dependence (Jacobi sweeps, divide-and-conquer deflation)
from the bench context (other streams, allocator state).  Also reports the
largest factor's spectrum spread.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db')
if os.path.isdir(_DB):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', _DB)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from eigh_probe import factor  # noqa: E402


def timed(mats: list[torch.Tensor], reps: int) -> list[float]:
    linalg.eigh_many([m.clone() for m in mats])
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        ms = [m.clone() for m in mats]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        linalg.eigh_many(ms)
        torch.cuda.synchronize()
        out.append(round((time.perf_counter() - t0) * 1e3, 2))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=101)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
    pre = kfac.KFACPreconditioner(
        model, factor_update_steps=10, inv_update_steps=100, damping=0.001,
        factor_decay=0.95, kl_clip=0.001, lr=lambda s: opt.param_groups[0]['lr'],
        grad_worker_fraction=0.5)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    gen = torch.Generator(device='cpu').manual_seed(1)
    pool = [(torch.randn(32, 3, 224, 224, generator=gen).to(dev).contiguous(
        memory_format=torch.channels_last), torch.randint(0, 1000, (32,), generator=gen).to(dev))
        for _ in range(4)]
    for i in range(args.steps):
        x, y = pool[i % len(pool)]
        opt.zero_grad(set_to_none=False)
        crit(model(x), y).backward()
        pre.step()
        opt.step()
    torch.cuda.synchronize()
    real = []
    for _, layer in pre._layers.values():
        for f in (layer.a_factor, layer.g_factor):
            if f is not None:
                real.append(f.detach().float().clone())
    sizes = [m.shape[-1] for m in real]
    synth = [factor(n, dev, 100 + i) for i, n in enumerate(sizes)]
    big = max(range(len(real)), key=lambda i: sizes[i])
    ev = torch.linalg.eigvalsh(real[big].double())
    out = {'factors': len(real), 'max_n': sizes[big],
           'real_ms': timed(real, args.reps), 'synthetic_ms': timed(synth, args.reps),
           'real_tiers': linalg.last_stats.get('tiers') if hasattr(linalg, 'last_stats') else None,
           'largest_eig_range': [float(ev.min()), float(ev.max())],
           'largest_eig_rel_gap_median': float(((ev[1:] - ev[:-1]) / ev.abs().max()).median())}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
