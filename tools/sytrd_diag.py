"""Diagnostics for the native sytrd eigensolver tier: per-size errors for
single matrices and for the ResNet-50 factor mix, with and without lane
threads.  One JSON line per case."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402

SIZES = {64: 12, 128: 12, 147: 1, 256: 26, 512: 19, 576: 3, 1000: 1,
         1024: 14, 1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}


def make(n, cnt, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed + n)
    x = torch.randn(cnt, n, 2 * n, device=dev, generator=g)
    return (x @ x.transpose(1, 2)) / (2 * n) + 1e-3 * torch.eye(n, device=dev)


def errs(mats, res):
    out = {}
    for m, (d, q) in zip(mats, res):
        ref = torch.linalg.eigvalsh(m.double())
        e = float((d.double() - ref).abs().max() / ref.abs().max())
        rc = float(((q.double() * d.double()) @ q.double().T - m.double()).abs().max()
                   / m.abs().max())
        n = m.shape[0]
        o = out.setdefault(n, [0.0, 0.0])
        o[0] = max(o[0], e)
        o[1] = max(o[1], rc)
    return {str(k): [f'{v[0]:.1e}', f'{v[1]:.1e}'] for k, v in sorted(out.items())}


def main() -> None:
    dev = torch.device('cuda')
    os.environ['KFAC_SYTRD_MIN_N'] = '512'
    os.environ['KFAC_EIGH'] = 'sytrd'
    for n in (1024, 2304, 4608):
        m = make(n, 1, dev)[0]
        res = linalg.eigh_many([m])
        print(json.dumps({'case': 'single', 'n': n, 'err': errs([m], res)}), flush=True)
    for n, cnt in ((1024, 3), (4608, 3)):
        s = make(n, cnt, dev)
        mats = [s[i].contiguous() for i in range(cnt)]
        res = linalg.eigh_many(mats)
        print(json.dumps({'case': 'bucket', 'n': n, 'cnt': cnt, 'err': errs(mats, res)}),
              flush=True)
    mats = []
    for n, cnt in SIZES.items():
        s = make(n, cnt, dev)
        mats += [s[i].contiguous() for i in range(cnt)]
    for threads in ('1', '0'):
        os.environ['KFAC_EIGH_THREADS'] = threads
        res = linalg.eigh_many(mats)
        torch.cuda.synchronize()
        print(json.dumps({'case': 'mix', 'threads': threads, 'err': errs(mats, res)}),
              flush=True)
    big = [m for m in mats if m.shape[0] >= 512]
    res = linalg.eigh_many(big)
    print(json.dumps({'case': 'mix_big_only', 'err': errs(big, res)}), flush=True)


if __name__ == '__main__':
    main()
