"""Time the factor SYRKs (K-HIP-1/2, csrc/syrk.hip) on every ResNet-50
factor shape of the bench config (batch 32, 224x224, channels_last, fp32).

One row per distinct (kind, shape): the native op exactly as the layers call
it (ops/factors.py conv_cov_accumulate_ / cov_accumulate_), median of
``--reps`` event-timed calls, and the effective fp32 rate over the computed
upper-triangle tiles.  ``--json`` writes the rows; the total is the sum over
all 108 calls of one factor-update step (shapes repeat).

    python tools/syrk_probe.py [--reps 20] [--only A|G] [--json out.jsonl]
"""
from __future__ import annotations

import argparse
import json
import math
import statistics

import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def factor_calls(batch: int) -> list[dict]:
    from distributed_kfac_pytorch_amd.models import resnet
    m = resnet.resnet50().cuda().to(memory_format=torch.channels_last)
    calls: list[dict] = []

    def hook(mod, inp, out):  # type: ignore[no-untyped-def]
        x = inp[0]
        if isinstance(mod, nn.Conv2d):
            calls.append(dict(kind='A', conv=True, shape=tuple(x.shape), k=mod.kernel_size,
                              s=mod.stride, p=mod.padding, bias=mod.bias is not None))
            n = out.shape[0] * out.shape[2] * out.shape[3]
            calls.append(dict(kind='G', conv=False, shape=(n, mod.out_channels), bias=False))
        elif isinstance(mod, nn.Linear):
            calls.append(dict(kind='A', conv=False, shape=(x.shape[0], mod.in_features),
                              bias=mod.bias is not None))
            calls.append(dict(kind='G', conv=False, shape=(x.shape[0], mod.out_features),
                              bias=False))

    hs = [mm.register_forward_hook(hook) for mm in m.modules()
          if isinstance(mm, (nn.Conv2d, nn.Linear))]
    with torch.no_grad():
        m(torch.randn(batch, 3, 224, 224, device='cuda').to(memory_format=torch.channels_last))
    for h in hs:
        h.remove()
    return calls


def key(c: dict) -> tuple:
    return (c['kind'], c['conv'], c['shape'], c.get('k'), c.get('s'), c.get('p'), c['bias'])


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--only', default='')
    ap.add_argument('--json', default='')
    args = ap.parse_args()
    from distributed_kfac_pytorch_amd.ops import factors as F

    calls = factor_calls(args.batch)
    uniq: dict[tuple, list] = {}
    for c in calls:
        if args.only and c['kind'] != args.only:
            continue
        uniq.setdefault(key(c), [c, 0])[1] += 1
    rows = []
    total_ms = 0.0
    for k, (c, count) in uniq.items():
        if c['conv'] and (c['k'] != (1, 1) or c['s'] != (1, 1)):
            x = torch.randn(c['shape'], device='cuda').to(memory_format=torch.channels_last)
            b, ch, h, w = c['shape']
            d = ch * c['k'][0] * c['k'][1] + int(c['bias'])
            oh = (h + 2 * c['p'][0] - c['k'][0]) // c['s'][0] + 1
            ow = (w + 2 * c['p'][1] - c['k'][1]) // c['s'][1] + 1
            n = b * oh * ow
            out = torch.zeros(d, d, device='cuda')

            def run() -> None:
                if not F.conv_cov_accumulate_(out, x, c['k'], c['s'], c['p'], bias=c['bias'],
                                              alpha=1.0 / n, beta=0.5):
                    # explicit patches (the layer's path for C % 4 != 0: the stem)
                    pm, _ = F.conv_patches(x, c['k'], c['s'], c['p'], True)
                    F.cov_accumulate_(out, pm, bias=c['bias'], alpha=1.0 / n, beta=0.5)
            mode = 'patch' if c['shape'][1] % 4 == 0 else 'im2col'
        else:
            if c['conv']:
                b, ch, h, w = c['shape']
                n, kk = b * h * w, ch
            else:
                n, kk = c['shape']
            x = torch.randn(n, kk, device='cuda')
            d = kk + int(c['bias'])
            out = torch.zeros(d, d, device='cuda')

            def run() -> None:
                F.cov_accumulate_(out, x, bias=c['bias'], alpha=1.0 / n, beta=0.5)
            mode = 'dense'
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        t = math.ceil(d / 128)
        flops = 2.0 * n * (t * (t + 1) // 2) * 128 * 128
        row = dict(kind=c['kind'], mode=mode, n=n, d=d, count=count, ms=round(ms, 4),
                   tflops=round(flops / ms / 1e9, 1),
                   splits=int(F.native().syrk_default_splits(n, d)))
        rows.append(row)
        total_ms += ms * count
        print(json.dumps(row), flush=True)
    print(json.dumps(dict(total_ms_one_factor_step=round(total_ms, 3),
                          calls=sum(v[1] for v in uniq.values()))), flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            for r in rows:
                f.write(json.dumps(r) + '\n')


if __name__ == '__main__':
    main()
