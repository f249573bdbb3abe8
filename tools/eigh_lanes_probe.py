"""Probe: does issuing the rocSOLVER syevd lanes from one host thread per
lane (instead of one thread for all) let the GPU overlap them?  rocSOLVER's one-stage sytrd issues ~5 tiny kernels per
column (≈22k launches for n=4608), so an eager call is host-launch bound.

Prints one JSON line per configuration: time for the whole ResNet-50 factor
mix and the max eigenvalue / reconstruction errors.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402

SIZES = {64: 12, 128: 12, 147: 1, 256: 26, 512: 19, 576: 3, 1000: 1,
         1024: 14, 1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}


def make(n, cnt, dev):
    x = torch.randn(cnt, n, 2 * n, device=dev)
    return (x @ x.transpose(1, 2)) / (2 * n) + 1e-3 * torch.eye(n, device=dev)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main() -> None:
    dev = torch.device('cuda')
    # whole ResNet-50 mix through eigh_many: single-thread vs threaded lanes
    mats = []
    for n, cnt in SIZES.items():
        s = make(n, cnt, dev)
        mats += [s[i].contiguous() for i in range(cnt)]
    ref = [torch.linalg.eigvalsh(m.double()) for m in mats]
    # PROBE_CONFIGS="threads:streams:split_n,..." overrides the default list
    spec = os.environ.get('PROBE_CONFIGS')
    if spec:
        configs = [tuple(c.split(':')) for c in spec.split(',')]
    else:
        configs = [('1', '8', '100000'), ('0', '8', '100000'),
                   ('1', '8', '4608'), ('1', '12', '4608'), ('1', '12', '2304')]
    for cfg in configs:
        threads, streams, split = cfg[:3]
        mode = cfg[3] if len(cfg) > 3 else 'auto'
        min_n = cfg[4] if len(cfg) > 4 else '512'
        os.environ['KFAC_EIGH_THREADS'] = threads
        os.environ['KFAC_EIGH_STREAMS'] = streams
        os.environ['KFAC_EIGH_SPLIT_N'] = split
        os.environ['KFAC_EIGH'] = mode
        os.environ['KFAC_SYTRD_MIN_N'] = min_n
        row = {'mix': 'resnet50', 'threads': threads, 'streams': streams, 'split_n': split,
               'eigh': mode, 'sytrd_min_n': min_n,
               'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES', 'default')}
        row['ms'] = round(timed(lambda: linalg.eigh_many(mats), 2), 1)
        got = linalg.eigh_many(mats)
        row['max_rel_eval_err'] = max(
            float((d.double() - r).abs().max() / r.abs().max()) for (d, _), r in zip(got, ref))
        row['max_recon_err'] = max(
            float(((q * d) @ q.T - m).abs().max() / m.abs().max()) for (d, q), m in zip(got, mats))
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
