"""Time the eigensolver paths on the ResNet-50 K-FAC factor size mix.

Per distinct factor dimension n (with its multiplicity in ResNet-50): batched
torch.linalg.eigh, batched rocSOLVER syevd / syevj / syevdj through the native
extension, and the native Jacobi kernel for n <= 128.  Then the full
``eigh_many`` over all 108 factors (multi-stream) for comparison with the
sequential sum.  One JSON line per measurement.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402

SIZES = {64: 12, 128: 12, 147: 1, 256: 26, 512: 19, 576: 3, 1000: 1,
         1024: 14, 1152: 4, 2048: 6, 2049: 1, 2304: 6, 4608: 3}


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def make(n, cnt, dev):
    x = torch.randn(cnt, n, 2 * n, device=dev)
    return (x @ x.transpose(1, 2)) / (2 * n) + 1e-3 * torch.eye(n, device=dev)


def main() -> None:
    dev = torch.device('cuda')
    lib = native()
    totals = {}
    allmats = []
    for n, cnt in SIZES.items():
        a = make(n, cnt, dev)
        allmats += [a[i] for i in range(cnt)]
        reps = 1 if n >= 2048 else 2
        row = {'n': n, 'count': cnt}
        row['torch_batched'] = timed(lambda: torch.linalg.eigh(a), reps)
        for name, algo in (('syevd', 0), ('syevj', 1), ('syevdj', 2)):
            if name == 'syevj' and n > 2304:
                continue
            try:
                row[name] = timed(lambda: lib.rocsolver_eigh(a.clone(), algo, 100, 1e-7), reps)
            except Exception as e:  # noqa: BLE001
                row[name] = str(e)[:80]
        if n <= linalg.jacobi_max_n():
            row['jacobi'] = timed(lambda: lib.jacobi_eigh(a.contiguous(), 15, 1e-7), reps)
        for k, v in row.items():
            if isinstance(v, float):
                row[k] = round(v, 2)
                totals[k] = totals.get(k, 0.0) + v
        # accuracy of syevj/syevd vs torch
        d_ref = torch.linalg.eigvalsh(a.double())
        for name, algo in (('syevd', 0), ('syevj', 1)):
            if name in row and isinstance(row[name], float):
                w, v = lib.rocsolver_eigh(a.clone(), algo, 100, 1e-7)
                rec = v @ torch.diag_embed(w) @ v.transpose(1, 2)
                row[f'{name}_recon_err'] = float((rec - a).abs().max() / a.abs().max())
                row[f'{name}_eval_err'] = float((w.double() - d_ref).abs().max() / d_ref.abs().max())
        print(json.dumps(row), flush=True)
    print(json.dumps({'sequential_totals_ms': {k: round(v, 1) for k, v in totals.items()}}), flush=True)
    for mode in ('auto', 'syevd', 'torch'):
        os.environ['KFAC_EIGH'] = mode
        for streams in ('1', '4'):
            os.environ['KFAC_EIGH_STREAMS'] = streams
            ms = timed(lambda: linalg.eigh_many(allmats), 2)
            print(json.dumps({'eigh_many': mode, 'streams': streams, 'ms': round(ms, 1)}), flush=True)


if __name__ == '__main__':
    main()
