"""Summarise a rocprofv3 kernel_trace.csv: total GPU busy time, top kernels,
and the busy fraction of the wall span (idle gaps = launch/host bound)."""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def main(path: str, out: str, window: str | None = None, steps: int = 0) -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            try:
                s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            except (KeyError, ValueError):
                continue
            rows.append((s, e, r.get('Kernel_Name', '?')))
    rows.sort()
    if window:
        marks = [i for i, r in enumerate(rows) if window in r[2]]
        if len(marks) >= 2:
            rows = rows[marks[-2] + 1: marks[-1]]
    if not rows:
        open(out, 'w').write('no rows\n')
        return
    span = rows[-1][1] - rows[0][0]
    busy = 0
    cur_s, cur_e = rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        agg[n][0] += e - s
        agg[n][1] += 1
    with open(out, 'w') as f:
        f.write(f'kernels={len(rows)} span_ms={span/1e6:.2f} busy_ms={busy/1e6:.2f} '
                f'busy_frac={busy/span:.3f}\n')
        if steps:
            f.write(f'per_step: span_ms={span/1e6/steps:.3f} busy_ms={busy/1e6/steps:.3f} '
                    f'kernels={len(rows)/steps:.1f}\n')
        cats = defaultdict(float)
        for n, (t, _) in agg.items():
            cats[_category(n)] += t
        f.write('categories (ms total' + (', ms/step' if steps else '') + '):\n')
        for c, t in sorted(cats.items(), key=lambda kv: -kv[1]):
            f.write(f'  {c:28s} {t/1e6:10.3f}' + (f' {t/1e6/steps:8.3f}' if steps else '') + '\n')
        f.write('top kernels: total_ms calls name\n')
        for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:60]:
            f.write(f'{t/1e6:10.3f} ms  {c:7d}  {n[:160]}\n')


def _category(name: str) -> str:
    n = name.lower()
    if 'kfac::' in n:
        return 'kfac native (HIP)'
    if 'rocsolver' in n:
        return 'rocsolver (eigh)'
    if n.startswith('igemm_') or 'conv' in n:
        return 'conv (miopen/ck)'
    if n.startswith('subtensorop'):
        return 'miopen tensor ops'
    if n.startswith('cijk_') or 'gemm' in n:
        return 'gemm (hipblaslt/rocblas)'
    if 'batchnorm' in n:
        return 'batchnorm (miopen)'
    if 'nccl' in n or 'rccl' in n:
        return 'rccl'
    if 'at::native' in n or 'elementwise' in n or 'reduce' in n:
        return 'torch elementwise/reduce'
    return 'other'


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None,
         int(sys.argv[4]) if len(sys.argv) > 4 else 0)
