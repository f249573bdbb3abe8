"""Split a rocprofv3 kernel trace of bench.py into training steps and diff
the kernels of an SGD step against a K-FAC plain step.

    python tools/step_kernel_diff.py <kernel_trace.csv> [marker]

Steps are delimited by a kernel that runs once per step (default: the
max-pool forward).  Steps are classified by the kernels they contain:
``inverse`` (rocSOLVER), ``factor`` (SYRK), ``plain`` (grouped GEMM) or
``sgd`` (none of those).  Prints per-kind median busy / wall time and, for
the median plain and sgd steps, the per-kernel-name time difference.
"""
from __future__ import annotations

import csv
import statistics
import sys
from collections import defaultdict


def main(path: str, marker: str = 'max_pool_forward') -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    starts = [s for s, _, n in rows if marker in n]
    steps = []
    j = 0
    for a, b in zip(starts, starts[1:]):
        ks = []
        while j < len(rows) and rows[j][0] < a:
            j += 1
        k = j
        while k < len(rows) and rows[k][0] < b:
            ks.append(rows[k])
            k += 1
        steps.append((a, b, ks))

    def kind(ks):
        names = ' '.join(n for _, _, n in ks)
        if 'rocsolver' in names or 'sytrd' in names or 'jacobi_kernel' in names:
            return 'inverse'
        if 'syrk_kernel' in names:
            return 'factor'
        if 'gemm3s_kernel' in names:
            return 'plain'
        return 'sgd'

    by = defaultdict(list)
    for a, b, ks in steps:
        busy = sum(e - s for s, e, _ in ks)
        by[kind(ks)].append(((b - a) / 1e6, busy / 1e6, len(ks), ks))
    for k, v in by.items():
        print(f'{k:8s} steps {len(v):4d}  wall {statistics.median(x[0] for x in v):8.3f} ms  '
              f'busy {statistics.median(x[1] for x in v):8.3f} ms  kernels {statistics.median(x[2] for x in v)}')

    def agg(v):
        v = sorted(v, key=lambda x: x[0])[len(v) // 4: 3 * len(v) // 4 or 1]
        d = defaultdict(float)
        for _, _, _, ks in v:
            for s, e, n in ks:
                d[n[:90]] += (e - s) / 1e3 / len(v)
        return d

    if 'factor' in by and 'plain' in by:
        f, p = agg(by['factor']), agg(by['plain'])
        diff = sorted(((f.get(n, 0) - p.get(n, 0), n) for n in set(f) | set(p)), reverse=True)
        print('\nper-step kernel time, factor-update minus plain K-FAC step (us):')
        for dt, n in diff[:20]:
            print(f'{dt:9.1f}  factor {f.get(n, 0):8.1f}  plain {p.get(n, 0):8.1f}  {n}')
    if 'sgd' in by:
        s = agg(by['sgd'])
        print('\nper-step kernel time of an SGD step, top 30 (us):')
        for n, t in sorted(s.items(), key=lambda kv: -kv[1])[:30]:
            print(f'{t:9.1f}  {n}')
    if 'plain' in by and 'sgd' in by:
        p, s = agg(by['plain']), agg(by['sgd'])
        diff = sorted(((p.get(n, 0) - s.get(n, 0), n) for n in set(p) | set(s)), reverse=True)
        print('\nper-step kernel time, plain K-FAC minus SGD (us):')
        for dt, n in diff[:30]:
            print(f'{dt:9.1f}  plain {p.get(n, 0):8.1f}  sgd {s.get(n, 0):8.1f}  {n}')
        print('...')
        for dt, n in diff[-8:]:
            print(f'{dt:9.1f}  plain {p.get(n, 0):8.1f}  sgd {s.get(n, 0):8.1f}  {n}')


if __name__ == '__main__':
    main(*sys.argv[1:])
