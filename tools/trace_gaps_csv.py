"""Idle gaps of the GPU timeline in a rocprofv3 kernel_trace.csv, inside the
window bench --profile-mark brackets with identity_kernel launches.

    python tools/trace_gaps_csv.py kernel_trace.csv out.txt [min_gap_us]

Writes the gap histogram and the largest gaps with the kernels on either
side (a gap after kernel X = the GPU waited for work issued after X: a host
stall, a cross-stream wait or a launch-bound stretch).
"""
from __future__ import annotations

import csv
import sys
from collections import Counter


def main(path: str, out: str, min_gap_us: float = 20.0) -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            try:
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                             r.get('Kernel_Name', '?'), r.get('Queue_Id', r.get('Stream_Id', '?'))))
            except (KeyError, ValueError):
                continue
    rows.sort()
    marks = [i for i, r in enumerate(rows) if 'identity_kernel' in r[2]]
    if len(marks) >= 2:
        rows = rows[marks[-2] + 1: marks[-1]]
    gaps = []
    end = rows[0][1] if rows else 0
    for i in range(1, len(rows)):
        s = rows[i][0]
        if s > end:
            gaps.append(((s - end) / 1e3, i))
        end = max(end, rows[i][1])
    hist = Counter()
    for g, _ in gaps:
        b = '<5us' if g < 5 else '5-20us' if g < 20 else '20-100us' if g < 100 else '100us-1ms' if g < 1000 else '>1ms'
        hist[b] += g
    with open(out, 'w') as f:
        span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0
        f.write(f'kernels={len(rows)} span_us={span:.0f} idle_us={sum(g for g, _ in gaps):.0f}\n')
        f.write('idle by gap size (us): ' + ', '.join(f'{k}={v:.0f}' for k, v in sorted(hist.items())) + '\n')
        queues = Counter(r[3] for r in rows)
        f.write(f'queues: {dict(queues)}\n')
        f.write('largest gaps: us | before | after\n')
        for g, i in sorted(gaps, reverse=True)[:40]:
            if g < min_gap_us:
                break
            f.write(f'{g:9.1f} | {rows[i - 1][2][:70]} [q{rows[i - 1][3]}] | {rows[i][2][:70]} [q{rows[i][3]}]\n')
        # gap-after counts per preceding kernel (top 25)
        after = Counter()
        for g, i in gaps:
            if g >= min_gap_us:
                after[rows[i - 1][2][:70]] += g
        f.write('idle after kernel (us, gaps >= min):\n')
        for k, v in after.most_common(25):
            f.write(f'{v:9.1f}  {k}\n')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 20.0)
