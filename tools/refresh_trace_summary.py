"""Summarise a rocprofv3 kernel trace of tools/refresh_probe.py: the last
refresh (kernels after the largest idle gap in the final second), per queue:
first start / last end relative to the refresh start, busy time, kernel
count and top kernels.  Usage: refresh_trace_summary.py <kernel_trace.csv>"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def main() -> None:
    rows = []
    with open(sys.argv[1]) as f:
        rd = csv.DictReader(f)
        print('columns:', rd.fieldnames)
        for r in rd:
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                         (r.get('Stream_Id'), r.get('Queue_Id')), r['Kernel_Name']))
    rows.sort()
    end = rows[-1][1]
    # the last refresh: walk back from the end to the last gap > 20 ms
    i = len(rows) - 1
    run_end = rows[0][1]
    gaps = []
    for j in range(1, len(rows)):
        run_end = max(run_end, rows[j - 1][1])
        if rows[j][0] - run_end > 100_000_000:
            gaps.append(j)
    i = gaps[-1] if gaps else 0
    win = rows[i:]
    t0 = win[0][0]
    print(f'refresh window: {len(win)} kernels, span {(end - t0) / 1e6:.1f} ms')
    by = defaultdict(list)
    for s, e, q, n in win:
        by[q].append((s, e, n))
    for q, ks in sorted(by.items(), key=lambda kv: kv[1][0][0]):
        busy = sum(e - s for s, e, _ in ks)
        first = (ks[0][0] - t0) / 1e6
        last = (max(e for _, e, _ in ks) - t0) / 1e6
        top = defaultdict(float)
        for s, e, n in ks:
            top[n.split('(')[0][-60:]] += (e - s) / 1e6
        tops = sorted(top.items(), key=lambda kv: -kv[1])[:4]
        print(f'queue {q}: {len(ks)} kernels, {first:.1f} -> {last:.1f} ms, busy {busy / 1e6:.1f} ms')
        for n, t in tops:
            print(f'    {t:8.2f} ms  {n}')


if __name__ == '__main__':
    main()
