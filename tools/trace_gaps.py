"""Per-kernel durations and launch gaps from a rocprofv3 kernel trace.

    python tools/trace_gaps.py gpurun_out/x/prof/*_results.db [--top 25] [--stream]

Reads the rocpd SQLite database rocprofv3 writes.  For every kernel name:
calls, total / mean duration, and the mean idle gap since the previous
kernel that ended on the same queue (the launch / dependency overhead a
persistent or graphed version would remove).  Also prints the busy fraction
of the traced interval.
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--top', type=int, default=25)
    ap.add_argument('--match', default='', help='only kernels whose name contains this')
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    rows = c.execute(
        'select s.kernel_name, d.start, d.end, d.queue_id from rocpd_kernel_dispatch d '
        'join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start').fetchall()
    last_end: dict = {}
    agg: dict = defaultdict(lambda: [0, 0.0, 0.0])
    for name, st, en, q in rows:
        short = name.split('(')[0][:90]
        gap = (st - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = max(en, last_end.get(q, 0))
        if args.match and args.match not in name:
            continue
        a = agg[short]
        a[0] += 1
        a[1] += (en - st) / 1e3
        a[2] += max(gap, 0.0)
    t0 = rows[0][1] if rows else 0
    t1 = max(r[2] for r in rows) if rows else 0
    busy = 0.0
    cur_s = cur_e = None
    for _, st, en, _ in rows:
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    if cur_e is not None:
        busy += cur_e - cur_s
    print(f'kernels {len(rows)}  span {(t1 - t0) / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms')
    print(f'{"kernel":90s} {"calls":>7s} {"tot_ms":>9s} {"avg_us":>8s} {"gap_us":>8s}')
    for name, (n, tot, gap) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f'{name:90s} {n:7d} {tot / 1e3:9.2f} {tot / n:8.2f} {gap / n:8.2f}')


if __name__ == '__main__':
    main()
