"""Where a Householder chain's time goes: per-kernel durations and the
idle gaps between consecutive kernels of the chain's queue, from a
rocprofv3 kernel_trace.csv of ``tools/eigh_probe.py``.

    python tools/chain_trace.py kernel_trace.csv [--last-ms 400]

Only the last ``--last-ms`` of the trace are analysed (the probe's final
repetition).  For every queue: kernels, busy time, and for each kernel name
its count, mean duration and the mean gap before it (end of the previous
kernel on that queue -> its start).
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--last-ms', type=float, default=400.0)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            try:
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                             r.get('Kernel_Name', '?').split('(')[0][-60:],
                             r.get('Queue_Id', r.get('Stream_Id', '?'))))
            except (KeyError, ValueError):
                continue
    rows.sort()
    end = max(r[1] for r in rows)
    rows = [r for r in rows if r[0] >= end - args.last_ms * 1e6]
    t0 = rows[0][0]
    print(f'window {(end - t0) / 1e6:.2f} ms, {len(rows)} kernels')
    by_q = defaultdict(list)
    for r in rows:
        by_q[r[3]].append(r)
    for q, rs in sorted(by_q.items(), key=lambda kv: -len(kv[1])):
        busy = sum(e - s for s, e, _, _ in rs)
        span = rs[-1][1] - rs[0][0]
        print(f'queue {q}: {len(rs)} kernels, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms')
        stats = defaultdict(lambda: [0, 0, 0])
        prev_end = None
        for s, e, name, _ in rs:
            st = stats[name]
            st[0] += 1
            st[1] += e - s
            if prev_end is not None:
                st[2] += max(0, s - prev_end)
            prev_end = e
        for name, (cnt, dur, gap) in sorted(stats.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
            print(f'   {cnt:6d} x {name:60s} mean {dur / cnt / 1e3:8.2f} us, '
                  f'gap before {gap / cnt / 1e3:7.2f} us, total {(dur + gap) / 1e6:8.2f} ms')


if __name__ == '__main__':
    main()
