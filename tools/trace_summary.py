"""Summarise a rocprofv3 kernel_trace.csv: total GPU busy time, top kernels,
and the busy fraction of the wall span (idle gaps = launch/host bound)."""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def main(path: str, out: str) -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            try:
                s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            except (KeyError, ValueError):
                continue
            rows.append((s, e, r.get('Kernel_Name', '?')))
    rows.sort()
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
        for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:60]:
            f.write(f'{t/1e6:10.3f} ms  {c:7d}  {n[:160]}\n')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
