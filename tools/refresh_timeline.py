"""Timeline of one eigen refresh from a rocprofv3 kernel trace of
tools/refresh_probe.py: per-queue busy time, span, and which kernel families
run late (the critical path tail)."""
from __future__ import annotations

import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
print('columns:', list(rows[0].keys()))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Queue_Id', '?'),
             r.get('Stream_Id', '?'), r['Kernel_Name']) for r in rows)
# the last timed rep: split the trace at gaps > 20 ms
segs, cur = [], [ks[0]]
for k in ks[1:]:
    if k[0] - cur[-1][1] > 20_000_000:
        segs.append(cur)
        cur = []
    cur.append(k)
segs.append(cur)
print('segments', [(len(s), round((s[-1][1] - s[0][0]) / 1e6, 1)) for s in segs])
seg = max(segs[-3:], key=len)
t0 = seg[0][0]
span = (max(e for _, e, *_ in seg) - t0) / 1e6
print(f'refresh segment: {len(seg)} kernels, span {span:.1f} ms')
busy = defaultdict(float)
last = defaultdict(int)
for s, e, q, st, n in seg:
    busy[(q, st)] += (e - s) / 1e6
    last[(q, st)] = max(last[(q, st)], e)
for key in sorted(busy, key=lambda k: -busy[k]):
    print(f'queue {key}: busy {busy[key]:8.1f} ms  ends at {(last[key] - t0) / 1e6:8.1f} ms')
# union of busy intervals
iv = sorted((s, e) for s, e, *_ in seg)
u, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f'GPU busy (union) {u / 1e6:.1f} ms of {span:.1f} ms span')
fam = defaultdict(lambda: [0.0, 0])
for s, e, q, st, n in seg:
    f = n.split('(')[0].split('<')[0][-60:]
    fam[f][0] += (e - s) / 1e6
    fam[f][1] += 1
for f, (t, c) in sorted(fam.items(), key=lambda x: -x[1][0])[:15]:
    print(f'{t:8.1f} ms {c:6d}  {f}')
# what runs in the last 20% of the span
tail = defaultdict(float)
for s, e, q, st, n in seg:
    if (s - t0) / 1e6 > 0.8 * span:
        tail[n.split('(')[0][-60:]] += (e - s) / 1e6
print('tail (last 20% of span):')
for f, t in sorted(tail.items(), key=lambda x: -x[1])[:8]:
    print(f'{t:8.1f} ms  {f}')
