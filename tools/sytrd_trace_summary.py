"""Per-column durations of the native sytrd kernels from a rocprofv3 kernel
trace of tools/sytrd_time.py (ONLY=4608): how symv / col time scales with
the trailing size m = n - k."""
from __future__ import annotations

import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
for name in ('sytrd_symv_kernel', 'sytrd_col_kernel'):
    d = [(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows if name in r['Kernel_Name']]
    d.sort()
    n = 4608
    per = len(d) // 3  # three reps
    seq = d[per:2 * per]  # the middle rep
    print(name, len(d))
    for k in range(0, len(seq), 384):
        dur = [(e - s) / 1e3 for s, e in seq[k:k + 8]]
        gap = [(seq[j + 1][0] - seq[j][1]) / 1e3 for j in range(k, min(k + 8, len(seq) - 1))]
        print(f'  k~{k:5d}  m~{n - k:5d}  dur_us {sum(dur) / len(dur):7.2f}  gap_us {sum(gap) / max(len(gap), 1):7.2f}')
