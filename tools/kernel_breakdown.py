"""Per-(kernel, grid) duration breakdown of a rocprofv3 kernel_trace.csv for
kernels whose name contains a filter string.  Usage:
python tools/kernel_breakdown.py trace.csv filter out.txt"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict


def main(path: str, filt: str, out: str) -> None:
    agg = defaultdict(lambda: [0, 0])
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get('Kernel_Name', '?')
            if filt not in name:
                continue
            try:
                d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            except (KeyError, ValueError):
                continue
            m = re.search(r'(\w*' + re.escape(filt) + r'\w*)(<[^>(]*>)?', name)
            short = m.group(0) if m else name[:40]
            key = (short, r.get('Grid_Size_X', r.get('Grid_Size', '?')))
            agg[key][0] += d
            agg[key][1] += 1
    lines = ['total_us calls avg_us grid kernel']
    for (n, g), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        lines.append(f'{t / 1e3:10.1f} {c:6d} {t / c / 1e3:8.2f} {g:>9} {n}')
    open(out, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3])
