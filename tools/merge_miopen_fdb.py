"""Merge MIOpen find-db files (``*.ufdb.txt``) from several find runs: for
every problem key keep, per solver, the minimum measured time, and list the
solvers fastest-first (immediate mode takes the first).  Usage:
    python tools/merge_miopen_fdb.py OUT.ufdb.txt IN1.ufdb.txt IN2.ufdb.txt ...
"""
from __future__ import annotations

import sys


def parse(path: str) -> dict[str, dict[str, tuple[float, str]]]:
    out: dict[str, dict[str, tuple[float, str]]] = {}
    with open(path, encoding='utf-8') as f:
        for line in f:
            line = line.strip()
            if not line or '=' not in line:
                continue
            key, vals = line.split('=', 1)
            ent = out.setdefault(key, {})
            for item in vals.split(';'):
                if ':' not in item:
                    continue
                solver, rest = item.split(':', 1)
                fields = rest.split(',')
                try:
                    t = float(fields[0])
                except ValueError:
                    continue
                if solver not in ent or t < ent[solver][0]:
                    ent[solver] = (t, ','.join(fields[1:]))
    return out


def main(out_path: str, ins: list[str]) -> None:
    merged: dict[str, dict[str, tuple[float, str]]] = {}
    for p in ins:
        for key, ent in parse(p).items():
            m = merged.setdefault(key, {})
            for solver, (t, rest) in ent.items():
                if solver not in m or t < m[solver][0]:
                    m[solver] = (t, rest)
    with open(out_path, 'w', encoding='utf-8') as f:
        for key in sorted(merged):
            items = sorted(merged[key].items(), key=lambda kv: kv[1][0])
            f.write(key + '=' + ';'.join(f'{s}:{t:g},{rest}' for s, (t, rest) in items) + '\n')
    print(f'{len(merged)} problems merged from {len(ins)} files -> {out_path}')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])
