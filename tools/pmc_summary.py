"""Summarise rocprofv3 --pmc CSV passes into one row per kernel.

Reads ``<dir>/<prefix>_<pass>/<prefix>_<pass>_counter_collection.csv`` and
``..._kernel_trace.csv`` for the passes sq / fetch / write (tools/
gpu_r2_pmc.sh) and writes a CSV plus a markdown table:

* time: summed dispatch durations of the sq pass (counter passes serialise
  dispatches, so absolute times are profiled times);
* (GRBM_GUI_ACTIVE is collected but not turned into a clock: summed over
  serialised dispatches and hardware units it does not give one);
* MFMA pipe utilisation: SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x
  1024 SIMDs), and MFMA TFLOP/s from SQ_INSTS_VALU_MFMA_MOPS_* (x 512 FLOP);
* HBM: FETCH_SIZE / WRITE_SIZE in KB (FETCH_SIZE under-counts wide
  streaming reads by 2x on gfx950: MI355X_MICROARCH.md), L2 hit rate;
* LDS bank-conflict cycles / LDS active cycles.

    python tools/pmc_summary.py gpurun_out/pmc step out_prefix [pass1,pass2,...]

(the first pass's dispatch timestamps give the kernel times)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def _read(path: str) -> list[dict]:
    if not os.path.exists(path):
        return []
    with open(path, newline='') as f:
        return list(csv.DictReader(f))


def _col(row: dict, *names: str) -> str | None:
    for n in names:
        if n in row:
            return n
    return None


def short(name: str) -> str:
    for junk in ('void ', 'kfac::', '(anonymous namespace)::', 'kfac::tile::'):
        name = name.replace(junk, '')
    name = name.split('(')[0]
    return name[:90]


def _find(d: str, suffix: str) -> str:
    """The rocprofv3 CSV ending in ``suffix`` under pass directory ``d``
    (directly, or in rocprofv3's host / pid subdirectories)."""
    hits = sorted(glob.glob(os.path.join(d, '**', '*' + suffix), recursive=True))
    return hits[0] if hits else os.path.join(d, suffix)


def load(base: str, prefix: str, passes: tuple[str, ...] = ('sq', 'fetch', 'write')) -> dict:
    counters: dict = defaultdict(lambda: defaultdict(float))
    times: dict = defaultdict(float)
    counts: dict = defaultdict(int)
    for p in passes:
        d = os.path.join(base, f'{prefix}_{p}')
        rows = _read(_find(d, 'counter_collection.csv'))
        for r in rows:
            k = _col(r, 'Kernel_Name', 'Kernel-Name', 'KernelName')
            c = _col(r, 'Counter_Name', 'Counter-Name')
            v = _col(r, 'Counter_Value', 'Counter-Value')
            if k and c and v:
                counters[short(r[k])][r[c]] += float(r[v] or 0)
        if p == passes[0]:
            trace = _read(_find(d, 'kernel_trace.csv'))
            if not trace:
                # counter-only pass (no --kernel-trace): one row per
                # (dispatch, counter) carries the dispatch's timestamps
                seen = {}
                for r in rows:
                    if 'Dispatch_Id' in r:
                        seen[r['Dispatch_Id']] = r
                trace = list(seen.values())
            for r in trace:
                k = _col(r, 'Kernel_Name', 'Kernel-Name')
                s = _col(r, 'Start_Timestamp', 'Start-Timestamp')
                e = _col(r, 'End_Timestamp', 'End-Timestamp')
                if k and s and e:
                    times[short(r[k])] += (int(r[e]) - int(r[s])) * 1e-6
                    counts[short(r[k])] += 1
    out = {}
    for k, t in times.items():
        c = counters.get(k, {})
        row = {'kernel': k, 'dispatches': counts[k], 'time_ms': round(t, 3)}
        if t > 0:
            # MFMA pipe busy fraction at the nominal 2.4 GHz (a lower bound
            # when the chip clocks down under load)
            row['mfma_util'] = round(
                c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / (t * 1e-3 * 2.4e9 * SIMDS), 4)
        mops = c.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0.0) + c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
        if t > 0:
            row['mfma_tflops'] = round(mops * 512 / (t * 1e-3) / 1e12, 2)
            row['mfma_mops_bf16'] = c.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0.0)
            row['mfma_mops_f32'] = c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
            fetch_kb = c.get('FETCH_SIZE', 0.0)
            write_kb = c.get('WRITE_SIZE', 0.0)
            row['fetch_kb'] = round(fetch_kb, 1)
            row['write_kb'] = round(write_kb, 1)
            row['fetch_gbs'] = round(fetch_kb * 1024 / (t * 1e-3) / 1e9, 1)
            row['write_gbs'] = round(write_kb * 1024 / (t * 1e-3) / 1e9, 1)
        hit, miss = c.get('TCC_HIT_sum', 0.0), c.get('TCC_MISS_sum', 0.0)
        if hit + miss:
            row['l2_hit'] = round(hit / (hit + miss), 3)
        lds = c.get('SQ_LDS_IDX_ACTIVE', 0.0)
        if lds:
            row['lds_conflict'] = round(c.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds, 4)
        row['waves'] = c.get('SQ_WAVES', 0.0)
        for name, key in (('valu_insts', 'SQ_INSTS_VALU'), ('lds_insts', 'SQ_INSTS_LDS'),
                          ('wait_inst_any', 'SQ_WAIT_INST_ANY'), ('wave_cycles', 'SQ_WAVE_CYCLES'),
                          ('busy_cycles', 'SQ_BUSY_CYCLES')):
            if key in c:
                row[name] = c[key]
        out[k] = row
    return out


def main() -> None:
    base, prefix, dest = sys.argv[1], sys.argv[2], sys.argv[3]
    passes = tuple(sys.argv[4].split(',')) if len(sys.argv) > 4 else ('sq', 'fetch', 'write')
    rows = sorted(load(base, prefix, passes).values(), key=lambda r: -r['time_ms'])
    keys = ['kernel', 'dispatches', 'time_ms', 'mfma_util', 'mfma_tflops',
            'fetch_gbs', 'write_gbs', 'l2_hit', 'lds_conflict', 'fetch_kb', 'write_kb',
            'mfma_mops_bf16', 'mfma_mops_f32', 'waves', 'valu_insts', 'lds_insts',
            'wait_inst_any', 'wave_cycles', 'busy_cycles']
    with open(dest + '.csv', 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=keys, extrasaction='ignore')
        w.writeheader()
        for r in rows:
            w.writerow(r)
    with open(dest + '.md', 'w') as f:
        f.write('| kernel | n | ms | MFMA util | MFMA TF/s | fetch GB/s | write GB/s | L2 hit | LDS confl |\n')
        f.write('|---|---|---|---|---|---|---|---|---|\n')
        for r in rows[:25]:
            f.write('| {} | {} | {} | {} | {} | {} | {} | {} | {} |\n'.format(
                r['kernel'], r['dispatches'], r['time_ms'],
                r.get('mfma_util', ''), r.get('mfma_tflops', ''), r.get('fetch_gbs', ''),
                r.get('write_gbs', ''), r.get('l2_hit', ''), r.get('lds_conflict', '')))
    print(json.dumps(rows[:12], indent=None)[:4000])


if __name__ == '__main__':
    main()
