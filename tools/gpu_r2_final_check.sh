#!/bin/bash
# round-end rehearsal: build check import, smoke(), default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ('value','ms_per_step','steps','warmup','kind_ms','kind_counts','sgd_ms_per_step','kfac_overhead_ms','vs_baseline')})"
