#!/bin/bash
# candidate fixes for non-finite replays after a refresh: recapture after each refresh; eager steps
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh7
cd $R
KFAC_GRAPHS_RECAPTURE=1 KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh7/r.log 2>&1 || { tail -5 gpurun_out/nh7/r.log; exit 1; }
echo "recapture diag: $(grep '\[nan\]' gpurun_out/nh7/r.log | cut -c1-60) $(grep -o '"params_finite": [a-z]*' gpurun_out/nh7/r.log)"
KFAC_GRAPHS_RECAPTURE=1 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/nh7/rb.json 2> gpurun_out/nh7/rb.err || { tail -5 gpurun_out/nh7/rb.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/nh7/rb.json').read().strip().splitlines()[-1]);print('recapture bench',d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'])"
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --graphs 0 > gpurun_out/nh7/eb.json 2> gpurun_out/nh7/eb.err || { tail -5 gpurun_out/nh7/eb.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/nh7/eb.json').read().strip().splitlines()[-1]);print('eager bench',d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'])"
