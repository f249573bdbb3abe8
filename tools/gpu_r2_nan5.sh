#!/bin/bash
# syevd default: finite? (twice, diagnostic step check), then the sytrd tier in eager mode
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh5
cd $R
for i in 1 2; do
  KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh5/d$i.log 2>&1 || { tail -5 gpurun_out/nh5/d$i.log; exit 1; }
  echo "syevd run $i: $(grep -c '\[nan\]' gpurun_out/nh5/d$i.log) nan lines $(grep -o '"params_finite": [a-z]*' gpurun_out/nh5/d$i.log)"
done
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/nh5/bench.json 2> gpurun_out/nh5/bench.err || { tail -5 gpurun_out/nh5/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/nh5/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'],d.get('sgd_ms_per_step'))"
