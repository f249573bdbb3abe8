#!/bin/bash
# recapture after every refresh (default now): finiteness, graph tests, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rc
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphs.py tests/test_e2e_gpu.py > gpurun_out/rc/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/rc/tests.log | head; tail -20 gpurun_out/rc/tests.log; exit 1; }
tail -1 gpurun_out/rc/tests.log
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/rc/d.log 2>&1 || { tail -5 gpurun_out/rc/d.log; exit 1; }
echo "diag: $(grep '\[nan\]' gpurun_out/rc/d.log | cut -c1-60) $(grep -o '"params_finite": [a-z]*' gpurun_out/rc/d.log)"
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/rc/b$i.json 2> gpurun_out/rc/b.err || { tail -5 gpurun_out/rc/b.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/rc/b$i.json').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'],d.get('step_graphs'),d.get('sgd_ms_per_step'))"
done
