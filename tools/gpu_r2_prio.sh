#!/bin/bash
# refresh: high-priority critical chain A/B, graph replay A/B; tests; default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prio
cd $R
O=gpurun_out/prio
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd or eigh" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "1 1" "0 1"; do
  set -- $v
  KFAC_SYTRD_PRIORITY=$1 KFAC_SYTRD_GRAPHS=$2 timeout -k 10 400 python -u tools/refresh_probe.py --per-bucket 0 --reps 4 --mode-list sytrd2000_warm > $O/probe_$1_$2.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
  echo "prio=$1 graphs=$2 $(tail -1 $O/probe_$1_$2.jsonl | cut -c1-200)"
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['kind_ms'],d['inverse_ms_each'])"
bash tools/gpu_r2_rtrace.sh
