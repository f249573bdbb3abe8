#!/bin/bash
# early preconditioning during backward: tests, bench A/B (default on vs off, frac sweep)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ov
cd $R
O=gpurun_out/ov
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_e2e_gpu.py tests/test_graphs.py > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "1 0.5" "0 0.5" "1 0.7" "1 0.35" "0 0.5" "1 0.5"; do
  set -- $cfg
  KFAC_PRECOND_OVERLAP=$1 KFAC_PRECOND_OVERLAP_FRAC=$2 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/b_$1_$2.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1]);print('$1 $2',d['value'],d['ms_per_step'],d['kind_ms'])"
done
