#!/bin/bash
# capture without empty_cache: graph tests, bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cache
cd $R
O=gpurun_out/cache
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphs.py tests/test_e2e_gpu.py > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1 0; do
  KFAC_CAPTURE_EMPTY_CACHE=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/b_$v.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]);print('empty_cache=$v',d['value'],d['ms_per_step'],d['kind_ms'])"
done
