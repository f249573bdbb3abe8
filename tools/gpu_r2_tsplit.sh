#!/bin/bash
# largest bucket's tail split over high-priority lanes: tests, refresh probe A/B, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ts
cd $R
O=gpurun_out/ts
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_graphs.py > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/refresh_probe.py --per-bucket 0 --reps 4 --mode-list sytrd2000_warm > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
tail -1 $O/probe.jsonl | cut -c1-250
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['kind_ms'],d.get('sgd_ms_per_step'))"
