#!/bin/bash
# refresh variance: host enqueue vs completion per rep, sytrd tier vs syevd
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/var
cd $R
O=gpurun_out/var
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd_tier" > $O/pre.log 2>&1 || { tail -30 $O/pre.log; exit 1; }
timeout -k 10 600 python -u tools/refresh_probe.py --per-bucket 0 --reps 6 --mode-list sytrd2000_warm,auto_warm > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; cat $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd or eigh" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json; python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['kind_ms'],d['inverse_ms_each'])"
