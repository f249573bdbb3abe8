#!/bin/bash
# Round 3 end: eigensolver / kernel GPU tests + smoke + default bench after the refresh defaults changed
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3f5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -10; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench rc=$?"; tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'],d['ms_per_step'],d['kind_ms'],d.get('sgd_ms_per_step'),d['params_finite'],d.get('bf16'))"
