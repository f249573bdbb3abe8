#!/bin/bash
# Round 3: BT2 burst loads; hybrid eigensolver tiers (two-stage >= 4000, chains below) vs chains only
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_twostage_gpu.py > $O/ts_pytest.log 2>&1; rc=$?; tail -3 $O/ts_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/twostage_probe.py --sizes 4608,2304 --batch 3 > $O/ts_probe_b3.jsonl 2> $O/ts_probe_b3.err || { echo "probe rc=$?"; tail -5 $O/ts_probe_b3.err; exit 1; }
cat $O/ts_probe_b3.jsonl
timeout -k 10 600 python -u bench.py --secondary-bf16 0 > $O/bench_hybrid.json 2> $O/bench_hybrid.err || { tail -5 $O/bench_hybrid.err; exit 1; }
KFAC_TWOSTAGE_MIN_N=100000 timeout -k 10 600 python -u bench.py --secondary-bf16 0 --baseline 0 > $O/bench_chains.json 2> $O/bench_chains.err || { tail -5 $O/bench_chains.err; exit 1; }
python -c "
import json
for f in ('bench_hybrid','bench_chains'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['kind_ms'], d.get('eigen_refresh_ms'), d.get('sgd_ms_per_step'), d['params_finite'])"
