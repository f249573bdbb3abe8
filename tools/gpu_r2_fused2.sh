#!/bin/bash
# one-launch-per-column sytrd: correctness first, then chain timing, refresh, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/f2
cd $R
O=gpurun_out/f2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ONLY=4608 timeout -k 10 120 python -u tools/sytrd_time.py > $O/chain_fused.jsonl 2>$O/chain.err || { tail -20 $O/chain.err; exit 1; }
KFAC_SYTRD_FUSED=0 ONLY=4608 timeout -k 10 120 python -u tools/sytrd_time.py > $O/chain_unfused.jsonl 2>>$O/chain.err || { tail -20 $O/chain.err; exit 1; }
cut -c1-200 $O/chain_fused.jsonl $O/chain_unfused.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "eigh" > $O/tests2.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests2.log | head -30; exit 1; }
tail -1 $O/tests2.log
timeout -k 10 400 python -u tools/refresh_probe.py --per-bucket 0 --reps 3 --mode-list sytrd2000_warm > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
cut -c1-300 $O/probe.jsonl
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['kind_ms'])"
