#!/bin/bash
# sytrd tier: segmented multi-chain + blocked back-transform; tests, refresh probe, bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/chains
cd $R
O=gpurun_out/chains
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd or eigh" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/refresh_probe.py --per-bucket 0 --reps 2 --mode-list auto_warm,sytrd1000_warm,sytrd500_warm,sytrd256_warm,sytrd1000x4000-2000_warm,sytrd500x4000-2000_warm,sytrd1000x2000_warm,sytrd500x4000-1500_warm > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; cat $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
KFAC_EIGH=sytrd KFAC_SYTRD_MIN_N=1000 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/bench_sytrd.json 2> $O/bench_sytrd.err || { tail -20 $O/bench_sytrd.err; exit 1; }
cut -c1-700 $O/bench_sytrd.json
