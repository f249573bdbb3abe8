#!/bin/bash
# fused sytrd (one launch per column): tests, 3x4608 chain A/B, refresh probe, default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fuse
cd $R
O=gpurun_out/fuse
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd or eigh" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ONLY=4608 timeout -k 10 120 python -u tools/sytrd_time.py > $O/chain_fused.jsonl 2>$O/chain.err || { tail -20 $O/chain.err; exit 1; }
KFAC_SYTRD_FUSE=0 ONLY=4608 timeout -k 10 120 python -u tools/sytrd_time.py > $O/chain_unfused.jsonl 2>>$O/chain.err || { tail -20 $O/chain.err; exit 1; }
cut -c1-200 $O/chain_fused.jsonl $O/chain_unfused.jsonl
timeout -k 10 600 python -u tools/refresh_probe.py --per-bucket 0 --reps 2 --mode-list auto_warm,sytrd2000_warm,sytrd1000_warm,sytrd2000x2000_warm > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; cat $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
