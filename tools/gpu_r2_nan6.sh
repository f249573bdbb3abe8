#!/bin/bash
# is the post-refresh non-finite replay pre-existing? syevd tier, no result check; eager control
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh6
cd $R
for i in 1 2; do
  KFAC_EIGH_CHECK=0 KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh6/c$i.log 2>&1 || { tail -5 gpurun_out/nh6/c$i.log; exit 1; }
  echo "syevd nocheck run $i: $(grep '\[nan\]' gpurun_out/nh6/c$i.log | cut -c1-60) $(grep -o '"params_finite": [a-z]*' gpurun_out/nh6/c$i.log)"
done
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 --graphs 0 > gpurun_out/nh6/e.log 2>&1 || { tail -5 gpurun_out/nh6/e.log; exit 1; }
echo "eager: $(grep '\[nan\]' gpurun_out/nh6/e.log | cut -c1-60) $(grep -o '"params_finite": [a-z]*' gpurun_out/nh6/e.log)"
KFAC_BENCH_NANSTEP=1 KFAC_FACTOR_STREAM=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh6/f.log 2>&1 || { tail -5 gpurun_out/nh6/f.log; exit 1; }
echo "no factor stream: $(grep '\[nan\]' gpurun_out/nh6/f.log | cut -c1-60) $(grep -o '"params_finite": [a-z]*' gpurun_out/nh6/f.log)"
