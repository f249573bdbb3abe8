#!/bin/bash
# first non-finite step of the default bench (diagnostic timing)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh4
cd $R
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh4/a.log 2>&1 || { tail -5 gpurun_out/nh4/a.log; exit 1; }
grep "\[nan\]" gpurun_out/nh4/a.log || echo "no nan step"; grep -o '"params_finite": [a-z]*' gpurun_out/nh4/a.log
KFAC_BENCH_NANSTEP=1 KFAC_EIGH_CHECK=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh4/b.log 2>&1 || { tail -5 gpurun_out/nh4/b.log; exit 1; }
grep "\[nan\]" gpurun_out/nh4/b.log || echo "no nan step (nocheck)"; grep -o '"params_finite": [a-z]*' gpurun_out/nh4/b.log
