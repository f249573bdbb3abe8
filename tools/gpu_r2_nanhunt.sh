#!/bin/bash
# intermittent non-finite G factors under rocprofv3: repeat the profiled bench, then without the factor side stream
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/nh
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/nh/r$i -o r -- python3 -u $R/bench.py --steps 30 --warmup 5 --baseline 0 > $R/gpurun_out/nh/r$i.log 2>&1 || { tail -5 $R/gpurun_out/nh/r$i.log; exit 1; }
  echo "profiled run $i: $(grep -c non-finite $R/gpurun_out/nh/r$i.log) non-finite warnings, $(grep -o '"params_finite": [a-z]*' $R/gpurun_out/nh/r$i.log)"
  find $R/gpurun_out/nh -name "*.csv" -delete
done
for i in 1 2; do
  timeout -k 10 300 python3 -u $R/bench.py --steps 30 --warmup 5 --baseline 0 > $R/gpurun_out/nh/p$i.log 2>&1 || { tail -5 $R/gpurun_out/nh/p$i.log; exit 1; }
  echo "plain run $i: $(grep -c non-finite $R/gpurun_out/nh/p$i.log) non-finite warnings, $(grep -o '"params_finite": [a-z]*' $R/gpurun_out/nh/p$i.log) $(grep -o '"value": [0-9.]*' $R/gpurun_out/nh/p$i.log)"
done
