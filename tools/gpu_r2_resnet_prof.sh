#!/bin/bash
# kernel-level profile of the ResNet-50 K-FAC bench (period window) + bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rn_prof -o rn -- \
  python3 -u $R/bench.py --steps 30 --warmup 5 --baseline 0 > $R/gpurun_out/rn_prof.log 2>&1 || { tail -20 $R/gpurun_out/rn_prof.log; exit 1; }
grep metric $R/gpurun_out/rn_prof.log | cut -c1-300
find $R/gpurun_out/rn_prof -name "*.csv" -size +20M -delete
cd $R && timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > gpurun_out/bench_now.json 2> gpurun_out/bench_now.err || { tail -20 gpurun_out/bench_now.err; exit 1; }
cut -c1-900 gpurun_out/bench_now.json
