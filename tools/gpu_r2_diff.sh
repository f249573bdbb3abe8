#!/bin/bash
# kernel trace of the default bench (K-FAC + SGD baseline in one process): plain K-FAC step vs SGD step diff
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/diff
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/diff/raw -o d -- python3 -u $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/diff/bench.log 2>&1 || { tail -20 $R/gpurun_out/diff/bench.log; exit 1; }
F=$(find $R/gpurun_out/diff/raw -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_kernel_diff.py $F > $R/gpurun_out/diff/diff.txt && cat $R/gpurun_out/diff/diff.txt
find $R/gpurun_out/diff/raw -name "*.csv" -delete
