#!/bin/bash
# kernel trace of the refresh probe (one sytrd2000 refresh), summarised per queue on the box
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rtrace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/rtrace/raw -o rt -- python3 -u $R/tools/refresh_probe.py --steps 100 --per-bucket 0 --reps 1 --no-acc --mode-list sytrd2000_warm > $R/gpurun_out/rtrace/probe.log 2>&1 || { tail -20 $R/gpurun_out/rtrace/probe.log; exit 1; }
F=$(find $R/gpurun_out/rtrace/raw -name "*kernel_trace.csv" | head -1)
python3 $R/tools/refresh_trace_summary.py $F > $R/gpurun_out/rtrace/summary.txt && cat $R/gpurun_out/rtrace/summary.txt
find $R/gpurun_out/rtrace/raw -name "*.csv" -delete
