#!/bin/bash
# does the default bench produce non-finite factors under rocprofv3 with the syevd tier too?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pn
KFAC_EIGH_LARGE=syevd timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pn/a -o a -- python3 -u $R/bench.py --steps 30 --warmup 5 --baseline 0 > $R/gpurun_out/pn/syevd.log 2>&1 || { tail -5 $R/gpurun_out/pn/syevd.log; }
grep -c "non-finite" $R/gpurun_out/pn/syevd.log || true
grep "non-finite" $R/gpurun_out/pn/syevd.log | head -3 || true
grep -o '"value": [0-9.]*' $R/gpurun_out/pn/syevd.log || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pn/b -o b -- python3 -u $R/bench.py --steps 30 --warmup 5 --baseline 0 > $R/gpurun_out/pn/sytrd.log 2>&1 || { tail -5 $R/gpurun_out/pn/sytrd.log; }
grep "non-finite" $R/gpurun_out/pn/sytrd.log | head -3 || true
grep -o '"value": [0-9.]*' $R/gpurun_out/pn/sytrd.log || true
find $R/gpurun_out/pn -name "*kernel_trace.csv" -delete
