#!/bin/bash
# Round 3: kernel trace of the fp32 bench (graphs on): plain K-FAC step vs SGD step
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; O=$R/gpurun_out/r3s2; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o step -- python3 $R/bench.py --steps 30 --warmup 5 --secondary-bf16 0 > $O/bench.json 2> $O/bench.err || { echo "rc=$?"; tail -5 $O/bench.err; exit 1; }
cd $R; f=$(find $O/prof -name "*kernel_trace.csv" | head -1); echo $f
python3 tools/step_kernel_diff.py "$f" > $O/step_diff.txt 2>&1; head -60 $O/step_diff.txt
rm -rf $O/prof
