#!/bin/bash
# Round 3: per-kernel profile of the two-stage eigensolver (n = 4608, batch 1 and 3)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ts1 -o ts1 -- python3 $R/tools/twostage_probe.py --sizes 4608 --batch 1 --reps 1 > $R/$O/ts1.log 2>&1 || { echo "prof rc=$?"; tail -5 $R/$O/ts1.log; exit 1; }
cd $R && find $O/ts1 -name "*kernel_stats.csv" | head -2
f=$(find $O/ts1 -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8
