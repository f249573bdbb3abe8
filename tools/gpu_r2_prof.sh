#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/syevd -o syevd -- python3 $R/tools/syevd_profile.py > $R/gpurun_out/prof/syevd.log 2>&1 || { tail -20 $R/gpurun_out/prof/syevd.log; exit 1; }
find $R/gpurun_out/prof/syevd -name "*stats*" | head
