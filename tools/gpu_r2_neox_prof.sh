#!/bin/bash
# kernel-level profile of the NeoX-125M K-FAC step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/neox_prof -o neox -- \
  python3 -u $R/tools/bench_neox.py --steps 30 --warmup 2 --no-sgd > $R/gpurun_out/neox_prof.log 2>&1 || { tail -20 $R/gpurun_out/neox_prof.log; exit 1; }
grep metric $R/gpurun_out/neox_prof.log | cut -c1-400
f=$(find $R/gpurun_out/neox_prof -name "*kernel_stats.csv" | head -1)
echo "stats: $f"
head -45 "$f" | cut -c1-200
find $R/gpurun_out/neox_prof -name "*.csv" -size +20M -delete
find $R/gpurun_out/neox_prof -name "*.db" -delete
du -sh $R/gpurun_out
