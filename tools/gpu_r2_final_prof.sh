#!/bin/bash
# final evidence: steady-state kernel stats of the default bench, PMC passes of the sytrd chain kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/fp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fp/bench -o b -- python3 -u $R/bench.py --steps 30 --warmup 5 --baseline 0 > $R/gpurun_out/fp/bench.log 2>&1 || { tail -20 $R/gpurun_out/fp/bench.log; exit 1; }
find $R/gpurun_out/fp/bench -name "*kernel_trace.csv" -delete
O=$R/gpurun_out/pmc; mkdir -p $O
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/sy_$name -o sy_$name --pmc "$@" -- python3 $R/tools/sytrd_pmc_driver.py > $O/sy_$name.log 2>&1 || { echo "PASS sy_$name FAILED"; tail -5 $O/sy_$name.log; exit 1; }
  echo "pass $name ok"
}
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
mkdir -p $R/gpurun_out/pmcsum
python3 $R/tools/pmc_summary.py $O sy $R/gpurun_out/pmcsum/pmc_sytrd || exit 1
rm -rf $O
cat $R/gpurun_out/pmcsum/pmc_sytrd.md | head -20
