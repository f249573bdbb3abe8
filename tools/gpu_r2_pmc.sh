#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace, one pass per
# counter group, each under its own time limit).  Workloads: the ResNet-50
# K-FAC step (INVERSE method: rocSOLVER faults under counter collection, so
# the eigensolver kernels are profiled through the block-Jacobi probe).
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc; mkdir -p $O
pass() {
  local name=$1; shift
  PMC_METHOD=inverse timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/step_$name -o step_$name --pmc "$@" -- python3 $R/tools/pmc_driver.py > $O/step_$name.log 2>&1 || { echo "PASS step_$name FAILED"; grep -v "^    @" $O/step_$name.log | tail -5; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/bj_$name -o bj_$name --pmc "$@" -- python3 $R/tools/bj_probe.py --sizes 1152 --syevd 0 --configs 1:1e-6:4e-6:1 > $O/bj_$name.log 2>&1 || { echo "PASS bj_$name FAILED"; grep -v "^    @" $O/bj_$name.log | tail -5; exit 1; }
  echo "pass $name ok"
}
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum

mkdir -p $R/gpurun_out/pmcsum
python3 $R/tools/pmc_summary.py $O step $R/gpurun_out/pmcsum/pmc_step && python3 $R/tools/pmc_summary.py $O bj $R/gpurun_out/pmcsum/pmc_block_jacobi || exit 1
rm -rf $O
