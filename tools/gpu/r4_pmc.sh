#!/bin/bash
# Round 4: PMC counter passes for the eigensolver kernels (native sytrd chain
# + divide and conquer + back-transform, one 4608 factor), issued from ONE
# host thread (KFAC_EIGH_THREADS=0: round 3's counter runs segfaulted with
# the threaded lane pool).  Raw CSVs stay in /tmp; summaries come back.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
O=/tmp/pmc4; mkdir -p $O
S=$R/gpurun_out/r4o/pmc; mkdir -p $S
export KFAC_EIGH_THREADS=0
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --output-format csv -d $O/eig_$name -o eig_$name --pmc "$@" -- python3 $R/tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > $O/eig_$name.log 2>&1 || { echo "PASS $name FAILED rc=$?"; grep -v "^    @" $O/eig_$name.log | tail -8 > $S/fail_$name.txt; return 1; }
  echo "pass $name ok"
}
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum && \
python3 $R/tools/pmc_summary.py $O eig $S/pmc_eig
ls $S
