#!/bin/bash
# Round 4 (second try: tools/pmc_bisect.py eigh, one host thread): eigensolver counters, n = 4608, one factor, at most 4 counters per
# pass (an 8-counter pass over its ~19k dispatches crashes rocprofv3 while
# every counter alone and 5-counter passes complete: profiles/pmc/
# pmc_counter_bisect_r4.txt).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r4t; mkdir -p $O/pmc
export KFAC_EIGH_THREADS=0
pass() {
  local name=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --output-format csv -d /tmp/pm_$name -o pm --pmc "$@" -- python3 $R/tools/pmc_bisect.py eigh --n 4608 > /tmp/pm_$name.log 2>&1)
  local rc=$?
  echo "$name rc=$rc" >> $O/pmc/summary.txt
  if [ $rc -ne 0 ]; then grep -v "^W2026" /tmp/pm_$name.log | tail -40 > $O/pmc/fail_$name.txt; return 1; fi
  return 0
}
pass busy SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass insts SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
pass l2 TCC_HIT_sum TCC_MISS_sum && \
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
pass mfma SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16
python3 tools/pmc_summary.py /tmp pm $O/pmc/pmc_eig4608 busy,insts,fetch,write,l2,lds,mfma > $O/pmc/summary.json 2> $O/pmc/summary.err || true
du -sh gpurun_out
