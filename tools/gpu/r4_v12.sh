#!/bin/bash
# Round 4: symv with 8 float4 blocks in flight per row (KFAC_SYTRD_SU=8) vs 4;
# PMC: the round-3/4 'sq' counter pass crashed rocprofv3 while SQ_WAVES,
# SQ_BUSY/WAVE_CYCLES, MFMA busy and GRBM passed -- each remaining counter
# alone (stops at the first crash), then the eigensolver counter passes.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r4r; mkdir -p $O/pmc
E="python -u tools/eigh_probe.py --no-acc"
for su in 4 8; do
  KFAC_SYTRD_SU=$su timeout -k 10 200 $E --sizes 4608 --count 1 > $O/eig_su$su.jsonl 2>> $O/eig.err || exit 1
  KFAC_SYTRD_SU=$su timeout -k 10 200 $E --sizes 4608 --count 3 >> $O/eig_su$su.jsonl 2>> $O/eig.err || exit 1
  KFAC_SYTRD_SU=$su timeout -k 10 200 $E --mix resnet50 >> $O/eig_su$su.jsonl 2>> $O/eig.err || exit 1
done
KFAC_SYTRD_SU=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_eigh_native_gpu.py > $O/pytest_su8.log 2>&1 || exit 1
pass() {
  local name=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --output-format csv -d /tmp/pm_$name -o pm --pmc "$@" -- python3 $R/tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /tmp/pm_$name.log 2>&1)
  local rc=$?
  echo "$name rc=$rc" >> $O/pmc/summary.txt
  if [ $rc -ne 0 ]; then grep -v "^W2026" /tmp/pm_$name.log | tail -80 > $O/pmc/fail_$name.txt; return 1; fi
  cp $(ls /tmp/pm_$name/*counter_collection.csv /tmp/pm_$name/*/*counter_collection.csv 2>/dev/null | head -1) /tmp/cc_$name.csv
  return 0
}
pass ldsbank SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
pass ldsidx SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE && \
pass mfmaf32 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE && \
pass mfmabf16 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE && \
pass busy SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
python3 tools/pmc_summary.py /tmp pm $O/pmc/pmc_eig busy,fetch,write,ldsbank,ldsidx,mfmaf32,mfmabf16 > $O/pmc/summary.json 2> $O/pmc/summary.err || true
ls /tmp/cc_*.csv > $O/pmc/files.txt 2>&1
du -sh gpurun_out
