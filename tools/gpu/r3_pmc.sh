#!/bin/bash
# Round 3: PMC passes (sq / fetch / write, one counter group per run) for the
# eigensolver kernels (native sytrd chains; two-stage n = 4608) and the factor SYRKs
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc3; mkdir -p $O
trap 'rm -rf $O' EXIT  # raw CSVs exceed the 64 MiB copy-back limit
pass() {
  local wl=$1 name=$2; shift 2
  local cmd
  case $wl in
    sytrd) cmd="python3 $R/tools/sytrd_pmc_driver.py" ;;
    ts) cmd="python3 $R/tools/twostage_probe.py --sizes 4608 --batch 1 --reps 1" ;;
    syrk) cmd="python3 $R/tools/syrk_probe.py --reps 2" ;;
  esac
  timeout -s KILL 200 rocprofv3 --output-format csv -d $O/${wl}_$name -o ${wl}_$name --pmc "$@" -- $cmd > $O/${wl}_$name.log 2>&1 || { echo "PASS ${wl}_$name FAILED"; grep -v "^    @" $O/${wl}_$name.log | tail -5; return 1; }
  echo "pass ${wl}_$name ok"
}
for wl in syrk ts; do
  # (the two-stage probe segfaults inside rocprofv3's counter collection on
  # this image: its passes are best effort)
  pass $wl sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || { [ $wl = ts ] && break; exit 1; }
  pass $wl fetch FETCH_SIZE GRBM_GUI_ACTIVE || { [ $wl = ts ] && break; exit 1; }
  pass $wl write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || { [ $wl = ts ] && break; exit 1; }
done
mkdir -p $R/gpurun_out/pmcsum3
for wl in syrk ts; do [ -d $O/${wl}_sq ] && python3 $R/tools/pmc_summary.py $O $wl $R/gpurun_out/pmcsum3/pmc_$wl; done
rm -rf $O
