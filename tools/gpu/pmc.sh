#!/bin/bash
# PMC counter passes over one python program, summarised per kernel.
#
#   tools/gpu/pmc.sh <tag> <prefix> <script.py | binary> [args...]
#
# Four rocprofv3 --pmc passes (each its own run, each under its own time
# limit, no trace domains, at most 4 SQ counters each: an 8-counter pass
# over the bench hung at start-up): sq / sq2 (MFMA busy / MOPS, LDS, waves),
# fetch (FETCH_SIZE), write (WRITE_SIZE, L2 hit / miss).  Raw CSVs stay in /tmp;
# tools/pmc_summary.py writes gpurun_out/<tag>/pmc/<prefix>.{csv,md}.
# The eigensolver's lane pool runs on one host thread (KFAC_EIGH_THREADS=0):
# counter collection serialises dispatches anyway.
set -o pipefail
R="$GRAFT_REPO_ROOT"
tag=$1; prefix=$2; shift 2
# a python script runs under python3, anything else (a built binary) directly
if [[ "$1" == *.py ]]; then prog=(python3 "$R/$1"); else prog=("$R/$1"); fi
shift
cd /tmp && export TMPDIR=/tmp
O=/tmp/pmc_$tag; mkdir -p "$O"
S=$R/gpurun_out/$tag/pmc; mkdir -p "$S"
export KFAC_EIGH_THREADS=0
pass() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --output-format csv -d "$O/${prefix}_$name" -o "${prefix}_$name" \
    --pmc "$@" -- "${prog[@]}" "${ARGS[@]}" > "$O/${prefix}_$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $name failed rc=$rc"
    grep -v "^    @" "$O/${prefix}_$name.log" | tail -20 > "$S/fail_${prefix}_$name.txt"
    return 1
  fi
  echo "pass $name ok"
}
ARGS=("$@")
# progress line every minute (bytes the counter passes have written so far):
# bench-style programs print nothing until they finish
( while sleep 60; do echo "[pmc] $(date +%T) $(du -sk "$O" | cut -f1) KB"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 &&
pass sq2 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum &&
python3 "$R/tools/pmc_summary.py" "$O" "$prefix" "$S/$prefix" sq,sq2,fetch,write &&
ls "$S"
