#!/bin/bash
# One gpurun command = a chain of GPU steps, each under its own time limit.
#
#   tools/gpu/steps.sh <tag> <seconds> '<command>' [<seconds> '<command>' ...]
#
# Step i writes stdout+stderr to gpurun_out/<tag>/<i>.log; the chain stops at
# the first step that fails, times out or faults (no retries), and the tail
# of that step's log is printed.  Every round's GPU evidence is produced by
# this runner; the logs worth keeping are copied to profiles/.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export PYTHONUNBUFFERED=1
i=0
while [ $# -ge 2 ]; do
  secs=$1; cmd=$2; shift 2
  i=$((i + 1))
  echo "[steps] $i: $cmd (limit ${secs}s)"
  echo "\$ $cmd" > "$out/$i.log"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" >> "$out/$i.log" 2>&1
  rc=$?
  echo "[steps] $i: rc=$rc in $(( $(date +%s) - start ))s"
  if [ $rc -ne 0 ]; then
    tail -n 40 "$out/$i.log" | cut -c1-400
    exit $rc
  fi
  tail -n 3 "$out/$i.log" | cut -c1-400
done
