#!/bin/bash
# Kernel trace of a bench.py run, cut to the timed window (bench
# --profile-mark brackets it with identity_kernel launches) and summarised
# by tools/trace_summary.py.
#
#   tools/gpu/profile_bench.sh <tag> [bench.py args ...]
#
# Writes gpurun_out/<tag>/window.txt (per-kernel totals of the window) and
# the bench JSON line; the raw trace stays in /tmp on the box.
set -o pipefail
tag=$1; shift
out=$PWD/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
raw=/tmp/prof_$tag
rm -rf "$raw"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$raw" -o run -- \
  python3 bench.py --profile-mark "$@" > "$out/bench.json" 2> "$out/rocprof.err" || exit $?
csv=$(find "$raw" -name '*kernel_trace.csv' | head -n 1)
[ -n "$csv" ] || { echo "no kernel trace"; exit 1; }
python3 tools/trace_summary.py "$csv" "$out/window.txt" identity_kernel "${STEPS:-20}"
python3 tools/trace_gaps_csv.py "$csv" "$out/gaps.txt" 20
python3 tools/step_kernel_diff.py "$csv" > "$out/step_diff.txt"
[ -z "$KEEP_CSV" ] || gzip -c "$csv" > "$out/kernel_trace.csv.gz"
head -n 30 "$out/window.txt"
