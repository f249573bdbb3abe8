# Steady-state rocprofv3 kernel profile of the 1-GPU bench: the timed steps
# are bracketed by marker kernels (bench.py --profile-mark) and
# trace_summary.py cuts that window out and reports per-step busy time,
# per-category and per-kernel totals.  Only summaries are kept (the full
# trace exceeds the gpurun_out budget).
set -o pipefail
R="$GRAFT_REPO_ROOT"
STEPS=${STEPS:-50}
EXTRA=${EXTRA:-}
TAG=${TAG:-kfac}
mkdir -p "$R/gpurun_out/prof_keep"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kfac_prof_$TAG -o bench -- python3 "$R/bench.py" --steps $STEPS --warmup 20 --baseline 0 --profile-mark $EXTRA > "$R/gpurun_out/prof_${TAG}.json" 2> "$R/gpurun_out/prof_${TAG}.err"
rc=$?
find /tmp/kfac_prof_$TAG -name "*kernel_stats*.csv" -exec cp {} "$R/gpurun_out/prof_keep/${TAG}_kernel_stats.csv" \;
find /tmp/kfac_prof_$TAG -name "*kernel_trace*.csv" -exec python3 "$R/tools/trace_summary.py" {} "$R/gpurun_out/prof_keep/${TAG}_steady_summary.txt" identity_kernel $STEPS \;
exit $rc
