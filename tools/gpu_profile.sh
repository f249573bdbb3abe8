# rocprofv3 kernel-trace/stats of the 1-GPU bench + eigensolver size sweep.
# Only the *_stats.csv summaries are kept (the full trace exceeds the 64 MiB
# gpurun_out budget).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/prof_keep"
timeout -k 10 400 python3 "$R/tools/bench_eigh.py" > "$R/gpurun_out/eigh_sizes.jsonl" 2> "$R/gpurun_out/eigh_sizes.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kfac_prof -o bench -- python3 "$R/bench.py" --steps 100 --warmup 10 --baseline 0 > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
rc=$?
find /tmp/kfac_prof -name "*stats*.csv" -exec cp {} "$R/gpurun_out/prof_keep/" \;
find /tmp/kfac_prof -name "*kernel_trace*.csv" -exec python3 "$R/tools/trace_summary.py" {} "$R/gpurun_out/prof_keep/trace_summary.txt" \;
exit $rc
