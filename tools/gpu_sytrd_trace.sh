set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd /tmp && export TMPDIR=/tmp
ONLY=4608 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_sytrd_t" -o run -- python3 "$R/tools/sytrd_time.py" > "$R/gpurun_out/prof_sytrd_t.log" 2>&1 || exit $?
cd "$R"; f=$(find gpurun_out/prof_sytrd_t -name "*kernel_trace.csv"); python3 tools/sytrd_trace_summary.py $f > gpurun_out/sytrd_trace_summary.txt; rc=$?
find gpurun_out/prof_sytrd_t -name "*.csv" -delete; cat gpurun_out/sytrd_trace_summary.txt; exit $rc
