set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_refresh" -o run -- python3 "$R/tools/refresh_probe.py" --per-bucket 0 --reps 1 --mode-list auto_warm > "$R/gpurun_out/prof_refresh.log" 2>&1 || exit $?
cd "$R"; f=$(find gpurun_out/prof_refresh -name "*kernel_trace.csv"); timeout 160 python3 tools/refresh_timeline.py $f > gpurun_out/refresh_timeline.txt; rc=$?
find gpurun_out/prof_refresh -name "*.csv" -delete; cat gpurun_out/refresh_timeline.txt; exit $rc
