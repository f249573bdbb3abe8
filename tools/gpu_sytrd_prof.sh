set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 200 python3 -u tools/sytrd_time.py > gpurun_out/sytrd_time.jsonl 2> gpurun_out/sytrd_time.err || exit $?
ONLY=4608 timeout -k 10 200 python3 -u tools/sytrd_time.py > gpurun_out/sytrd_time_4608.jsonl 2>> gpurun_out/sytrd_time.err || exit $?
cd /tmp && export TMPDIR=/tmp
ONLY=4608 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sytrd" -o run -- python3 "$R/tools/sytrd_time.py" > "$R/gpurun_out/prof_sytrd.log" 2>&1 || exit $?
cd "$R"; cat gpurun_out/sytrd_time.jsonl gpurun_out/sytrd_time_4608.jsonl
find gpurun_out/prof_sytrd -name "*kernel_stats.csv" | head -3
