# native sytrd tier: parity tests, then stage timings (mix and 3 x 4608)
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sytrd" > gpurun_out/sytrd_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sytrd_tests.log; [ $rc = 0 ] || exit $rc
ONLY=4608 timeout -k 10 200 python3 -u tools/sytrd_time.py > gpurun_out/sytrd_time_4608.jsonl 2> gpurun_out/sytrd_time.err || exit $?
timeout -k 10 200 python3 -u tools/sytrd_time.py > gpurun_out/sytrd_time.jsonl 2>> gpurun_out/sytrd_time.err || exit $?
cat gpurun_out/sytrd_time_4608.jsonl gpurun_out/sytrd_time.jsonl
if [ -n "$PROF" ]; then
cd /tmp && export TMPDIR=/tmp
ONLY=4608 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_sytrd" -o run -- python3 "$R/tools/sytrd_time.py" > "$R/gpurun_out/prof_sytrd.log" 2>&1 || exit $?
cd "$R"; find gpurun_out/prof_sytrd -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_sytrd/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f}ms {r['Calls']:>7} {float(r['AverageNs'])/1e3:8.2f}us {r['Name'][:80]}")
PY
fi
