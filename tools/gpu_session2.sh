# Re-validation after container restore: GPU tests, 1-GPU bench, rocprof of
# the large-n syevd.  Each GPU step has its own limit; failures stop the chain.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out/prof_keep
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/eigprof -o eig -- python3 "$R/tools/eigh_one.py" 4608 3 > "$R/gpurun_out/eig4608.log" 2>&1 || exit $?
find /tmp/eigprof -name "*kernel_stats*.csv" -exec cp {} "$R/gpurun_out/prof_keep/eig4608_kernel_stats.csv" \;
