set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 300 python3 -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench.json | cut -c1-200; grep -o '"sgd_ms_per_step[^,]*\|"phase_ms_per_step.*' gpurun_out/bench.json
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --phase-timing --grad-set-to-none 1 > gpurun_out/bench_none.json 2> gpurun_out/bench_none.err || exit $?
tail -1 gpurun_out/bench_none.json | cut -c1-200; grep -o '"sgd_ms_per_step[^,]*\|"phase_ms_per_step.*' gpurun_out/bench_none.json
