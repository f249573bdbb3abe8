set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 300 python3 -m pytest tests/test_gemm3_gpu.py -x -q > gpurun_out/pytest_gemm3.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gemm3.log
tail -3 gpurun_out/pytest_gemm3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/bench_gemm3.py > gpurun_out/gemm3.json 2> gpurun_out/gemm3.err || exit $?
cat gpurun_out/gemm3.json
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench.json
