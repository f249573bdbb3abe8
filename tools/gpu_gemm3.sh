# gemm3 kernel tests + e2e GPU tests + bench with the grouped GEMM path.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 300 python3 -m pytest tests/test_gemm3_gpu.py -x -q > gpurun_out/pytest_gemm3.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gemm3.log
tail -5 gpurun_out/pytest_gemm3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --cudnn-benchmark 1 --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
KFAC_PRECOND_GEMM=torch timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --cudnn-benchmark 1 --baseline 0 --phase-timing > gpurun_out/bench_torchgemm.json 2> gpurun_out/bench_torchgemm.err || exit $?
