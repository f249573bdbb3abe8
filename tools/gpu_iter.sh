# Iteration script: GPU tests, GEMM precision sweep, bench (+ phase timing).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python3 tools/bench_gemm.py > gpurun_out/gemm.jsonl 2> gpurun_out/gemm.err || exit $?
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --cudnn-benchmark 1 --baseline 1 > gpurun_out/bench_cudnnbench.json 2> gpurun_out/bench_cudnnbench.err || exit $?
