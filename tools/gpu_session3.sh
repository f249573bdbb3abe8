# eigh padding: GPU kernel + graph tests, lanes/padding probe, 1-GPU bench
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s3.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/eigh_lanes_probe.py > gpurun_out/eigh_pad.jsonl 2> gpurun_out/eigh_pad.err || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_s3.json 2> gpurun_out/bench_s3.err
