# whole-step graphs: GPU test, then bench with and without graphs (same box)
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_graphs.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --graphs 1 > gpurun_out/bench_graphs.json 2> gpurun_out/bench_graphs.err || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --graphs 0 > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err
