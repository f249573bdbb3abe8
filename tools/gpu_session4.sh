# implicit-im2col SYRK: kernel + e2e GPU tests, then the 1-GPU bench
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --phase-timing --graphs 0 > gpurun_out/bench_s4_phase.json 2> gpurun_out/bench_s4_phase.err || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_s4.json 2> gpurun_out/bench_s4.err
