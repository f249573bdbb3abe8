# GPU regression check: full -m gpu suite, steady-state K-FAC profile, bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
STEPS=100 TAG=kfac bash tools/gpu_profile.sh || exit $?
cd "$R"
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench.json
