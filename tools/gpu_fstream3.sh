set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 120 --timeout-method thread -k "side_stream or graph_replay" > gpurun_out/pytest_fs.log 2>&1 || { tail -40 gpurun_out/pytest_fs.log; exit 1; }
tail -2 gpurun_out/pytest_fs.log
bash tools/gpu_rehearsal.sh
