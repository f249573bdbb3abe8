# GPU check script: kernel numerics + e2e tests, then the 1-GPU bench.
# Each GPU step has its own time limit; a failing step stops the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
# assertion failures (rc=1) still allow the bench; anything else stops here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench1.json 2> gpurun_out/bench1.err
