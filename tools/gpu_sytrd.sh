# native sytrd tier: kernel tests, then the ResNet-50 mix timing (syevd vs sytrd)
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "sytrd or eigh" > gpurun_out/pytest_sytrd.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_sytrd.log
tail -5 gpurun_out/pytest_sytrd.log
[ $rc -eq 0 ] || exit $rc
PROBE_CONFIGS="1:8:100000:syevd,1:8:100000:auto:512,1:8:100000:auto:1000,1:8:100000:auto:200" \
  timeout -k 10 300 python3 -u tools/eigh_lanes_probe.py > gpurun_out/eigh_sytrd.jsonl 2> gpurun_out/eigh_sytrd.err || exit $?
cat gpurun_out/eigh_sytrd.jsonl
