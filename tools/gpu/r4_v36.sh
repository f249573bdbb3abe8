#!/bin/bash
# Round 4: exercise the twin test's tolerance path -- under the bench's tuned
# MIOpen database the twins diverge from step 0 (tools/determinism_probe.py) --
# then the file again as the suite sees it.  A test failure (rc 1) in the first
# step goes on to the second; a timeout or crash ends the script.
set -o pipefail
mkdir -p gpurun_out/r4q5
export PYTHONUNBUFFERED=1
MIOPEN_USER_DB_PATH=$PWD/miopen_db timeout -k 10 600 python -u -m pytest tests/test_graphs_refresh_gpu.py -m gpu -k "gemm or False" -v -s --timeout 300 --timeout-method thread > gpurun_out/r4q5/tuned.log 2>&1
rc=$?; echo "tuned rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_graphs_refresh_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r4q5/default.log 2>&1
  rc=$?; echo "default rc=$rc"
fi
grep -h "twins diverged\|PASSED\|FAILED\|passed\|failed\|Error" gpurun_out/r4q5/*.log
exit $rc
