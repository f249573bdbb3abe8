#!/bin/bash
# Round 4: the twin test under the bench's tuned MIOpen database (twins diverge
# at step 0: exercises the one-step tolerance), then the full GPU suite and the
# smoke on the final tree.  A test failure (rc 1) in the first step goes on; a
# timeout or crash ends the script.
set -o pipefail
mkdir -p gpurun_out/r4q7
export PYTHONUNBUFFERED=1
MIOPEN_USER_DB_PATH=$PWD/miopen_db timeout -k 10 400 python -u -m pytest tests/test_graphs_refresh_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r4q7/tuned.log 2>&1
rc=$?; echo "tuned rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 660 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q7/pytest_gpu_all.log 2>&1
  rc=$?; echo "suite rc=$rc"
fi
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4q7/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"
fi
grep -h "diverged\|PASSED\|FAILED\|passed\|failed" gpurun_out/r4q7/*.log | cut -c1-300
exit $rc
