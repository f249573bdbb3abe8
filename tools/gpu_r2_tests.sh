#!/bin/bash
# Full GPU test suite (no -x: report every failure), then smoke().
set -o pipefail
mkdir -p gpurun_out/tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/tests/pytest_gpu.log | tail -30
exit $rc
