#!/bin/bash
# full GPU suite (one pytest process)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -60 gpurun_out/pytest_gpu.log | grep -v Warning; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
