#!/bin/bash
# Round 4: new ResNet-50 refresh parity test, then the whole GPU suite.
set -o pipefail
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet50_refresh_parity_gpu.py > $O/parity.log 2>&1
echo "parity rc=$?" >> $O/summary.txt
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest_gpu_all.log 2>&1
echo "all rc=$?" >> $O/summary.txt
tail -5 $O/parity.log; tail -15 $O/pytest_gpu_all.log
