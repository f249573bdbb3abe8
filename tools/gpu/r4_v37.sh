#!/bin/bash
# Round 4: how far do two EAGER bf16 twins drift under the tuned MIOpen database
# (nondeterministic solvers), in the twin test's tolerance metrics?
set -o pipefail
mkdir -p gpurun_out/r4q6
export PYTHONUNBUFFERED=1
timeout -k 10 240 python tools/determinism_probe.py --steps 18 --conv1x1 gemm --go-on > gpurun_out/r4q6/eager_gemm_tuned.log 2>&1 && \
timeout -k 10 240 python tools/determinism_probe.py --steps 18 --conv1x1 miopen --go-on > gpurun_out/r4q6/eager_miopen_tuned.log 2>&1
rc=$?; echo "rc=$rc"
cut -c1-400 gpurun_out/r4q6/*.log
exit $rc
