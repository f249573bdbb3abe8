#!/bin/bash
# Round 4: is the bf16 eager step bit-reproducible (gemm 1x1 vs MIOpen 1x1), and
# where does the graphed gemm twin first diverge?  The probe exits 0 on a mismatch.
set -o pipefail
mkdir -p gpurun_out/r4q3
export PYTHONUNBUFFERED=1
timeout -k 10 240 python tools/determinism_probe.py --steps 40 --conv1x1 gemm > gpurun_out/r4q3/eager_gemm.log 2>&1 && \
timeout -k 10 240 python tools/determinism_probe.py --steps 40 --conv1x1 miopen > gpurun_out/r4q3/eager_miopen.log 2>&1 && \
timeout -k 10 240 python tools/determinism_probe.py --steps 40 --conv1x1 gemm --graphed > gpurun_out/r4q3/graphed_gemm.log 2>&1
rc=$?; echo "rc=$rc"
tail -n 1 gpurun_out/r4q3/*.log
exit $rc
