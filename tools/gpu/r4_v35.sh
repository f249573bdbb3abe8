#!/bin/bash
# Round 4: bf16 eager step reproducibility under the tuned vs a fresh MIOpen
# database, and with torch.use_deterministic_algorithms.  Exit 0 on mismatch.
set -o pipefail
mkdir -p gpurun_out/r4q4
export PYTHONUNBUFFERED=1
P="timeout -k 10 240 python tools/determinism_probe.py --steps 40"
$P --conv1x1 gemm --db=fresh > gpurun_out/r4q4/eager_gemm_fresh.log 2>&1 && \
$P --conv1x1 miopen --db=fresh > gpurun_out/r4q4/eager_miopen_fresh.log 2>&1 && \
$P --conv1x1 gemm --det-algos > gpurun_out/r4q4/eager_gemm_tuned_det.log 2>&1 && \
$P --conv1x1 gemm --db=fresh --graphed > gpurun_out/r4q4/graphed_gemm_fresh.log 2>&1
rc=$?; echo "rc=$rc"
tail -n 1 gpurun_out/r4q4/*.log
exit $rc
