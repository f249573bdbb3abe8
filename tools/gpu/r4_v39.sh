#!/bin/bash
# Round 4: poison audit of the bf16 gemm-mode graph under the tuned MIOpen
# database (the twin test goes non-finite at step 3 in that setting).
set -o pipefail
mkdir -p gpurun_out/r4q8
export PYTHONUNBUFFERED=1
timeout -k 10 420 python tools/graph_oop_audit.py --bf16 --miopen-db --conv-mode gemm --deterministic 0 > gpurun_out/r4q8/audit_bf16_gemm_tuned.log 2>&1
rc=$?; echo "rc=$rc"
tail -n 30 gpurun_out/r4q8/audit_bf16_gemm_tuned.log | cut -c1-400
exit $rc
