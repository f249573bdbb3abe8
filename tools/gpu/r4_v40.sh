#!/bin/bash
# Round 4: clean-replay spread of the bf16 gemm-mode graph without the tuned
# MIOpen database, and of the fp32 graph with it (compare r4_v39.sh).
set -o pipefail
mkdir -p gpurun_out/r4q9
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/graph_oop_audit.py --bf16 --conv-mode gemm --deterministic 0 > gpurun_out/r4q9/audit_bf16_gemm_default_db.log 2>&1 && \
timeout -k 10 300 python tools/graph_oop_audit.py --miopen-db --deterministic 0 > gpurun_out/r4q9/audit_fp32_tuned.log 2>&1
rc=$?; echo "rc=$rc"
grep -h '"poison"' gpurun_out/r4q9/*.log
exit $rc
