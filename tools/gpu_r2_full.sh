#!/bin/bash
# full GPU suite, gloo multi-rank rehearsal (ranks share the GPU), smoke + default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_r2_tests.sh && bash tools/gpu_rehearsal.sh && bash tools/gpu_r2_final_check.sh
