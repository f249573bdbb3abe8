#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc/counters.txt 2>&1 || true
grep -iE "^ *(SQ_INSTS_VALU_MFMA|SQ_VALU_MFMA|SQ_LDS|SQ_BUSY|SQ_WAVE|FETCH_SIZE|WRITE_SIZE|TCC_HIT|TCC_MISS|GRBM_GUI|SQ_INSTS_LDS|SQ_INSTS_VALU\b|SQ_ACTIVE)" $GRAFT_REPO_ROOT/gpurun_out/pmc/counters.txt | head -40
wc -l $GRAFT_REPO_ROOT/gpurun_out/pmc/counters.txt
