#!/bin/bash
# Round 4: finer poison bisection (backward pieces).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
cd /root/repo
timeout -k 10 300 python -u tools/graph_oop_bisect.py --stages grad_api,fc_bwd,stem_bwd,layer4_bwd,head_bwd,fwd_bwd > gpurun_out/r4c/fp32.jsonl 2> gpurun_out/r4c/fp32.err
