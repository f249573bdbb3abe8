#!/bin/bash
# Round 4: per-stage poison bisection of whole-step graph replays.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
cd /root/repo
timeout -k 10 300 python -u tools/graph_oop_bisect.py > gpurun_out/r4b/fp32_bn1.jsonl 2> gpurun_out/r4b/fp32_bn1.err && \
timeout -k 10 300 python -u tools/graph_oop_bisect.py --fused-bn 0 > gpurun_out/r4b/fp32_bn0.jsonl 2> gpurun_out/r4b/fp32_bn0.err
