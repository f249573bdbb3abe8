#!/bin/bash
# Round 4: per-conv backward poison bisection.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
cd /root/repo
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs > gpurun_out/r4d/fp32.jsonl 2> gpurun_out/r4d/fp32.err && \
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --bf16 --stages-quiet 1 > gpurun_out/r4d/bf16.jsonl 2> gpurun_out/r4d/bf16.err
