#!/bin/bash
# Round 4: bench-config interleaved twin (graph vs eager) across a refresh.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
cd /root/repo
A="--image 224 --batch 32 --fused-sgd 1 --num-classes 1000 --inv-steps 100 --factor-steps 10 --lr 0.0125 --pool 8 --steps 130 --print-every 10"
timeout -k 10 400 python -u tools/graph_nan_probe.py $A > gpurun_out/r4f/bf16_kfac.jsonl 2> gpurun_out/r4f/bf16.err && \
timeout -k 10 400 python -u tools/graph_nan_probe.py $A --fp32 > gpurun_out/r4f/fp32_kfac.jsonl 2> gpurun_out/r4f/fp32.err
