#!/bin/bash
# Round 4: find out-of-pool memory read by whole-step graph replays.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
cd /root/repo
timeout -k 10 240 python -u tools/graph_oop_audit.py --no-kfac --steps 3 > gpurun_out/r4a/fp32_nokfac.jsonl 2> gpurun_out/r4a/fp32_nokfac.err && \
timeout -k 10 240 python -u tools/graph_oop_audit.py --steps 3 > gpurun_out/r4a/fp32_kfac.jsonl 2> gpurun_out/r4a/fp32_kfac.err && \
timeout -k 10 240 python -u tools/graph_oop_audit.py --bf16 --steps 3 > gpurun_out/r4a/bf16_kfac.jsonl 2> gpurun_out/r4a/bf16_kfac.err
