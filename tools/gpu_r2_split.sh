#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u tools/syevd_split_probe.py > gpurun_out/prof/split.jsonl 2>gpurun_out/prof/split.err || { tail -20 gpurun_out/prof/split.err; exit 1; }
cat gpurun_out/prof/split.jsonl
