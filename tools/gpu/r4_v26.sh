#!/bin/bash
# Round 4: GPT-NeoX-125M K-FAC vs SGD (tools/bench_neox.py, bf16, seq 2048).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j2; mkdir -p $O
timeout -k 10 900 python3 tools/bench_neox.py > $O/bench_neox.json 2> $O/bench_neox.err || { tail -20 $O/bench_neox.err; exit 1; }
tail -c 1500 $O/bench_neox.json
