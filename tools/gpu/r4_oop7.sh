#!/bin/bash
# Round 4: per-conv poison bisection under the bench's MIOpen setup (tuned db,
# non-deterministic algorithms allowed).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
cd /root/repo
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 > gpurun_out/r4g/fp32_db.jsonl 2> gpurun_out/r4g/fp32_db.err && \
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 --bf16 > gpurun_out/r4g/bf16_db.jsonl 2> gpurun_out/r4g/bf16_db.err && \
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages grad_api,fwd_bwd,full --miopen-db --deterministic 0 --bf16 > gpurun_out/r4g/bf16_db_full.jsonl 2> gpurun_out/r4g/bf16_db_full.err
