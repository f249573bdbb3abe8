#!/bin/bash
# Round 4: db-mode gross-poison bisection; DDP world-1 graphs; bf16 bench replays.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
cd /root/repo
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs,fwd_bwd,full --miopen-db --deterministic 0 --stages-quiet 1 > gpurun_out/r4h/fp32_db.jsonl 2> gpurun_out/r4h/fp32_db.err && \
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs,fwd_bwd,full --miopen-db --deterministic 0 --stages-quiet 1 --bf16 > gpurun_out/r4h/bf16_db.jsonl 2> gpurun_out/r4h/bf16_db.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --ddp 1 --steps 30 --warmup 5 --baseline 0 --secondary-bf16 0 > gpurun_out/r4h/bench_ddp1.json 2> gpurun_out/r4h/bench_ddp1.err ; \
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python -u bench.py --bf16 --graphs-bf16 1 --steps 40 --warmup 5 --baseline 0 > gpurun_out/r4h/bench_bf16_graphs.json 2> gpurun_out/r4h/bench_bf16.err
