#!/bin/bash
# Round 4: db bisection, new GPU tests, DDP world-1 bench on RCCL.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
cd /root/repo
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 > gpurun_out/r4g/fp32_db.jsonl 2> gpurun_out/r4g/fp32_db.err && \
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 --bf16 > gpurun_out/r4g/bf16_db.jsonl 2> gpurun_out/r4g/bf16_db.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_factor_stream_gpu.py tests/test_graphs_refresh_gpu.py > gpurun_out/r4g/pytest.log 2>&1 ; \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --ddp 1 --steps 30 --warmup 5 --baseline 0 --secondary-bf16 0 > gpurun_out/r4g/bench_ddp1.json 2> gpurun_out/r4g/bench_ddp1.err
