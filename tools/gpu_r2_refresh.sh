#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/refresh
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "block_jacobi or warm or eigh" > gpurun_out/refresh/tests.log 2>&1 || { tail -40 gpurun_out/refresh/tests.log; exit 1; }
tail -1 gpurun_out/refresh/tests.log
timeout -k 10 600 python -u tools/refresh_probe.py --modes 2 --per-bucket 0 > gpurun_out/refresh/probe2.jsonl 2>gpurun_out/refresh/probe2.err || { tail -30 gpurun_out/refresh/probe2.err; cat gpurun_out/refresh/probe2.jsonl; exit 1; }
cat gpurun_out/refresh/probe2.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --baseline 0 > gpurun_out/refresh/bench.json 2>gpurun_out/refresh/bench.err || { tail -20 gpurun_out/refresh/bench.err; exit 1; }
cat gpurun_out/refresh/bench.json
