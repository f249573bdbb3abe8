#!/bin/bash
# NeoX native path: GPU tests, NeoX-125M K-FAC vs SGD line, fp32 ResNet-50 row
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_neox.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_neox.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_neox.log
timeout -k 10 400 python -u tools/bench_neox.py --steps 30 --warmup 5 > gpurun_out/bench_neox.json 2> gpurun_out/bench_neox.err || { tail -20 gpurun_out/bench_neox.err; exit 1; }
cat gpurun_out/bench_neox.json
timeout -k 10 300 python -u bench.py --fp32 --steps 30 --warmup 5 > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err || { tail -20 gpurun_out/bench_fp32.err; exit 1; }
cat gpurun_out/bench_fp32.json
