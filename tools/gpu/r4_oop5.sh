#!/bin/bash
# Round 4: verify the strided-1x1 fix (graph-safe convs) on every probe.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
cd /root/repo
S=conv:layer2.0.downsample.0,conv:layer3.0.downsample.0,conv:layer4.0.downsample.0,grad_api,fwd_bwd,full
timeout -k 10 300 python -u tools/graph_oop_bisect.py --stages $S > gpurun_out/r4e/bisect_safe.jsonl 2> gpurun_out/r4e/bisect_safe.err && \
timeout -k 10 300 python -u tools/graph_oop_bisect.py --stages $S --bf16 > gpurun_out/r4e/bisect_safe_bf16.jsonl 2> gpurun_out/r4e/bisect_safe_bf16.err && \
timeout -k 10 240 python -u tools/graph_oop_audit.py --no-kfac --steps 3 > gpurun_out/r4e/audit_fp32_nokfac.jsonl 2> gpurun_out/r4e/audit1.err && \
timeout -k 10 240 python -u tools/graph_oop_audit.py --bf16 --steps 3 > gpurun_out/r4e/audit_bf16_kfac.jsonl 2> gpurun_out/r4e/audit2.err && \
timeout -k 10 300 python -u tools/graph_nan_probe.py --image 224 --batch 32 --fused-sgd 1 --no-kfac --fp32 --steps 6 > gpurun_out/r4e/interleave_fp32_nokfac_safe.jsonl 2> gpurun_out/r4e/i1.err && \
timeout -k 10 300 python -u tools/graph_nan_probe.py --image 224 --batch 32 --fused-sgd 1 --no-kfac --fp32 --steps 6 --graph-safe 0 > gpurun_out/r4e/interleave_fp32_nokfac_unsafe.jsonl 2> gpurun_out/r4e/i2.err && \
timeout -k 10 300 python -u tools/graph_nan_probe.py --image 224 --batch 32 --fused-sgd 1 --steps 12 > gpurun_out/r4e/interleave_bf16_kfac_safe.jsonl 2> gpurun_out/r4e/i3.err && \
KFAC_BENCH_NANSTEP=1 timeout -k 10 400 python -u bench.py --bf16 --graphs-bf16 1 --steps 40 --warmup 5 --baseline 0 > gpurun_out/r4e/bench_bf16_graphs.json 2> gpurun_out/r4e/bench.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/prof -o kt -- python3 tools/graph_oop_bisect.py --stages conv:layer3.0.downsample.0 --graph-safe 0 > gpurun_out/r4e/prof_unsafe.jsonl 2> gpurun_out/r4e/prof.err
