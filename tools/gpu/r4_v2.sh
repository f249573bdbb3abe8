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
mkdir -p gpurun_out/r4h/eig
timeout -k 10 200 python -u tools/eigh_probe.py --sizes 4608 --count 1 > gpurun_out/r4h/eig/e4608.jsonl 2> gpurun_out/r4h/eig/e.err && \
timeout -k 10 200 python -u tools/eigh_probe.py --sizes 4608 --count 3 --no-acc >> gpurun_out/r4h/eig/e4608.jsonl 2>> gpurun_out/r4h/eig/e.err && \
timeout -k 10 300 python -u tools/eigh_probe.py --mix resnet50 --no-acc >> gpurun_out/r4h/eig/e4608.jsonl 2>> gpurun_out/r4h/eig/e.err && \
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r4h/eig/prof1 -o p1 -- python3 tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /dev/null 2>> gpurun_out/r4h/eig/e.err
O=gpurun_out/r4h/mw
mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --baseline 1 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d.get('sgd_ms_per_step'), d['params_finite'])"; }
b base A=1 && b nogtcwrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 && b base2 A=1 && b nogtcwrw2 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
KFAC_SYTRD_GRAPHS=1 timeout -k 10 200 python -u tools/eigh_probe.py --sizes 4608 --count 1 --no-acc > gpurun_out/r4h/eig/e4608_graphs.jsonl 2>> gpurun_out/r4h/eig/e.err && \
KFAC_SYTRD_GRAPHS=1 timeout -k 10 200 python -u tools/eigh_probe.py --sizes 4608 --count 3 --no-acc >> gpurun_out/r4h/eig/e4608_graphs.jsonl 2>> gpurun_out/r4h/eig/e.err && \
KFAC_SYTRD_GRAPHS=1 timeout -k 10 300 python -u tools/eigh_probe.py --mix resnet50 --no-acc >> gpurun_out/r4h/eig/e4608_graphs.jsonl 2>> gpurun_out/r4h/eig/e.err && \
KFAC_SYTRD_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r4h/eig/prof2 -o p2 -- python3 tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /dev/null 2>> gpurun_out/r4h/eig/e.err
