#!/bin/bash
# Round 4: symv wave budget per chain (ResNet-50 mix); fp32 bench back on the
# 'strided' graph-safe default; fp32 tuned-db poison bisection (GTC wrw on);
# bf16 eager MIOpen vs GEMM 1x1; kernel stats of bf16 graphs with GEMM 1x1.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
E="python -u tools/eigh_probe.py --mix resnet50 --no-acc"
for w in 0 3072,1024 3072,768,256 2048,1024,512 1024; do
  KFAC_SYTRD_WAVES=$w timeout -k 10 200 $E > $O/mix_w$w.jsonl 2>> $O/eig.err || exit 1
done
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 --secondary-bf16 0 > $O/bench_fp32.json 2> $O/bench_fp32.err || exit 1
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 > $O/bisect_fp32_db.jsonl 2> $O/bisect.err || exit 1
B="python -u bench.py --bf16 --steps 40 --warmup 5 --baseline 0"
timeout -k 10 300 $B --graphs 0 > $O/bf16_eager_miopen.json 2> $O/bf16.err || exit 1
timeout -k 10 300 $B --graphs 0 --conv1x1 gemm > $O/bf16_eager_gemm.json 2>> $O/bf16.err || exit 1
KFAC_GRAPH_SAFE_CONV=gemm timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o p5 -- python3 bench.py --bf16 --graphs-bf16 1 --steps 30 --warmup 5 --baseline 0 > $O/bf16_graphs_gemm_prof.json 2>> $O/bf16.err || exit 1
cp $(ls /tmp/p5/*kernel_stats.csv /tmp/p5/*/*kernel_stats.csv 2>/dev/null | head -1) $O/bf16_graphs_gemm_kernel_stats.csv
du -sh gpurun_out
