#!/bin/bash
# Round 4: bench fp32 default (LPT-ordered precondition GEMMs, host issue
# times) + kernel trace of the plain step; host profile of eager factor
# steps; MIOpen fp32 NHWC wrw solver A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 > $O/bench_fp32.json 2> $O/bench_fp32.err && \
timeout -k 10 300 python -u tools/host_profile.py --kind factor --steps 5 > $O/host_factor_fp32.txt 2> $O/host.err && \
timeout -k 10 300 python -u tools/host_profile.py --kind factor --steps 5 --bf16 > $O/host_factor_bf16.txt 2>> $O/host.err && \
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p3 -o p3 -- python3 bench.py --steps 30 --warmup 10 --baseline 0 --secondary-bf16 0 > /dev/null 2> $O/prof.err && \
python3 tools/trace_gaps.py $(ls /tmp/p3/*.db /tmp/p3/*/*.db 2>/dev/null | head -1) --top 40 > $O/trace_bench.txt 2>&1
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --baseline 1 --secondary-bf16 0 > $O/mw_$name.json 2> $O/mw_$name.err || { echo "$name rc=$?"; return 1; }; }
b base A=1 && b nogtcwrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 && b base2 A=1 && b nogtcwrw2 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
du -sh gpurun_out
timeout -k 10 300 python -u tools/conv1x1_probe.py > $O/conv1x1_fp32.jsonl 2> $O/conv1x1.err
timeout -k 10 300 python -u tools/conv1x1_probe.py --bf16 > $O/conv1x1_bf16.jsonl 2>> $O/conv1x1.err
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 --conv1x1 gemm > $O/bench_fp32_gemm1x1.json 2> $O/bench_gemm1x1.err
