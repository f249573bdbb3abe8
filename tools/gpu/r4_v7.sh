#!/bin/bash
# Round 4: sytrd v3 (descriptor pinned in SGPRs, symv staging loads
# unrolled, col gets the symv block count as an argument) correctness +
# timing; tuned-db poison bisection of every conv with MIOpen's GTC NHWC wrw
# solver off (package default) in fp32 and bf16; bf16 1x1 conv probe;
# benches with the 'strided' graph-safe conversion (fp32 default, bf16 graphs).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_eigh_native_gpu.py tests/test_kernels_gpu.py -k "eigh or sytrd" > $O/pytest_eigh.log 2>&1 && \
E="python -u tools/eigh_probe.py" && \
timeout -k 10 200 $E --sizes 4608 --count 1 > $O/eig.jsonl 2> $O/eig.err && \
timeout -k 10 200 $E --sizes 4608 --count 3 --no-acc >> $O/eig.jsonl 2>> $O/eig.err && \
timeout -k 10 300 $E --mix resnet50 --no-acc >> $O/eig.jsonl 2>> $O/eig.err && \
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p1 -o p1 -- python3 tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /dev/null 2>> $O/eig.err && \
python3 tools/trace_gaps.py $(ls /tmp/p1/*.db /tmp/p1/*/*.db 2>/dev/null | head -1) > $O/trace_4608.txt 2>&1
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 --bf16 > $O/bisect_bf16_db_safe.jsonl 2> $O/bisect.err && \
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs --miopen-db --deterministic 0 --stages-quiet 1 > $O/bisect_fp32_db_safe.jsonl 2>> $O/bisect.err
timeout -k 10 200 python -u tools/conv1x1_probe.py --bf16 > $O/conv1x1_bf16.jsonl 2> $O/conv1x1.err
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 > $O/bench_fp32.json 2> $O/bench_fp32.err
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python -u bench.py --bf16 --graphs-bf16 1 --steps 100 --warmup 10 --baseline 0 > $O/bench_bf16_graphs.json 2> $O/bench_bf16.err
du -sh gpurun_out
