#!/bin/bash
# Round 4: sytrd col/symv latency rewrite -- correctness, timing, trace;
# db-mode bf16 poison bisection; DDP world-1 graphs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_eigh_native_gpu.py tests/test_kernels_gpu.py -k "eigh or sytrd or jacobi" > $O/pytest_eigh.log 2>&1 && \
E="python -u tools/eigh_probe.py" && \
timeout -k 10 200 $E --sizes 4608 --count 1 > $O/eig.jsonl 2> $O/eig.err && \
timeout -k 10 200 $E --sizes 4608 --count 3 --no-acc >> $O/eig.jsonl 2>> $O/eig.err && \
timeout -k 10 300 $E --mix resnet50 --no-acc >> $O/eig.jsonl 2>> $O/eig.err && \
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p1 -o p1 -- python3 tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /dev/null 2>> $O/eig.err && \
python3 tools/trace_gaps.py $(ls /tmp/p1/*.db /tmp/p1/*/*.db 2>/dev/null | head -1) > $O/trace_4608.txt 2>&1
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs,fwd_bwd,full --miopen-db --deterministic 0 --stages-quiet 1 --bf16 > $O/bisect_bf16_db.jsonl 2> $O/bisect.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --ddp 1 --steps 30 --warmup 15 --baseline 0 --secondary-bf16 0 > $O/bench_ddp1.json 2> $O/bench_ddp1.err
du -sh gpurun_out
timeout -k 10 300 python -u tools/graph_oop_audit.py --bf16 --steps 3 --miopen-db --deterministic 0 > $O/audit_bf16_db.jsonl 2> $O/audit.err
