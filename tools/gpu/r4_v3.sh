#!/bin/bash
# Round 4: eigensolver timing (eager vs graphed chains) + traces, bf16 graph
# bench, DDP world-1 graph capture, db-mode poison bisection.  Large traces
# stay in /tmp on the box; only summaries land in gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
E="python -u tools/eigh_probe.py"
timeout -k 10 200 $E --sizes 4608 --count 1 > $O/eig.jsonl 2> $O/eig.err && \
timeout -k 10 200 $E --sizes 4608 --count 3 --no-acc >> $O/eig.jsonl 2>> $O/eig.err && \
timeout -k 10 300 $E --mix resnet50 --no-acc >> $O/eig.jsonl 2>> $O/eig.err && \
KFAC_SYTRD_GRAPHS=1 timeout -k 10 200 $E --sizes 4608 --count 1 --no-acc > $O/eig_graphs.jsonl 2>> $O/eig.err && \
KFAC_SYTRD_GRAPHS=1 timeout -k 10 200 $E --sizes 4608 --count 3 --no-acc >> $O/eig_graphs.jsonl 2>> $O/eig.err && \
KFAC_SYTRD_GRAPHS=1 timeout -k 10 300 $E --mix resnet50 --no-acc >> $O/eig_graphs.jsonl 2>> $O/eig.err && \
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p1 -o p1 -- python3 tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /dev/null 2>> $O/eig.err && \
python3 tools/trace_gaps.py /tmp/p1/*/p1_results.db > $O/trace_4608_eager.txt 2>&1 || python3 tools/trace_gaps.py $(ls /tmp/p1/*.db /tmp/p1/*/*.db 2>/dev/null | head -1) > $O/trace_4608_eager.txt 2>&1
KFAC_SYTRD_GRAPHS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p2 -o p2 -- python3 tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /dev/null 2>> $O/eig.err && \
python3 tools/trace_gaps.py $(ls /tmp/p2/*.db /tmp/p2/*/*.db 2>/dev/null | head -1) > $O/trace_4608_graphs.txt 2>&1
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python -u bench.py --bf16 --graphs-bf16 1 --steps 40 --warmup 5 --baseline 0 > $O/bench_bf16_graphs.json 2> $O/bench_bf16.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --ddp 1 --steps 30 --warmup 5 --baseline 0 --secondary-bf16 0 > $O/bench_ddp1.json 2> $O/bench_ddp1.err
timeout -k 10 400 python -u tools/graph_oop_bisect.py --stages convs,fwd_bwd,full --miopen-db --deterministic 0 --stages-quiet 1 --bf16 > $O/bisect_bf16_db.jsonl 2> $O/bisect.err
du -sh gpurun_out
