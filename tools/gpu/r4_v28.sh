#!/bin/bash
# Round 4: DDP at world size 1 over RCCL under torchrun, graphs captured
# through the DDP reducer, on the final default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l2; mkdir -p $O
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --ddp 1 --steps 100 --warmup 10 --baseline 0 --secondary-bf16 0 > $O/bench_ddp1_final.json 2> $O/ddp.err || { tail -20 $O/ddp.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_ddp1_final.json').read().strip().splitlines()[-1]);print(d['value'], d['kind_ms'], d.get('step_graphs'), d['params_finite'])"
