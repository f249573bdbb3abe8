#!/bin/bash
# Round 4: 2-rank gloo rehearsal of the multi-rank bench path with the final
# default (GEMM 1x1 convolutions), both ranks on cuda:0.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k2; mkdir -p $O
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --backend gloo --same-device --steps 10 --warmup 3 --baseline 0 > $O/rehearsal_gloo_w2_final.json 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/rehearsal_gloo_w2_final.json').read().strip().splitlines()[-1]);print('w2', d['value'], d['kind_ms'], d.get('params_finite'), d['config'].get('conv1x1'), d.get('bf16',{}).get('params_finite'))"
