#!/bin/bash
# Round 3: 2- and 4-rank gloo rehearsal of the distributed bench path on one GPU + NeoX-125M bench
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3m; mkdir -p $O
for w in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2950$w bench.py --gpus $w --backend gloo --same-device --steps 20 --warmup 5 --baseline 0 --secondary-bf16 0 > $O/rehearsal_w$w.json 2> $O/rehearsal_w$w.err || { echo "w$w rc=$?"; grep -v "^\s*$" $O/rehearsal_w$w.err | tail -8; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/rehearsal_w$w.json').read().strip().splitlines()[-1]);print('w$w', d['value'], d['n_gpus'], d.get('world_size'), d['kind_ms'], d['params_finite'], d.get('refresh_ms_per_rank'))"
done
timeout -k 10 400 python3 -u tools/bench_neox.py > $O/neox.json 2> $O/neox.err || { echo "neox rc=$?"; tail -5 $O/neox.err; exit 1; }
tail -c 1500 $O/neox.json
