#!/bin/bash
# Round 4: the driver's bench command (fp32 + SGD baseline + bf16 secondary
# with replay counts) and smoke, on the suite-verified kernels; a 2-rank gloo
# rehearsal of the multi-rank bench path (both ranks on cuda:0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --same-device --steps 10 --warmup 3 --secondary-bf16 0 --baseline 0 > $O/rehearsal_gloo_w2.json 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/rehearsal_gloo_w2.json').read().strip().splitlines()[-1]);print('w2', d['value'], d['kind_ms'], d.get('params_finite'))"
python3 -c "import json;d=json.loads(open('$O/bench_driver_cmd.json').read().strip().splitlines()[-1]);print(d['value'],d['kind_ms'],d.get('kfac_overhead_ms'),d.get('step_graphs'));print(d['bf16'])"
