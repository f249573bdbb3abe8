#!/bin/bash
# Round 4 final check: the driver's bench command twice on the new default
# (GEMM 1x1 convolutions), then the whole GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_driver_cmd_$i.json').read().strip().splitlines()[-1]);print($i, d['value'],d['kind_ms'],d.get('sgd_ms_per_step'),d.get('kfac_overhead_ms'),d.get('step_graphs'));print(d['bf16']['value'], d['bf16']['kind_ms'], d['bf16']['step_graphs'], d['bf16']['params_finite'])"
done
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest_gpu_all.log 2>&1
echo "suite rc=$?"; tail -3 $O/pytest_gpu_all.log
