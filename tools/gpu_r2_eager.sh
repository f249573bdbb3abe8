#!/bin/bash
# eager steps with persistent gradients (new bench default): finiteness + throughput, with and without StepGraphs
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/eg
cd $R
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/eg/b1.json 2> gpurun_out/eg/b.err || { tail -5 gpurun_out/eg/b.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/eg/b1.json').read().strip().splitlines()[-1]);print('eager persistent',d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'],d.get('sgd_ms_per_step'))"
KFAC_GRAPHS=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/eg/b2.json 2> gpurun_out/eg/b.err || { tail -5 gpurun_out/eg/b.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/eg/b2.json').read().strip().splitlines()[-1]);print('eager persistent, no StepGraphs',d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'],d.get('sgd_ms_per_step'))"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_graphs.py tests/test_e2e_gpu.py > gpurun_out/eg/pytest.log 2>&1 || { tail -30 gpurun_out/eg/pytest.log; exit 1; }
tail -2 gpurun_out/eg/pytest.log
for i in 1 2; do
KFAC_GRAPH_SYNC_AFTER_REFRESH=1 KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --graphs 1 --grad-set-to-none 1 > gpurun_out/eg/s$i.json 2> gpurun_out/eg/s$i.err || { tail -5 gpurun_out/eg/s$i.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/eg/s$i.json').read().strip().splitlines()[-1]);print('graphs + sync after refresh',d['value'],d['params_finite'])"
grep '\[nan\]' gpurun_out/eg/s$i.err || true
done
