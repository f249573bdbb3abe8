#!/bin/bash
# SYRK kernel tests + fp32 / NeoX factor-step timing after the bf16x3 fp32 path
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "syrk" > gpurun_out/pytest_syrk.log 2>&1 || { tail -30 gpurun_out/pytest_syrk.log; exit 1; }
tail -1 gpurun_out/pytest_syrk.log
timeout -k 10 400 python3 tools/bench_neox.py --steps 30 --warmup 5 > gpurun_out/bench_neox2.json 2> gpurun_out/bench_neox2.err || { tail -20 gpurun_out/bench_neox2.err; exit 1; }
cut -c1-200 gpurun_out/bench_neox2.json; python3 -c "import json;d=json.load(open('gpurun_out/bench_neox2.json'));print(d['value'], d['kind_ms'], d.get('sgd_ms_per_step'), d.get('kfac_overhead_ms'))"
timeout -k 10 300 python3 bench.py --fp32 --steps 30 --warmup 5 > gpurun_out/bench_fp32b.json 2> gpurun_out/bench_fp32b.err || { tail -20 gpurun_out/bench_fp32b.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_fp32b.json').read().strip().splitlines()[-1]);print(d['value'], d['kind_ms'], d.get('sgd_ms_per_step'), d.get('kfac_overhead_ms'))"
