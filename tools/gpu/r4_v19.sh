#!/bin/bash
# Round 4: symv staging sized to the chain (VT 8/16/32) and 4 waves per SIMD
# for VT <= 16: eigensolver tests + probes; the driver's bench command; smoke.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_eigh_native_gpu.py tests/test_kernels_gpu.py -k "eigh or sytrd" > $O/pytest_eigh.log 2>&1 || { tail -20 $O/pytest_eigh.log; exit 1; }
E="python -u tools/eigh_probe.py --no-acc"
timeout -k 10 200 $E --sizes 4608 --count 1 > $O/eig.jsonl 2> $O/eig.err || exit 1
timeout -k 10 200 $E --sizes 4608 --count 3 >> $O/eig.jsonl 2>> $O/eig.err || exit 1
timeout -k 10 200 $E --sizes 2304 --count 6 >> $O/eig.jsonl 2>> $O/eig.err || exit 1
timeout -k 10 200 $E --mix resnet50 >> $O/eig.jsonl 2>> $O/eig.err || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/eig.jsonl | cut -c1-200; tail -1 $O/smoke.log
python3 -c "import json;d=json.loads(open('$O/bench_driver_cmd.json').read().strip().splitlines()[-1]);print(d['value'],d['kind_ms'],d.get('kfac_overhead_ms'),d['bf16']['value'],d['bf16']['graphs'],d['bf16']['params_finite'])"
