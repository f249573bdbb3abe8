#!/bin/bash
# NeoX-125M K-FAC vs SGD with the native large-n tier vs syevd; ResNet-50 fp32 row
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/neox2
cd $R
O=gpurun_out/neox2
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/bench_neox.py --steps 30 --warmup 5 > $O/neox_sytrd.json 2> $O/neox.err || { tail -20 $O/neox.err; exit 1; }
tail -1 $O/neox_sytrd.json | cut -c1-600
KFAC_EIGH_LARGE=syevd timeout -k 10 400 python -u tools/bench_neox.py --steps 30 --warmup 5 > $O/neox_syevd.json 2> $O/neox.err || { tail -20 $O/neox.err; exit 1; }
tail -1 $O/neox_syevd.json | cut -c1-600
timeout -k 10 300 python -u bench.py --fp32 --steps 30 --warmup 5 > $O/bench_fp32.json 2> $O/bench_fp32.err || { tail -20 $O/bench_fp32.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_fp32.json').read().strip().splitlines()[-1]);print('fp32',d['value'],d['ms_per_step'],d['kind_ms'],d.get('sgd_ms_per_step'))"
timeout -k 10 300 python -u bench.py --kfac-inv-method --steps 30 --warmup 5 > $O/bench_inv.json 2> $O/bench_inv.err || { tail -20 $O/bench_inv.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_inv.json').read().strip().splitlines()[-1]);print('inverse',d['value'],d['ms_per_step'],d['kind_ms'])"
