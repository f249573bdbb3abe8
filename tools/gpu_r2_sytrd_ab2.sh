#!/bin/bash
# eigen refresh: native sytrd tier restricted to the largest factors
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/sytrd_ab2.txt
: > $O
run() {  # label, env..., -- cmd
  local label=$1; shift
  env "$@" > gpurun_out/tmp.json 2> gpurun_out/tmp.err || { tail -20 gpurun_out/tmp.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/tmp.json'));print('$label', d.get('eigen_refresh_ms'), d.get('kind_ms'), d.get('value'))" >> $O
}
run resnet_syevd KFAC_EIGH=auto timeout -k 10 300 python3 bench.py --steps 12 --warmup 2 --baseline 0
run resnet_sytrd4000 KFAC_EIGH=sytrd KFAC_SYTRD_MIN_N=4000 timeout -k 10 300 python3 bench.py --steps 12 --warmup 2 --baseline 0
run resnet_sytrd2000 KFAC_EIGH=sytrd KFAC_SYTRD_MIN_N=2000 timeout -k 10 300 python3 bench.py --steps 12 --warmup 2 --baseline 0
run neox_sytrd3000 KFAC_EIGH=sytrd KFAC_SYTRD_MIN_N=3000 timeout -k 10 300 python3 tools/bench_neox.py --steps 12 --warmup 2 --no-sgd
run neox_sytrd2000 KFAC_EIGH=sytrd KFAC_SYTRD_MIN_N=2000 timeout -k 10 300 python3 tools/bench_neox.py --steps 12 --warmup 2 --no-sgd
cat $O
