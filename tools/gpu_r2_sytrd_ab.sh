#!/bin/bash
# eigen refresh A/B on the NeoX-125M mix: batched syevd vs the native sytrd tier
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for e in auto sytrd auto sytrd; do
  KFAC_EIGH=$e timeout -k 10 300 python3 -u tools/bench_neox.py --steps 12 --warmup 2 --no-sgd > gpurun_out/neox_eigh_$e.json 2> gpurun_out/neox_eigh_$e.err || { tail -20 gpurun_out/neox_eigh_$e.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/neox_eigh_$e.json'));print('$e', d['eigen_refresh_ms'], d['kind_ms'])"
done
