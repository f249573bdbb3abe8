#!/bin/bash
# ResNet-50 bench A/B of the eigen refresh: batched syevd (default) vs the
# native sytrd tier for n >= KFAC_SYTRD_MIN_N (alternating runs, same box)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for rep in 1 2; do
 for v in syevd sytrd4000 sytrd2000; do
  case $v in
   syevd) e=auto; mn=100000;;
   sytrd4000) e=sytrd; mn=4000;;
   sytrd2000) e=sytrd; mn=2000;;
  esac
  KFAC_EIGH=$e KFAC_SYTRD_MIN_N=$mn timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --baseline 0 > gpurun_out/rab_$v.json 2> gpurun_out/rab_$v.err || { tail -5 gpurun_out/rab_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/rab_$v.json').read().strip().splitlines()[-1]);print('$v', $rep, d['value'], d['ms_per_step'], d['kind_ms'])"
 done
done
