#!/bin/bash
# bench A/B: sytrd chain HIP graphs on/off (alternating), with phase timing
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/gab
cd $R
O=gpurun_out/gab
for v in 1 first 0 1 first 0; do
  KFAC_SYTRD_GRAPHS=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 --phase-timing > $O/b_$v.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]);print('graphs=$v',d['value'],d['kind_ms'],'inverse_phase',round(d['phase_ms_per_step']['inverse']*100,1))"
done
