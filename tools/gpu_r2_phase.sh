#!/bin/bash
# bench with phase timing: where the inverse step's time goes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/phase
cd $R
O=gpurun_out/phase
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --baseline 0 --phase-timing > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print(d['value'],d['kind_ms']);print({k:round(v*100,2) for k,v in d['phase_ms_per_step'].items()});print(d['phase_counts'])"
