#!/bin/bash
# Round 3: warm-start acceptance test on / off for the refresh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3ac; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --baseline 0 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['params_finite'])"; }
for i in 1 2; do b on$i A=1 || exit 1; b off$i KFAC_EIGH_ACCEPT_MAX_N=0 || exit 1; done
