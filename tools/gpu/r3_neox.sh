#!/bin/bash
# Round 3: NeoX-125M refresh with the two-stage solver tiers
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3n; mkdir -p $O
n() { name=$1; shift; env "$@" timeout -k 10 400 python3 -u tools/bench_neox.py > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', d['value'], d['ms_per_step'], d['kind_ms'], d['eigen_refresh_ms'])"; }
n ts2000 KFAC_TWOSTAGE_MIN_N=2000 || exit 1
n tsall KFAC_EIGH_LARGE=twostage || exit 1
n ts700 KFAC_TWOSTAGE_MIN_N=700 || exit 1
