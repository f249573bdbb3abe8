#!/bin/bash
# Round 3: two-stage by bucket population (KFAC_TWOSTAGE_BUCKET_ROWS) on ResNet-50 and NeoX-125M
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3tr; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --baseline 0 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['params_finite'])"; }
b rn_rule A=1 || exit 1
b rn_off KFAC_TWOSTAGE_BUCKET_ROWS=100000000 || exit 1
timeout -k 10 400 python3 -u tools/bench_neox.py > $O/neox_rule.json 2> $O/neox_rule.err || { echo "neox rc=$?"; tail -5 $O/neox_rule.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/neox_rule.json').read().strip().splitlines()[-1]);print('neox_rule', d['value'], d['ms_per_step'], d['kind_ms'], d['eigen_refresh_ms'])"
