#!/bin/bash
# Round 3: bf16 headline bench NaN after the refresh: repeat + bisect knobs
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3bn4; mkdir -p $O
b() { name=$1; shift; env KFAC_BENCH_NANSTEP=1 "$@" timeout -k 10 240 python3 -u bench.py --bf16 --steps 30 --warmup 10 --baseline 0 $BARGS > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], 'finite', d['params_finite'])"; grep "\[nan\]" $O/$name.err | head -1; }
b base1 A=1 || exit 1
b base2 A=1 || exit 1
b syncref KFAC_GRAPH_SYNC_AFTER_REFRESH=1 || exit 1
BARGS="--fused-weight-cast 0" b nocast A=1 || exit 1
b miobn KFAC_FUSED_BN=0 || exit 1
b nofstream KFAC_FACTOR_STREAM=0 || exit 1
BARGS="--graphs 0" b eager A=1 || exit 1
