#!/bin/bash
# Round 3: which MIOpen solver family breaks channels_last graph replays
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3n; mkdir -p $O
run() { name=$1; shift; env $ENVV timeout -k 10 120 python -u tools/graph_sgd_probe.py "$@" > $O/$name.json 2> $O/$name.err; rc=$?; python3 -c "
import json; d=json.loads(open('$O/$name.json').read())
print('$name', [('%.1e'%r['maxrel'], r['n_bad']) for r in d['replays']], d['replays'][-1]['worst'][:2])
" || { echo "$name rc=$rc"; grep -v '^frame' $O/$name.err | grep -i error | head -3; }; [ $rc -eq 0 ] || exit 1; }
for fam in IMPLICIT_GEMM DIRECT WINOGRAD GEMM FFT; do
  for i in 1 2 3; do ENVV="MIOPEN_DEBUG_CONV_$fam=0" run no_${fam}_$i; done
done
for i in 1 2 3; do ENVV="KFAC_X=1" run default_$i; done
