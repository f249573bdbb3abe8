#!/bin/bash
# Round 3: graph vs eager with deterministic MIOpen: which stage departs first
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3c; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 150 python -u tools/graph_nan_probe.py --steps 5 $EXTRA > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }; echo "== $name"; python3 -c "
import json,sys
for l in open('$O/$name.jsonl'):
    d=json.loads(l); print(d['step'], d['kind'], 'loss', ['%.5f'%x for x in d['loss']], ' '.join(f\"{k}:{v['nonfinite']},{(v['maxrel'] or 0):.1e}\" for k,v in d.items() if isinstance(v,dict) and 'n' in v)); print('   worst', d['worst_layers'])
"; }
EXTRA="--fp32" run fp32_det KFAC_X=1 || exit 1
EXTRA="" run bf16_det KFAC_X=1 || exit 1
EXTRA="" run bf16_nosplit KFAC_SYRK_SPLITS=1 || exit 1
EXTRA="--fused-cast 0" run bf16_nocast KFAC_FUSED_BN=0 || exit 1
