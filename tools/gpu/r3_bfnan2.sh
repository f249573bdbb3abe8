#!/bin/bash
# Round 3: graph replay vs eager without K-FAC: which model-side fused kernel breaks replay
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3bn2; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 5 --image 224 --batch 32 --fused-sgd 1 --no-kfac $PROBE_ARGS > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }; python3 -c "
import json
for l in open('$O/$name.jsonl'):
    d=json.loads(l); print('$name', d['step'], d['how'], 'param', d['param']['nonfinite'], d['param']['maxrel'], 'grad', d['grad']['maxrel'], 'buf', d['buffer']['maxrel'], 'mom', d['momentum']['maxrel'])
"; }
run bf16_bn1 KFAC_FUSED_BN=1 || exit 1
run bf16_bn0 KFAC_FUSED_BN=0 || exit 1
PROBE_ARGS=--fp32 run fp32_bn1 KFAC_FUSED_BN=1 || exit 1
PROBE_ARGS=--fp32 run fp32_bn0 KFAC_FUSED_BN=0 || exit 1
PROBE_ARGS="--fused-cast 0" run bf16_nocast_bn0 KFAC_FUSED_BN=0 || exit 1
