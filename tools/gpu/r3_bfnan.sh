#!/bin/bash
# Round 3: bisect the bf16 whole-step graph replay divergence at the bench shape
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3bn; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 6 "$@" > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }; python3 -c "
import json
for l in open('$O/$name.jsonl'):
    d=json.loads(l); print('$name', d['step'], d['kind'], d['how'], 'param', d['param']['nonfinite'], d['param']['maxrel'], 'grad', d['grad']['nonfinite'], d['grad']['maxrel'], 'worst', d['worst_layers'][0][:2])
"; }
run nocast --image 224 --batch 32 --fused-sgd 1 --factor-steps 10 --fused-cast 0 || exit 1
run fp32 --image 224 --batch 32 --fused-sgd 1 --factor-steps 10 --fp32 || exit 1
run small --image 64 --batch 8 --fused-sgd 1 --factor-steps 10 || exit 1
run nokfac --image 224 --batch 32 --fused-sgd 1 --no-kfac || exit 1
run nofusedsgd --image 224 --batch 32 --factor-steps 10 || exit 1
