#!/bin/bash
# Round 3: plain-SGD whole-step graph replay, bf16: image size / MIOpen db dependence
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g4; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python -u tools/graph_nan_probe.py --steps 5 --no-kfac --deterministic 0 "$@" > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
bad=[(d['step'], d['how'], d['param']['nonfinite']) for d in recs if d['param']['nonfinite'] or d['grad']['nonfinite']]
print('$name', 'first nonfinite:', bad[:1] if bad else 'none', 'loss', [[round(x,4) for x in d['loss']] for d in recs])"; }
run i64b32 --batch 32 && run i224b32 --image 224 --batch 32 && MIOPEN_USER_DB_PATH=$R/miopen_db run i224b32db --image 224 --batch 32 && run i128b8 --image 128 && echo done
