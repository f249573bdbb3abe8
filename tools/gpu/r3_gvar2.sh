#!/bin/bash
# Round 3: graph replay NaN: K-FAC off / fused cast off / fp32 / det
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g2; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 6 "$@" > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
bad=[(d['step'], d['how'], {k: d[k]['nonfinite'] for k in ('param','grad','pbuf') if d[k]['nonfinite']}) for d in recs if d['param']['nonfinite'] or d['grad']['nonfinite'] or d['pbuf']['nonfinite']]
print('$name', 'first nonfinite (A):', bad[:1] if bad else 'none', 'last param maxrel', recs[-1]['param']['maxrel'])"; }
run nokfac --deterministic 0 --no-kfac && run nocast --deterministic 0 --fused-cast 0 && run fp32 --deterministic 0 --fp32 && run det1 --deterministic 1 && run det1_fp32 --deterministic 1 --fp32 && echo done
