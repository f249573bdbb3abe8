#!/bin/bash
# Round 3: plain-SGD whole-step graph replay (no K-FAC) at 64x64: which op breaks it
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g3; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 5 --no-kfac --deterministic 0 "$@" > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
bad=[(d['step'], d['how'], d['param']['nonfinite']) for d in recs if d['param']['nonfinite'] or d['grad']['nonfinite']]
print('$name', 'first nonfinite:', bad[:1] if bad else 'none', 'param maxrel per step', [round(d['param']['maxrel'] or 0, 6) for d in recs])"; }
run base && run nocast --fused-cast 0 && KFAC_FUSED_BN=0 run mio_bn && run bench1 --benchmark 1 && run fsgd --fused-sgd 1 && run nchw --channels-last 0 && run fp32 --fp32 && echo done
