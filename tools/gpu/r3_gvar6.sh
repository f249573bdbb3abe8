#!/bin/bash
# Round 3: whole-step graphs vs eager, deterministic: eigensolver tier dependence
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g6; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 300 python -u tools/graph_nan_probe.py --deterministic 1 --steps 10 > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
print('$name', [(d['step'], d['how'], d['pbuf']['maxrel'], d['param']['maxrel']) for d in recs])"; }
run twostage KFAC_X=1 && run sytrd KFAC_EIGH_LARGE=sytrd && run torch KFAC_EIGH=torch && run syevd KFAC_EIGH_LARGE=syevd && echo done
