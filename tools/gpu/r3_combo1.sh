#!/bin/bash
# Round 3: whole-step graphs vs eager, deterministic: eigensolver tier dependence
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g6; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 300 python -u tools/graph_nan_probe.py --deterministic 1 --steps 10 > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
print('$name', [(d['step'], d['how'], d['pbuf']['maxrel'], d['param']['maxrel']) for d in recs])"; }
run twostage KFAC_X=1 && run sytrd KFAC_EIGH_LARGE=sytrd && run torch KFAC_EIGH=torch && run syevd KFAC_EIGH_LARGE=syevd; echo done
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/ts1 -o ts1 -- python3 $R/tools/twostage_probe.py --sizes 4608 --batch 1 --reps 1 > $R/$O/ts1.log 2>&1 || { echo "prof rc=$?"; tail -5 $R/$O/ts1.log; exit 1; }
cd $R && find $O/ts1 -name "*kernel_stats.csv" | head -2
f=$(find $O/ts1 -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8
