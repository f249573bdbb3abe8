#!/bin/bash
# Round 3: whole-step graphs vs eager, deterministic: repeatability and eigensolver lanes
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g7; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 300 python -u tools/graph_nan_probe.py --deterministic 1 --steps 6 > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
bad=[d['step'] for d in recs if (d['param']['maxrel'] or 0) != 0 or d['param']['nonfinite']]
print('$name', 'first mismatch step:', bad[:1] if bad else 'none')"; }
for i in 1 2 3; do run def$i KFAC_X=1; done
for i in 1 2 3; do run nothreads$i KFAC_EIGH_THREADS=0 KFAC_EIGH_STREAMS=1; done
for i in 1 2; do run nofactorstream$i KFAC_FACTOR_STREAM=0; done
echo probes done
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ts1 -o ts1 -- python3 $R/tools/twostage_probe.py --sizes 4608 --batch 1 --reps 1 > $R/$O/ts1.log 2>&1 || { echo "prof rc=$?"; tail -5 $R/$O/ts1.log; exit 1; }
cd $R && find $O/ts1 -name "*kernel_stats.csv" | head -2
f=$(find $O/ts1 -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8
