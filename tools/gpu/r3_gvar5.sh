#!/bin/bash
# Round 3: StepGraphs (eager precondition-phase graphs) vs plain eager; whole-step graphs vs eager; deterministic MIOpen
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3g5; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python -u tools/graph_nan_probe.py --deterministic 1 "$@" > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python -c "
import json
recs=list(map(json.loads, open('$O/$name.jsonl')))
print('$name', [(d['step'], d['how'], d['pbuf']['maxrel'], d['param']['maxrel']) for d in recs])"; }
run stepgraphs --compare stepgraphs --steps 10 && run graphs --steps 18 && run graphs_fp32 --fp32 --steps 18 && echo done
