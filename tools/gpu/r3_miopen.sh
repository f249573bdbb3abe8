#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 300 python -u tools/miopen_graph_probe.py > $O/ops.jsonl 2> $O/ops.err; rc=$?
python3 -c "
import json
for l in open('$O/ops.jsonl'):
    d=json.loads(l); print(d['fmt'], d['case'], ['%.1e'%x for x in d['maxrel']])
"
[ $rc -eq 0 ] || { grep -v '^frame' $O/ops.err | grep -i error | head -3; exit $rc; }
