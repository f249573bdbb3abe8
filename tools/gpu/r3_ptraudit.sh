#!/bin/bash
# Round 3: host-side pointer audit of capture-built descriptor tables (no replay)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 200 python -u tools/graph_ptr_audit.py --fp32 > $O/audit.jsonl 2> $O/audit.err; rc=$?
echo "rc=$rc"; tail -3 $O/audit.err | cut -c1-300
python3 -c "
import json
for l in open('$O/audit.jsonl'):
    d=json.loads(l)
    if 'at' in d: print(d['at'], 'checked', d['checked'], 'bad', len(d['bad']), d['bad'][:6])
    else: print(d)
"
