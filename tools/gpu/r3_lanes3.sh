#!/bin/bash
# Round 3: bench with 2 / 3 / 4 / 6 hardware queues
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3la3; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --baseline 0 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['params_finite'])"; }
for q in 2 3 4 6 2 3 4 6; do b hwq$q GPU_MAX_HW_QUEUES=$q || exit 1; done
