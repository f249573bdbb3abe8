#!/bin/bash
# Round 3: bench default (100 steps) with 4 vs 8 hardware queues, alternating
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3la2; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --baseline 0 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['inverse_ms_each'], d['params_finite'])"; }
for i in 1 2 3; do
  b hwq8_$i GPU_MAX_HW_QUEUES=8 || exit 1
  b hwq4_$i GPU_MAX_HW_QUEUES=4 || exit 1
done
