#!/bin/bash
# Round 3: ResNet-50 refresh step vs hardware queues / chain split (2 refreshes per run)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3la; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 10 --baseline 0 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['inverse_ms_each'], d['params_finite'])"; }
b default A=1 || exit 1
b hwq4 GPU_MAX_HW_QUEUES=4 || exit 1
b hwq16 GPU_MAX_HW_QUEUES=16 || exit 1
b split3 KFAC_SYTRD_SPLIT=4000,2000,1000 || exit 1
b split1 KFAC_SYTRD_SPLIT=1000 || exit 1
