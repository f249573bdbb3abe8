#!/bin/bash
# Round 3: which state departs from eager after the first factor-graph replay
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3b; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 150 python -u tools/graph_nan_probe.py --steps 5 > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }; echo "== $name"; python3 -c "
import json,sys
for l in open('$O/$name.jsonl'):
    d=json.loads(l); print(d['step'], d['kind'], ' '.join(f\"{k}:{v['nonfinite']}/{v['n']},{(v['maxrel'] or 0):.1e}\" for k,v in d.items() if isinstance(v,dict) and 'n' in v))
"; }
run default KFAC_X=1 || exit 1
run gemm_bf16x3 KFAC_PRECOND_GEMM=bf16x3 || exit 1
run gemm_torch KFAC_PRECOND_GEMM=torch || exit 1
run nofstream KFAC_FACTOR_STREAM=0 || exit 1
run syrk_exact KFAC_SYRK_FP32=exact || exit 1
env KFAC_X=1 timeout -k 10 150 python -u tools/graph_nan_probe.py --steps 5 --fp32 > $O/fp32.jsonl 2> $O/fp32.err; echo "fp32 rc=$?"; cut -c1-400 $O/fp32.jsonl
