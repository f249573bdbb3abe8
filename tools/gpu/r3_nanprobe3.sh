#!/bin/bash
# Round 3: isolate the factor-replay -> plain-replay corruption (fp32, deterministic)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3d; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 150 python -u tools/graph_nan_probe.py --steps 7 --fp32 > $O/$name.jsonl 2> $O/$name.err || { echo "$name rc=$?"; tail -3 $O/$name.err; return 1; }; echo "== $name"; python3 -c "
import json,sys
for l in open('$O/$name.jsonl'):
    d=json.loads(l); print(d['step'], d['kind'], 'loss', ['%.5f'%x for x in d['loss']], 'param %.1e pbuf %.1e nf %d'%(d['param']['maxrel'] or 0, d['pbuf']['maxrel'] or 0, d['pbuf']['nonfinite']), d['worst_layers'][0][1])
"; }
run base KFAC_X=1 || exit 1
run plain_only KFAC_GRAPH_KINDS=plain || exit 1
run factor_only KFAC_GRAPH_KINDS=factor || exit 1
run shared_pool KFAC_GRAPH_SHARED_POOL=1 || exit 1
run sync KFAC_GRAPH_SYNC=1 || exit 1
run nofstream KFAC_FACTOR_STREAM=0 || exit 1
run nosplitk KFAC_SYRK_SPLITS=1 || exit 1
run gemm_torch KFAC_PRECOND_GEMM=torch || exit 1
