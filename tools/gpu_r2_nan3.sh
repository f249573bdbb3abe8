#!/bin/bash
# bisect: whole-step graphs + native eigensolver tier -> non-finite params
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh3
cd $R
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh3/$tag.log 2>&1 || { tail -5 gpurun_out/nh3/$tag.log; exit 1; }
  echo "$tag: $(grep -o '"params_finite": [a-z]*' gpurun_out/nh3/$tag.log) $(grep -o '"value": [0-9.]*' gpurun_out/nh3/$tag.log)"
}
run default KFAC_NOP=1
run noprio KFAC_SYTRD_PRIORITY=0
run nothreads KFAC_EIGH_THREADS=0
run ormtr KFAC_EIGH_ORMTR=rocsolver
run nocheck KFAC_EIGH_CHECK=0
run nowarm KFAC_EIGH_WARM=0
