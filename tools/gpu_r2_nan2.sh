#!/bin/bash
# which configuration makes the bench parameters non-finite?
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh2
cd $R
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/nh2/$tag.log 2>&1 || { tail -5 gpurun_out/nh2/$tag.log; exit 1; }
  echo "$tag: $(grep -o '"params_finite": [a-z]*' gpurun_out/nh2/$tag.log) $(grep -o '"value": [0-9.]*' gpurun_out/nh2/$tag.log)"
}
timeout -k 10 300 python3 -u bench.py --no-kfac --steps 30 --warmup 5 > gpurun_out/nh2/sgd.log 2>&1 && echo "sgd: $(grep -o '"params_finite": [a-z]*' gpurun_out/nh2/sgd.log)"
run syevd KFAC_EIGH_LARGE=syevd
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 --graphs 0 > gpurun_out/nh2/eager.log 2>&1 && echo "eager: $(grep -o '"params_finite": [a-z]*' gpurun_out/nh2/eager.log)"
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --baseline 0 --fp32 > gpurun_out/nh2/fp32.log 2>&1 && echo "fp32: $(grep -o '"params_finite": [a-z]*' gpurun_out/nh2/fp32.log)"
