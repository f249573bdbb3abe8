#!/bin/bash
# which model-side feature interacts with the post-refresh replays?
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/nh8
cd $R
d() {
  local tag=$1; shift
  KFAC_BENCH_NANSTEP=1 timeout -k 10 300 "$@" > gpurun_out/nh8/$tag.log 2>&1 || { tail -5 gpurun_out/nh8/$tag.log; exit 1; }
  echo "$tag: $(grep '\[nan\]' gpurun_out/nh8/$tag.log | cut -c1-60) $(grep -o '"params_finite": [a-z]*' gpurun_out/nh8/$tag.log)"
}
d nocast python3 -u bench.py --steps 30 --warmup 5 --baseline 0 --fused-weight-cast 0
d nobn env KFAC_FUSED_BN=0 python3 -u bench.py --steps 30 --warmup 5 --baseline 0
d default python3 -u bench.py --steps 30 --warmup 5 --baseline 0
