#!/bin/bash
# cold (step-0) refresh through the native tier with n >= 1000 (and >= 2000 for comparison)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cold
cd $R
O=gpurun_out/cold
timeout -k 10 300 python -u tools/refresh_probe.py --steps 0 --per-bucket 0 --reps 2 --mode-list sytrd2000,sytrd1000 > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; cat $O/probe.jsonl; exit 1; }
cut -c1-300 $O/probe.jsonl
