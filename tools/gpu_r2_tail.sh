#!/bin/bash
# tail of the native eigensolver tier per bucket, then a kernel profile of the default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -u tools/tail_probe.py > gpurun_out/tail_probe.jsonl 2> gpurun_out/tail_probe.err || { tail -20 gpurun_out/tail_probe.err; cat gpurun_out/tail_probe.jsonl; exit 1; }
cat gpurun_out/tail_probe.jsonl
bash tools/gpu_r2_resnet_prof.sh
