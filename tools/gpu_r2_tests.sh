#!/bin/bash
# full GPU suite (one pytest process) + 2-rank same-GPU rehearsal of the packed path
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 30 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 8 --image-size 112 --kfac-inv-update-steps 10 > gpurun_out/rehearsal_w2_packed.json 2> gpurun_out/rehearsal_w2_packed.err || { tail -30 gpurun_out/rehearsal_w2_packed.err; exit 1; }
tail -1 gpurun_out/rehearsal_w2_packed.json | cut -c1-600
