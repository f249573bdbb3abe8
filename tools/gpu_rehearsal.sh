# multi-rank rehearsal of the distributed path on the single GPU (gloo,
# ranks share cuda:0): 2 ranks (one grad worker per layer) and 4 ranks
# (hybrid grid), inverse update every 10 steps, phase timing
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 30 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 8 --image-size 112 --kfac-inv-update-steps 10 --phase-timing > gpurun_out/rehearsal_w2.json 2> gpurun_out/rehearsal_w2.err || { tail -30 gpurun_out/rehearsal_w2.err; exit 1; }
tail -1 gpurun_out/rehearsal_w2.json | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 4 --steps 20 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 4 --image-size 112 --kfac-inv-update-steps 10 > gpurun_out/rehearsal_w4.json 2> gpurun_out/rehearsal_w4.err || { tail -30 gpurun_out/rehearsal_w4.err; exit 1; }
tail -1 gpurun_out/rehearsal_w4.json | cut -c1-400
