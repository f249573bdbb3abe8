# Baseline: the upstream pure-PyTorch kfac_pytorch (copied into the
# git-ignored _refbench/ for this run only) on the same bench config, plus a
# 2- and 4-rank gloo rehearsal of our distributed path on the single GPU.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out
export KFAC_REFERENCE_PATH="$R/_refbench"
timeout -k 10 500 python bench.py --impl reference --no-channels-last --steps 100 --warmup 10 > gpurun_out/bench_reference.json 2> gpurun_out/bench_reference.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 8 --image-size 112 > gpurun_out/rehearsal_w2.json 2> gpurun_out/rehearsal_w2.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 4 --image-size 112 --kfac-inv-update-steps 10 > gpurun_out/rehearsal_w4.json 2> gpurun_out/rehearsal_w4.err
