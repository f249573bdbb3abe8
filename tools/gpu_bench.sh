# GPU: full gpu test suite, 1-GPU bench with phase timing, gloo multi-rank
# rehearsal (2 ranks sharing the GPU) of the hybrid-opt graph path.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 30 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 8 --image-size 112 --kfac-inv-update-steps 10 --phase-timing > gpurun_out/rehearsal_w2.json 2> gpurun_out/rehearsal_w2.err
