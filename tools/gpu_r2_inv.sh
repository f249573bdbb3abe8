#!/bin/bash
# K-HIP-5 blocked Cholesky tests + ResNet-32 INVERSE (bf16 / fp32) + ResNet-50 INVERSE bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O=gpurun_out/inv; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_graphs.py tests/test_e2e_gpu.py -k "spd or inverse" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  timeout -k 10 300 python3 -u examples/torch_cifar10_resnet.py --epochs 3 --max-steps-per-epoch 60 --synthetic-train-size 16384 --synthetic-val-size 1024 --workers 2 --no-resume --log-dir /tmp/logs_$1 --checkpoint-freq 1000 "${@:2}" > $O/cifar_$1.log 2>&1 || { tail -30 $O/cifar_$1.log; exit 1; }
  echo "== $1"; grep '"epoch"' $O/cifar_$1.log
}
run inv_fp32 --kfac-inv-method --precision fp32
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --baseline 0 --kfac-inv-method > $O/bench_inv.json 2>$O/bench_inv.err || { tail -20 $O/bench_inv.err; exit 1; }
cat $O/bench_inv.json
