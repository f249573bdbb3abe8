# ResNet-32 CIFAR (synthetic) INVERSE method: fused BN on / off and SGD, to
# compare train / val losses; TensorBoard logs + checkpoints go to /tmp
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/configs"; cd "$R"
O=gpurun_out/configs
run() {
  timeout -k 10 300 python3 -u examples/torch_cifar10_resnet.py --epochs 3 --max-steps-per-epoch 60 --synthetic-train-size 16384 --synthetic-val-size 1024 --workers 2 --no-resume --log-dir /tmp/logs_$1 --checkpoint-freq 1000 "${@:2}" > $O/cifar_$1.log 2>&1 || { tail -30 $O/cifar_$1.log; exit 1; }
  echo "== $1"; grep '"epoch"' $O/cifar_$1.log
}
run inv_fused --kfac-inv-method
KFAC_FUSED_BN=0 run inv_miopen --kfac-inv-method
run sgd_fused --kfac-inv-update-steps 0
run eigen_fused
