# The BASELINE.json configurations besides the headline, each briefly on the
# MI355X (synthetic data): ResNet-32 CIFAR with the INVERSE method, the
# Transformer LM with the EIGEN method, GPT-NeoX-125M K-FAC (mp=1 on one GPU
# and mp=2 with two gloo ranks sharing it), the ImageNet ResNet-50 CLI.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/configs"; cd "$R"
O=gpurun_out/configs
timeout -k 10 300 python3 -u examples/torch_cifar10_resnet.py --kfac-inv-method --epochs 2 --max-steps-per-epoch 60 --synthetic-train-size 16384 --synthetic-val-size 1024 --workers 2 --no-resume --log-dir /tmp/logs_cifar --checkpoint-freq 1000 > $O/cifar_resnet32_inverse.log 2>&1 || { tail -30 $O/cifar_resnet32_inverse.log; exit 1; }
tail -3 $O/cifar_resnet32_inverse.log
timeout -k 10 300 python3 -u examples/torch_language_model.py --kfac --epochs 1 --max-steps-per-epoch 150 --synthetic-tokens 300000 > $O/transformer_lm_eigen.log 2>&1 || { tail -30 $O/transformer_lm_eigen.log; exit 1; }
tail -3 $O/transformer_lm_eigen.log
timeout -k 10 300 python3 -u examples/torch_gpt_neox.py --model 125m --mp 1 --steps 30 --micro-batch 4 --factor-update-steps 5 --inv-update-steps 10 > $O/gpt_neox_125m_mp1.log 2>&1 || { tail -30 $O/gpt_neox_125m_mp1.log; exit 1; }
tail -3 $O/gpt_neox_125m_mp1.log
timeout -k 10 300 python3 -u examples/torch_imagenet_resnet.py --epochs 1 --max-steps-per-epoch 40 --synthetic-train-size 2048 --synthetic-val-size 256 --workers 2 --no-resume --log-dir /tmp/logs_imagenet --checkpoint-freq 1000 --kfac-strategy hybrid-opt --kfac-grad-worker-fraction 0.5 > $O/imagenet_resnet50.log 2>&1 || { tail -30 $O/imagenet_resnet50.log; exit 1; }
tail -3 $O/imagenet_resnet50.log
