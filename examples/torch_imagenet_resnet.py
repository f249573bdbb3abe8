"""ImageNet ResNet training with K-FAC (reference
``examples/torch_imagenet_resnet.py``; defaults from ``:85-198``: per-GPU
batch 32, base LR 0.0125/GPU, 55 epochs, factor update 10, inverse update
100, damping 0.001, label smoothing 0.1).

    torchrun --standalone --nproc-per-node 8 examples/torch_imagenet_resnet.py \
        --train-dir /data/imagenet/train --val-dir /data/imagenet/val

Without ``--train-dir`` it trains on synthetic 3x224x224 data (this is the
configuration ``bench.py`` times).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.utils.training import LabelSmoothLoss  # noqa: E402
from examples import cli  # noqa: E402
from examples.vision import datasets  # noqa: E402
from examples.vision import main  # noqa: E402


def parse_args(argv: list[str] | None = None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description='ImageNet ResNet + K-FAC (MI355X)',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--train-dir', default=None, help='ImageNet train ImageFolder root')
    p.add_argument('--val-dir', default=None, help='ImageNet val ImageFolder root')
    p.add_argument('--model', default='resnet50',
                   choices=['resnet18', 'resnet34', 'resnet50', 'resnet101', 'resnet152'])
    p.add_argument('--image-size', type=int, default=224)
    p.add_argument('--label-smoothing', type=float, default=0.1)
    main.add_common_args(p, batch_size=32, epochs=55, base_lr=0.0125,
                         lr_decay=[25, 35, 40, 45, 50], warmup=5, wd=5e-5)
    cli.add_kfac_args(p, inv_update_steps=100, factor_update_steps=10, damping=0.001)
    cli.add_runtime_args(p)
    args = p.parse_args(argv)
    return args


def main_(argv: list[str] | None = None) -> dict[str, float]:
    args = parse_args(argv)
    return main.run(
        args,
        lambda a: getattr(resnet, a.model)(),
        datasets.get_imagenet,
        LabelSmoothLoss(args.label_smoothing),
    )


if __name__ == '__main__':
    main_()
