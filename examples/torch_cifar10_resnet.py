"""CIFAR-10 ResNet training with K-FAC (reference
``examples/torch_cifar10_resnet.py``).

    torchrun --standalone --nproc-per-node 8 examples/torch_cifar10_resnet.py \
        --model resnet32 --kfac-strategy hybrid-opt

Reads the CIFAR-10 binary release from ``--data-dir`` if present, otherwise
trains on synthetic 3x32x32 data (no network in this environment).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.models import cifar_resnet  # noqa: E402
from examples import cli  # noqa: E402
from examples.vision import datasets  # noqa: E402
from examples.vision import main  # noqa: E402


def parse_args(argv: list[str] | None = None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description='CIFAR-10 ResNet + K-FAC (MI355X)',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--data-dir', default='/tmp/cifar10', help='CIFAR-10 binary directory')
    p.add_argument('--model', default='resnet32',
                   choices=['resnet20', 'resnet32', 'resnet44', 'resnet56', 'resnet110',
                            'resnet1202'])
    main.add_common_args(p, batch_size=128, epochs=100, base_lr=0.1,
                         lr_decay=[35, 75, 90], warmup=5, wd=5e-4)
    cli.add_kfac_args(p, inv_update_steps=10, factor_update_steps=1, damping=0.003)
    cli.add_runtime_args(p)
    args = p.parse_args(argv)
    args.image_size = 32
    args.synthetic_val_size = min(args.synthetic_val_size, 10_000)
    return args


def main_(argv: list[str] | None = None) -> dict[str, float]:
    args = parse_args(argv)
    from distributed_kfac_pytorch_amd.utils.training import LabelSmoothLoss
    return main.run(
        args,
        lambda a: cifar_resnet.get_model(a.model, num_classes=10),
        datasets.get_cifar,
        LabelSmoothLoss(0.0),
    )


if __name__ == '__main__':
    main_()
