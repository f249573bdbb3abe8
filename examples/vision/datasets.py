"""Data loaders for the vision examples (reference
``examples/vision/datasets.py:18-151``).

Without network access (and without torchvision) the loaders use, in order:
the CIFAR-10 *binary* release in ``--data-dir`` / an ImageNet-style
``root/<class>/<img>`` tree in ``--train-dir``/``--val-dir`` when present,
otherwise deterministic synthetic data of the real shape (reported as
synthetic in the logs).  Each rank reads its own shard through a
``DistributedSampler``; batches land in pinned memory for async H2D copies.
"""
from __future__ import annotations

import argparse
import os

import torch
from torch.utils.data import DataLoader
from torch.utils.data import Dataset
from torch.utils.data.distributed import DistributedSampler

from distributed_kfac_pytorch_amd.utils.data import CifarBinary
from distributed_kfac_pytorch_amd.utils.data import ImageFolder
from distributed_kfac_pytorch_amd.utils.data import SyntheticImages


def _loaders(train: Dataset, val: Dataset, args: argparse.Namespace
             ) -> tuple[DistributedSampler, DataLoader, DistributedSampler, DataLoader]:
    kw = {'num_workers': args.workers, 'pin_memory': args.cuda}
    if args.workers > 0:
        kw['persistent_workers'] = True
        kw['prefetch_factor'] = 4
    train_sampler = DistributedSampler(train, num_replicas=args.world_size, rank=args.rank,
                                       shuffle=True, seed=args.seed)
    val_sampler = DistributedSampler(val, num_replicas=args.world_size, rank=args.rank,
                                     shuffle=False)
    train_loader = DataLoader(train, batch_size=args.batch_size, sampler=train_sampler,
                              drop_last=True, **kw)
    val_loader = DataLoader(val, batch_size=args.val_batch_size, sampler=val_sampler, **kw)
    return train_sampler, train_loader, val_sampler, val_loader


def get_cifar(args: argparse.Namespace):  # type: ignore[no-untyped-def]
    if args.data_dir and CifarBinary.available(args.data_dir):
        args.data_source = f'cifar10-binary:{args.data_dir}'
        train, val = CifarBinary(args.data_dir, True), CifarBinary(args.data_dir, False)
    else:
        args.data_source = 'synthetic'
        train = SyntheticImages(args.synthetic_train_size, (3, 32, 32), 10, seed=1)
        val = SyntheticImages(args.synthetic_val_size, (3, 32, 32), 10, seed=2)
    return _loaders(train, val, args)


def get_imagenet(args: argparse.Namespace):  # type: ignore[no-untyped-def]
    if args.train_dir and os.path.isdir(args.train_dir):
        args.data_source = f'imagefolder:{args.train_dir}'
        train = ImageFolder(args.train_dir, train=True, size=args.image_size)
        val = ImageFolder(args.val_dir or args.train_dir, train=False, size=args.image_size)
    else:
        args.data_source = 'synthetic'
        shape = (3, args.image_size, args.image_size)
        train = SyntheticImages(args.synthetic_train_size, shape, 1000, seed=1)
        val = SyntheticImages(args.synthetic_val_size, shape, 1000, seed=2)
    return _loaders(train, val, args)


__all__ = ['get_cifar', 'get_imagenet', 'torch']
