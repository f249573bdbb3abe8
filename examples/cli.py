"""Shared command-line plumbing for the example applications.

The reference repeats the same ~100 lines of argparse / process-group setup
in every script (``examples/torch_cifar10_resnet.py:29-283``,
``examples/torch_imagenet_resnet.py:32-283``).  Here they are factored out:

* :func:`add_kfac_args` -- the ``--kfac-*`` flags with the reference names
  and defaults (plus ``--kfac-no-colocate-factors``, fixing SURVEY 5.10 #4
  where ``--kfac-colocate-factors`` could never be switched off, and
  ``--kfac-register-embeddings``);
* :func:`add_runtime_args` -- device / precision / backend / seed flags;
* :func:`init_distributed` -- one process per GPU from the ``torchrun`` env
  (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``), RCCL (``nccl``) on GPUs and
  gloo on CPU, ``cuda:LOCAL_RANK`` pinned before any allocation.
"""
from __future__ import annotations

import argparse
import atexit
import datetime
import os
import random

import numpy as np
import torch
import torch.distributed as dist


def add_kfac_args(p: argparse.ArgumentParser, *, inv_update_steps: int = 100,
                  factor_update_steps: int = 10, damping: float = 0.001) -> None:
    g = p.add_argument_group('K-FAC')
    g.add_argument('--kfac-inv-update-steps', type=int, default=inv_update_steps,
                   help='iterations between inverse/eigen updates (0 disables K-FAC)')
    g.add_argument('--kfac-factor-update-steps', type=int, default=factor_update_steps,
                   help='iterations between factor updates')
    g.add_argument('--kfac-update-steps-alpha', type=float, default=10,
                   help='multiplier applied to the update intervals at each decay epoch')
    g.add_argument('--kfac-update-steps-decay', nargs='+', type=int, default=None,
                   help='epochs at which the update intervals are scaled')
    g.add_argument('--kfac-inv-method', action='store_true', default=False,
                   help='use the inverse method instead of the eigen method')
    g.add_argument('--kfac-factor-decay', type=float, default=0.95,
                   help='running-average coefficient of the factors')
    g.add_argument('--kfac-damping', type=float, default=damping, help='Tikhonov damping')
    g.add_argument('--kfac-damping-alpha', type=float, default=0.5,
                   help='multiplier applied to the damping at each decay epoch')
    g.add_argument('--kfac-damping-decay', nargs='+', type=int, default=None,
                   help='epochs at which the damping is scaled')
    g.add_argument('--kfac-kl-clip', type=float, default=0.001, help='KL clip (<=0 disables)')
    g.add_argument('--kfac-skip-layers', nargs='+', type=str, default=[],
                   help='module name / class-name regexes to skip')
    g.add_argument('--kfac-colocate-factors', dest='kfac_colocate_factors',
                   action='store_true', default=True,
                   help='compute A and G of a layer on the same rank (default)')
    g.add_argument('--kfac-no-colocate-factors', dest='kfac_colocate_factors',
                   action='store_false', help='place A and G independently')
    g.add_argument('--kfac-strategy', type=str, default='comm-opt',
                   choices=['comm-opt', 'mem-opt', 'hybrid-opt'],
                   help='KAISA distribution strategy')
    g.add_argument('--kfac-grad-worker-fraction', type=float, default=0.25,
                   help='grad-worker fraction for hybrid-opt')
    g.add_argument('--kfac-symmetry-aware', action='store_true', default=False,
                   help='communicate only the upper triangle of the factors')
    g.add_argument('--kfac-bucket-cap-mb', type=float, default=25.0,
                   help='allreduce/broadcast bucket size in MB (0 = unbucketed)')
    g.add_argument('--kfac-register-embeddings', action='store_true', default=False,
                   help='also precondition nn.Embedding (diagonal A factor)')


def add_runtime_args(p: argparse.ArgumentParser, *, backend: str = 'nccl') -> None:
    g = p.add_argument_group('runtime')
    g.add_argument('--no-cuda', action='store_true', default=False, help='run on the CPU')
    g.add_argument('--seed', type=int, default=42, help='random seed')
    g.add_argument('--fp16', action='store_true', default=False,
                   help='fp16 autocast + GradScaler (the reference AMP mode)')
    g.add_argument('--precision', choices=['bf16', 'fp16', 'fp32'], default=None,
                   help='autocast dtype on the GPU (default bf16; --fp16 implies fp16)')
    g.add_argument('--backend', type=str, default=backend, choices=['nccl', 'gloo', 'mpi'],
                   help='torch.distributed backend (nccl is RCCL on ROCm)')
    g.add_argument('--verbose', action='store_true', default=None,
                   help='progress bars (default: on for rank 0)')
    g.add_argument('--cudnn-benchmark', type=int, default=1, choices=[0, 1],
                   help='torch.backends.cudnn.benchmark (MIOpen find by timing, the '
                        "reference's setting); 0 = MIOpen's heuristic / database solver")


def resolve_precision(args: argparse.Namespace) -> None:
    """Fill ``args.amp_dtype`` (None = fp32) and ``args.grad_scaler``."""
    prec = args.precision or ('fp16' if args.fp16 else ('bf16' if args.cuda else 'fp32'))
    args.amp_dtype = {'bf16': torch.bfloat16, 'fp16': torch.float16, 'fp32': None}[prec]
    args.precision = prec
    if prec == 'fp16':
        # fp16 needs loss scaling; K-FAC unscales G with the same scaler
        args.grad_scaler = torch.amp.GradScaler('cuda' if args.cuda else 'cpu')
    else:
        args.grad_scaler = None


def _shutdown() -> None:
    """Tear the process group down at exit (RCCL warns about leaked
    communicators otherwise)."""
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def init_distributed(args: argparse.Namespace) -> None:
    """Initialise the process group and the device of this rank.

    Works with ``torchrun`` (env://) and as a plain single process
    (world size 1, no process group needed but one is created so the
    example code path is identical).
    """
    args.cuda = not args.no_cuda and torch.cuda.is_available()
    args.local_rank = int(os.environ.get('LOCAL_RANK', 0))
    if args.cuda:
        torch.cuda.set_device(args.local_rank)
        args.device = torch.device('cuda', args.local_rank)
    else:
        args.device = torch.device('cpu')
        if args.backend == 'nccl':
            args.backend = 'gloo'
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29500')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    if not dist.is_initialized():
        kw = {}
        if args.cuda and args.backend == 'nccl':
            kw['device_id'] = args.device
        dist.init_process_group(args.backend, init_method='env://',
                                timeout=datetime.timedelta(minutes=30), **kw)
        atexit.register(_shutdown)
    args.rank = dist.get_rank()
    args.world_size = dist.get_world_size()
    if args.verbose is None:
        args.verbose = args.rank == 0
    torch.manual_seed(args.seed)
    random.seed(args.seed)
    np.random.seed(args.seed)
    if args.cuda:
        torch.cuda.manual_seed(args.seed)
        torch.backends.cudnn.benchmark = bool(getattr(args, 'cudnn_benchmark', 1))


def log(args: argparse.Namespace, msg: str) -> None:
    if getattr(args, 'rank', 0) == 0:
        print(msg, flush=True)


class ScalarWriter:
    """Rank-0 scalar log: TensorBoard when importable (reference
    ``examples/vision/engine.py:107-114``), else ``scalars.jsonl``."""

    def __init__(self, log_dir: str) -> None:
        os.makedirs(log_dir, exist_ok=True)
        self._tb = None
        try:
            from torch.utils.tensorboard import SummaryWriter
            self._tb = SummaryWriter(log_dir)
        except Exception:  # tensorboard is optional
            self._fh = open(os.path.join(log_dir, 'scalars.jsonl'), 'a', encoding='utf-8')

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        if self._tb is not None:
            self._tb.add_scalar(tag, value, step)
        else:
            import json
            self._fh.write(json.dumps({'tag': tag, 'value': float(value), 'step': step}) + '\n')
            self._fh.flush()

    def close(self) -> None:
        if self._tb is not None:
            self._tb.close()
        else:
            self._fh.close()


def make_log_writer(args: argparse.Namespace) -> ScalarWriter | None:
    if args.rank != 0 or not getattr(args, 'log_dir', None):
        return None
    return ScalarWriter(args.log_dir)
