"""Shared driver of the CIFAR-10 and ImageNet ResNet CLIs (reference
``examples/torch_cifar10_resnet.py:260-396`` and
``examples/torch_imagenet_resnet.py:268-405``).

process group -> data -> model (channels_last, DDP over RCCL) ->
SGD + LR schedule + K-FAC (+ its scheduler) -> auto-resume from the newest
``checkpoint_{epoch}`` -> epoch loop (train, test, schedulers, rank-0
checkpoint every ``--checkpoint-freq`` epochs).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import time
from typing import Callable

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.utils.training import latest_checkpoint
from distributed_kfac_pytorch_amd.utils.training import load_checkpoint
from distributed_kfac_pytorch_amd.utils.training import save_checkpoint
from examples import cli
from examples.vision import engine
from examples.vision import optimizers


def add_common_args(p: argparse.ArgumentParser, *, batch_size: int, epochs: int,
                    base_lr: float, lr_decay: list[int], warmup: int, wd: float) -> None:
    p.add_argument('--log-dir', default='./logs/', help='TensorBoard / scalar log dir')
    p.add_argument('--checkpoint-format', default='checkpoint_{epoch}.pth.tar',
                   help='checkpoint file format (under --log-dir)')
    p.add_argument('--checkpoint-freq', type=int, default=5, help='epochs between checkpoints')
    p.add_argument('--batch-size', type=int, default=batch_size, help='per-GPU batch size')
    p.add_argument('--val-batch-size', type=int, default=batch_size, help='per-GPU eval batch')
    p.add_argument('--batches-per-allreduce', type=int, default=1,
                   help='micro-batches accumulated per optimizer step')
    p.add_argument('--epochs', type=int, default=epochs)
    p.add_argument('--base-lr', type=float, default=base_lr, help='LR per GPU')
    p.add_argument('--lr-decay', nargs='+', type=int, default=lr_decay,
                   help='epochs at which the LR decays by 10x')
    p.add_argument('--warmup-epochs', type=int, default=warmup)
    p.add_argument('--momentum', type=float, default=0.9)
    p.add_argument('--weight-decay', type=float, default=wd)
    p.add_argument('--workers', type=int, default=4, help='data-loader workers per rank')
    p.add_argument('--no-channels-last', dest='channels_last', action='store_false',
                   default=True, help='keep NCHW activations')
    p.add_argument('--no-ddp-static-graph', dest='ddp_static_graph', action='store_false',
                   default=True)
    p.add_argument('--ddp-bucket-mb', type=float, default=100.0,
                   help='DDP gradient bucket (large buckets suit xGMI rings)')
    p.add_argument('--synthetic-train-size', type=int, default=50_000)
    p.add_argument('--synthetic-val-size', type=int, default=10_000)
    p.add_argument('--max-steps-per-epoch', type=int, default=None,
                   help='truncate epochs (smoke runs)')
    p.add_argument('--log-interval', type=int, default=10)
    p.add_argument('--graphs', type=int, default=0,
                   help='1: replay training steps from whole-step HIP graphs '
                        '(distributed_kfac_pytorch_amd.graphs.GraphedTrainStep; single-rank '
                        'jobs, or KFAC_STEP_GRAPHS_MULTI=1; no gradient accumulation, no fp16 '
                        'GradScaler); K-FAC second-order updates stay eager')
    p.add_argument('--conv1x1', default='miopen', choices=['miopen', 'gemm'],
                   help='gemm: 1x1 convolutions as GEMMs on the NHWC activation matrix '
                        '(distributed_kfac_pytorch_amd.ops.conv.GemmConv1x1, same values; '
                        "the bench's default, channels_last CUDA only)")
    p.add_argument('--conv-kxk', default='miopen', choices=['miopen', 'gemm'],
                   help='gemm: fp32 3x3 convolutions on the native implicit-GEMM kernel '
                        '(distributed_kfac_pytorch_amd.ops.conv.ImplicitGemmConv2d, bf16x3 '
                        "math ~5e-6 relative; the bench's default, channels_last CUDA only; "
                        'bf16 autocast steps keep MIOpen)')
    p.add_argument('--no-resume', dest='resume', action='store_false', default=True)


def run(args: argparse.Namespace,
        build_model: Callable[[argparse.Namespace], torch.nn.Module],
        get_data: Callable[[argparse.Namespace], tuple],
        loss_func: torch.nn.Module) -> dict[str, float]:
    cli.init_distributed(args)
    cli.resolve_precision(args)
    # the reference scales the LR by world size x accumulation
    # (examples/torch_cifar10_resnet.py:275-277)
    args.base_lr = args.base_lr * args.world_size * args.batches_per_allreduce
    train_sampler, train_loader, _, val_loader = get_data(args)
    cli.log(args, f'data: {args.data_source}; world {args.world_size}; '
                  f'precision {args.precision}; backend {args.backend}')

    model = build_model(args).to(args.device)
    if args.channels_last and args.cuda:
        model = model.to(memory_format=torch.channels_last)
        if getattr(args, 'conv1x1', 'miopen') == 'gemm':
            from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1
            use_gemm_conv1x1(model)
        if getattr(args, 'conv_kxk', 'miopen') == 'gemm':
            from distributed_kfac_pytorch_amd.ops.conv import use_implicit_gemm_conv
            use_implicit_gemm_conv(model)
    if args.world_size > 1:
        ctx = contextlib.nullcontext()
        if getattr(args, 'graphs', 0) and args.cuda:
            # the reducer holds the AccumulateGrad nodes: build it on the
            # stream the graphed steps run on
            from distributed_kfac_pytorch_amd.graphs import step_stream
            ctx = torch.cuda.stream(step_stream(args.device))
        with ctx:
            model = torch.nn.parallel.DistributedDataParallel(
                model,
                device_ids=[args.local_rank] if args.cuda else None,
                bucket_cap_mb=args.ddp_bucket_mb,
                gradient_as_bucket_view=True,
                static_graph=args.ddp_static_graph and args.batches_per_allreduce == 1,
            )
    optimizer, preconditioner, (lr_scheduler, kfac_scheduler) = optimizers.get_optimizer(
        model, args,
    )
    if preconditioner is not None:
        cli.log(args, f'K-FAC: {len(preconditioner._layers)} layers, '
                      f'strategy {args.kfac_strategy}')
    loss_func = loss_func.to(args.device)
    ckpt_fmt = os.path.join(args.log_dir, args.checkpoint_format)
    start_epoch = 0
    found = latest_checkpoint(ckpt_fmt) if args.resume else None
    if found is not None:
        path, epoch = found
        state = load_checkpoint(path, map_location=args.device)
        model.load_state_dict(state['model'])
        optimizer.load_state_dict(state['optimizer'])
        if state.get('lr_scheduler') is not None:
            lr_scheduler.load_state_dict(state['lr_scheduler'])
        if preconditioner is not None and state.get('preconditioner') is not None:
            preconditioner.load_state_dict(state['preconditioner'])
        start_epoch = epoch
        cli.log(args, f'resumed from {path} (epoch {epoch})')
    args.log_writer = cli.make_log_writer(args)
    results: dict[str, float] = {}
    t0 = time.perf_counter()
    for epoch in range(start_epoch, args.epochs):
        results = engine.train(epoch, model, optimizer, preconditioner, loss_func,
                               train_sampler, train_loader, args)
        results.update(engine.test(epoch, model, loss_func, val_loader, args))
        lr_scheduler.step()
        if kfac_scheduler is not None:
            kfac_scheduler.step(step=epoch)
        if (epoch + 1) % args.checkpoint_freq == 0 or epoch + 1 == args.epochs:
            if args.rank == 0:
                save_checkpoint(model, optimizer, preconditioner, lr_scheduler,
                                ckpt_fmt.format(epoch=epoch + 1))
            if args.world_size > 1:
                dist.barrier()
        cli.log(args, json.dumps({'epoch': epoch, **{k: round(v, 5) for k, v in results.items()}}))
    results['wall_s'] = time.perf_counter() - t0
    if args.log_writer is not None:
        args.log_writer.close()
    return results
