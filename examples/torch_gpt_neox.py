"""GPT-NeoX-style language model with tensor-parallel K-FAC (the reference's
``kfac/gpt_neox`` variant; there it needs a DeeperSpeed GPT-NeoX run, here
the model, the topology and the TP layers are part of the framework).

    torchrun --standalone --nproc-per-node 8 examples/torch_gpt_neox.py \
        --model 125m --mp 2 --steps 50

Ranks form a (data x model) grid (``PipeModelDataParallelTopology`` with one
pipeline stage): Megatron column/row-parallel linears split every block over
the ``--mp`` ranks of a model-parallel group, DDP averages gradients over the
data-parallel group, and ``GPTNeoXKFACPreconditioner`` gathers the sharded
activations / gradients to one primary rank per MP group, preconditions the
full matrices there and scatters the result back.  Synthetic token data.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_kfac_pytorch_amd.models.gpt_neox import GPTNeoX  # noqa: E402
from distributed_kfac_pytorch_amd.models.gpt_neox import gpt_neox_pipeline_layers  # noqa: E402
from distributed_kfac_pytorch_amd.neox.pipeline import PipelineModule  # noqa: E402
from distributed_kfac_pytorch_amd.neox.pipeline import allreduce_gradients  # noqa: E402
from distributed_kfac_pytorch_amd.neox.preconditioner import GPTNeoXKFACPreconditioner  # noqa: E402
from distributed_kfac_pytorch_amd.neox.topology import PipeModelDataParallelTopology  # noqa: E402
from examples import cli  # noqa: E402

MODELS = {
    '125m': dict(hidden=768, layers=12, heads=12, vocab=50304),
    'tiny': dict(hidden=64, layers=2, heads=4, vocab=512),
}


def parse_args(argv: list[str] | None = None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description='GPT-NeoX + tensor-parallel K-FAC (MI355X)',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--model', default='tiny', choices=sorted(MODELS))
    p.add_argument('--mp', type=int, default=1, help='model-parallel (tensor-parallel) size')
    p.add_argument('--pp', type=int, default=1, help='pipeline-parallel stages (GPipe schedule)')
    p.add_argument('--micro-batches', type=int, default=1,
                   help='micro-batches per step (pipeline / gradient accumulation)')
    p.add_argument('--seq-len', type=int, default=2048)
    p.add_argument('--micro-batch', type=int, default=8)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--lr', type=float, default=0.05)
    p.add_argument('--no-kfac', dest='kfac', action='store_false', default=True)
    p.add_argument('--factor-update-steps', type=int, default=10)
    p.add_argument('--inv-update-steps', type=int, default=100)
    p.add_argument('--damping', type=float, default=0.003)
    p.add_argument('--kl-clip', type=float, default=0.001)
    p.add_argument('--factor-checkpoint-dir', default=None,
                   help='save K-FAC factors as per-layer files here at the end')
    p.add_argument('--log-interval', type=int, default=5)
    cli.add_runtime_args(p)
    return p.parse_args(argv)


def build_groups(topo: PipeModelDataParallelTopology, rank: int) -> tuple:
    """Create every MP, DP and pipe group in the same order on all ranks."""
    found: dict[str, dist.ProcessGroup | None] = {'model': None, 'data': None, 'pipe': None}
    if not dist.is_initialized():
        return None, None, None
    for axis in ('model', 'data', 'pipe'):
        for ranks in topo.get_axis_comm_lists(axis):
            g = dist.new_group(ranks)
            if rank in ranks:
                found[axis] = g
    return found['model'], found['data'], found['pipe']


def main(argv: list[str] | None = None) -> dict[str, float]:
    args = parse_args(argv)
    cli.init_distributed(args)
    cli.resolve_precision(args)
    if args.world_size % (args.mp * args.pp) != 0:
        raise ValueError(f'world size {args.world_size} is not divisible by --mp x --pp')
    if args.micro_batch % args.micro_batches != 0:
        raise ValueError('--micro-batch must be divisible by --micro-batches')
    dp = args.world_size // (args.mp * args.pp)
    topo = PipeModelDataParallelTopology(num_pp=args.pp, num_mp=args.mp, num_dp=dp)
    mp_group, dp_group, pipe_group = build_groups(topo, args.rank)
    cfg = MODELS[args.model]
    torch.manual_seed(args.seed)
    if args.pp > 1:
        # embedding, blocks and head as separate pipeline layers
        layers = gpt_neox_pipeline_layers(vocab=cfg['vocab'], hidden=cfg['hidden'],
                                          layers=cfg['layers'], heads=cfg['heads'],
                                          group=mp_group)
    else:
        layers = [lambda: GPTNeoX(vocab=cfg['vocab'], hidden=cfg['hidden'], layers=cfg['layers'],
                                  heads=cfg['heads'], group=mp_group)]
    model = PipelineModule(layers, topo, rank=args.rank).to(args.device)
    if args.pp > 1:
        return _train_pipeline(args, model, topo, cfg, mp_group, dp_group, pipe_group)
    if dp > 1:
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[args.local_rank] if args.cuda else None,
            process_group=dp_group,
        )
    optimizer = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9)
    pre = None
    if args.kfac:
        pre = GPTNeoXKFACPreconditioner(
            model.module if dp > 1 else model,
            factor_update_steps=args.factor_update_steps,
            inv_update_steps=args.inv_update_steps,
            damping=args.damping,
            kl_clip=args.kl_clip,
            lr=lambda step: optimizer.param_groups[0]['lr'],
            model_parallel_group=mp_group,
            data_parallel_group=dp_group,
            factor_checkpoint_dir=args.factor_checkpoint_dir,
        )
        cli.log(args, f'K-FAC: {len(pre._layers)} tensor-parallel layers on this rank')
    coord = topo.get_coord(args.rank)
    gen = torch.Generator().manual_seed(args.seed + coord.data)  # same data within an MP group
    tokens_per_step = args.micro_batch * args.seq_len * dp
    cli.log(args, f'model {args.model}; dp {dp} x mp {args.mp}; precision {args.precision}; '
                  f'{tokens_per_step} tokens/step')
    loss_v = float('nan')
    t0 = None
    for step in range(args.steps):
        if step == 1:
            if args.cuda:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
        tokens = torch.randint(0, cfg['vocab'], (args.micro_batch, args.seq_len + 1), generator=gen)
        tokens = tokens.to(args.device)
        optimizer.zero_grad(set_to_none=True)
        ctx = (torch.autocast(args.device.type, dtype=args.amp_dtype)
               if args.amp_dtype is not None else torch.autocast(args.device.type, enabled=False))
        with ctx:
            logits = model(tokens[:, :-1])
        loss = torch.nn.functional.cross_entropy(
            logits.float().flatten(0, 1), tokens[:, 1:].flatten(),
        )
        loss.backward()
        if pre is not None:
            pre.step()
        optimizer.step()
        if (step + 1) % args.log_interval == 0 or step + 1 == args.steps:
            loss_v = loss.item()
            cli.log(args, json.dumps({'step': step + 1, 'loss': round(loss_v, 4)}))
    if args.cuda:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0 if t0 is not None else float('nan')
    timed = max(args.steps - 1, 1)
    out = {'loss': loss_v, 'tokens_per_s': tokens_per_step * timed / elapsed,
           'ms_per_step': elapsed / timed * 1e3}
    cli.log(args, json.dumps(out))
    if pre is not None and args.factor_checkpoint_dir:
        pre.state_dict()  # writes the per-layer factor files
        cli.log(args, f'factors saved under {args.factor_checkpoint_dir}')
    return out


def _train_pipeline(  # type: ignore[no-untyped-def]
    args, model, topo, cfg, mp_group, dp_group, pipe_group,
) -> dict[str, float]:
    """pp > 1: GPipe micro-batch schedule (``PipelineModule.train_batch``),
    data-parallel gradient average per stage, K-FAC per stage with the
    micro-batches as accumulation steps and the KL clip summed over the
    pipeline group."""
    optimizer = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9)
    pre = None
    if args.kfac:
        pre = GPTNeoXKFACPreconditioner(
            model,
            factor_update_steps=args.factor_update_steps,
            inv_update_steps=args.inv_update_steps,
            damping=args.damping,
            kl_clip=args.kl_clip,
            lr=lambda step: optimizer.param_groups[0]['lr'],
            accumulation_steps=args.micro_batches,
            model_parallel_group=mp_group,
            data_parallel_group=dp_group,
            pipeline_parallel_group=pipe_group,
            factor_checkpoint_dir=args.factor_checkpoint_dir,
        )
        cli.log(args, f'K-FAC: {len(pre._layers)} tensor-parallel layers on stage {model.stage_id}')
    coord = topo.get_coord(args.rank)
    gen = torch.Generator().manual_seed(args.seed + coord.data)
    dp = topo.get_dim('data')
    tokens_per_step = args.micro_batch * args.seq_len * dp
    mb = args.micro_batch // args.micro_batches
    act_shape = (mb, args.seq_len, cfg['hidden'])
    cli.log(args, f'model {args.model}; pp {args.pp} x dp {dp} x mp {args.mp}; '
                  f'{args.micro_batches} micro-batches; {tokens_per_step} tokens/step')

    def loss_fn(out: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        return torch.nn.functional.cross_entropy(out.float().flatten(0, 1), y.flatten())

    loss_v = float('nan')
    t0 = None
    for step in range(args.steps):
        if step == 1:
            if args.cuda:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
        tokens = torch.randint(0, cfg['vocab'], (args.micro_batch, args.seq_len + 1), generator=gen)
        tokens = tokens.to(args.device)
        optimizer.zero_grad(set_to_none=False)
        loss = model.train_batch(tokens[:, :-1], tokens[:, 1:], loss_fn, args.micro_batches,
                                 act_shape, autocast_dtype=args.amp_dtype)
        allreduce_gradients(model, dp_group)
        if pre is not None:
            pre.step()
        optimizer.step()
        if (step + 1) % args.log_interval == 0 or step + 1 == args.steps:
            # the loss lives on the last stage: hand it to this rank's first
            # stage over the pipe group so rank 0 logs it
            lt = (loss.detach().float() if loss is not None
                  else torch.zeros((), device=args.device)).reshape(1)
            last = topo.get_rank(pipe=args.pp - 1, data=coord.data, model=coord.model)
            dist.broadcast(lt, src=last, group=pipe_group)
            loss_v = float(lt)
            cli.log(args, json.dumps({'step': step + 1, 'loss': round(loss_v, 4)}))
    if args.cuda:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0 if t0 is not None else float('nan')
    timed = max(args.steps - 1, 1)
    out = {'loss': loss_v, 'tokens_per_s': tokens_per_step * timed / elapsed,
           'ms_per_step': elapsed / timed * 1e3}
    cli.log(args, json.dumps(out))
    if pre is not None and args.factor_checkpoint_dir:
        pre.state_dict()
    return out


if __name__ == '__main__':
    main()
