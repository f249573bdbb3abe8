"""Transformer language model with K-FAC (reference
``examples/torch_language_model.py``; defaults ``:35-173``: d_model 256,
d_hid 256, 4 heads, 2 layers, seq_len 64, batch 20, lr 20, ReduceLROnPlateau,
skip ``embedding``/``decoder``/``self_attn``).

    torchrun --standalone --nproc-per-node 8 examples/torch_language_model.py \
        --kfac --dataset wikitext2 --data-dir /data/wikitext-2

Additions: ``--register-embeddings`` preconditions the token embedding with
the diagonal-A K-FAC layer (drop ``embedding`` from ``--skip-layers`` to use
it), bf16 autocast on the GPU, and synthetic data when no local text exists.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.transformer import TransformerLM  # noqa: E402
from examples import cli  # noqa: E402
from examples.language import dataset as lm_data  # noqa: E402
from examples.language import engine  # noqa: E402


def parse_args(argv: list[str] | None = None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description='Transformer LM + K-FAC (MI355X)',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--embedding-dim', type=int, default=256)
    p.add_argument('--hidden-dim', type=int, default=256)
    p.add_argument('--attention-heads', type=int, default=4)
    p.add_argument('--layers', type=int, default=2)
    p.add_argument('--dropout', type=float, default=0.2)
    p.add_argument('--dataset', default='penntreebank',
                   choices=['penntreebank', 'wikitext2', 'wikitext103'])
    p.add_argument('--data-dir', '--download-dir', dest='data_dir', default=None,
                   help='directory with train/valid/test text files')
    p.add_argument('--seq-len', type=int, default=64)
    p.add_argument('--batch-size', type=int, default=20)
    p.add_argument('--epochs', type=int, default=20)
    p.add_argument('--lr', type=float, default=20.0)
    p.add_argument('--clip', type=float, default=0.5, help='grad-norm clip before K-FAC')
    p.add_argument('--synthetic-tokens', type=int, default=1_000_000)
    p.add_argument('--max-steps-per-epoch', type=int, default=None)
    p.add_argument('--kfac', action='store_true', default=False, help='enable K-FAC')
    p.add_argument('--inv-update-steps', type=int, default=10)
    p.add_argument('--factor-update-steps', type=int, default=1)
    p.add_argument('--factor-decay', type=float, default=0.95)
    p.add_argument('--damping', type=float, default=0.003)
    p.add_argument('--kl-clip', type=float, default=0.001)
    p.add_argument('--skip-layers', nargs='+', default=['embedding', 'decoder', 'self_attn'])
    p.add_argument('--strategy', default='comm_opt',
                   choices=['comm_opt', 'mem_opt', 'hybrid_opt'])
    p.add_argument('--register-embeddings', action='store_true', default=False)
    cli.add_runtime_args(p, backend='nccl')
    return p.parse_args(argv)


def main(argv: list[str] | None = None) -> dict[str, float]:
    args = parse_args(argv)
    cli.init_distributed(args)
    cli.resolve_precision(args)
    logging.basicConfig(format='[%(asctime)s] %(levelname)-5s (%(name)s): %(message)s',
                        level=logging.INFO if args.rank == 0 else logging.ERROR,
                        stream=sys.stdout)
    data = lm_data.get_dataset(
        args.dataset, args.data_dir, seq_len=args.seq_len, batch_size=args.batch_size,
        rank=args.rank, world_size=args.world_size, cuda=args.cuda,
        synthetic_tokens=args.synthetic_tokens,
    )
    cli.log(args, f'data: {data.source}; world {args.world_size}; precision {args.precision}')
    model: torch.nn.Module = TransformerLM(
        ntoken=data.vocab_size, d_model=args.embedding_dim, nhead=args.attention_heads,
        d_hid=args.hidden_dim, nlayers=args.layers, dropout=args.dropout,
    ).to(args.device)
    if args.world_size > 1:
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[args.local_rank] if args.cuda else None,
        )
    criterion = torch.nn.CrossEntropyLoss()
    optimizer = torch.optim.SGD(model.parameters(), lr=args.lr)
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(
        optimizer, factor=0.1, patience=2, min_lr=1e-4,
    )
    preconditioner = None
    if args.kfac:
        preconditioner = kfac.KFACPreconditioner(
            model,
            factor_update_steps=args.factor_update_steps,
            inv_update_steps=args.inv_update_steps,
            damping=args.damping,
            factor_decay=args.factor_decay,
            kl_clip=args.kl_clip if args.kl_clip > 0 else None,
            lr=lambda step: optimizer.param_groups[0]['lr'],
            grad_worker_fraction=kfac.DistributedStrategy[args.strategy.upper()],
            skip_layers=args.skip_layers,
            register_embeddings=args.register_embeddings,
            loglevel=logging.INFO,
        )
        cli.log(args, f'K-FAC: {len(preconditioner._layers)} layers')
    amp = args.amp_dtype if args.cuda else None
    start = time.perf_counter()
    val = float('nan')
    for epoch in range(args.epochs):
        data.train.sampler.set_epoch(epoch)
        tr = engine.train(model, criterion=criterion, optimizer=optimizer,
                          preconditioner=preconditioner, dataloader=data.train.loader,
                          epoch=epoch + 1, epochs=args.epochs, device=args.device,
                          amp_dtype=amp, clip=args.clip, verbose=args.verbose,
                          max_steps=args.max_steps_per_epoch)
        val = engine.evaluate(model, criterion=criterion, dataloader=data.val.loader,
                              device=args.device, amp_dtype=amp, verbose=args.verbose,
                              max_steps=args.max_steps_per_epoch)
        scheduler.step(val)
        cli.log(args, json.dumps({'epoch': epoch + 1, 'train_loss': round(tr, 4),
                                  'val_loss': round(val, 4)}))
    elapsed = time.perf_counter() - start
    cli.log(args, f'Training completed in {elapsed:.2f} seconds.')
    test = engine.evaluate(model, criterion=criterion, dataloader=data.test.loader,
                           device=args.device, amp_dtype=amp, prefix='Test',
                           verbose=args.verbose, max_steps=args.max_steps_per_epoch)
    return {'train_loss': tr, 'val_loss': val, 'test_loss': test, 'wall_s': elapsed}


if __name__ == '__main__':
    main()
