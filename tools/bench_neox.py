"""GPT-NeoX-125M K-FAC vs SGD training throughput on one GPU (tokens/s).

Secondary benchmark line next to the ResNet-50 headline (bench.py): the
reference's tensor-parallel ``kfac/gpt_neox`` variant on a NeoX-125M-shaped
model (hidden 768, 12 layers, 12 heads, vocab 50304, seq 2048, micro-batch
8), random-init weights and synthetic tokens, bf16 autocast, at the
reference example cadence (factor update every 10 steps, eigen refresh
every 100).  The timed window of exactly ``--steps`` steps starts on a
second-order update step; the headline value is the period average (one
refresh + factor-update steps + plain steps of one inverse period, each at
its in-window GPU time), as bench.py.  The same harness then times plain
SGD on the same model for ``kfac_overhead_ms``.

    python tools/bench_neox.py --steps 30 --warmup 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_kfac_pytorch_amd.models.gpt_neox import GPTNeoX  # noqa: E402
from distributed_kfac_pytorch_amd.neox.pipeline import PipelineModule  # noqa: E402
from distributed_kfac_pytorch_amd.neox.preconditioner import GPTNeoXKFACPreconditioner  # noqa: E402
from distributed_kfac_pytorch_amd.neox.topology import PipeModelDataParallelTopology  # noqa: E402
from distributed_kfac_pytorch_amd.warnings import ExperimentalFeatureWarning  # noqa: E402

warnings.filterwarnings('ignore', category=ExperimentalFeatureWarning)

MODELS = {
    '125m': dict(hidden=768, layers=12, heads=12, vocab=50304),
    'tiny': dict(hidden=64, layers=2, heads=4, vocab=512),
}


def parse_args() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument('--model', default='125m', choices=sorted(MODELS))
    p.add_argument('--steps', type=int, default=30)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--seq-len', type=int, default=2048)
    p.add_argument('--micro-batch', type=int, default=8)
    p.add_argument('--factor-update-steps', type=int, default=10)
    p.add_argument('--inv-update-steps', type=int, default=100)
    p.add_argument('--damping', type=float, default=0.003)
    p.add_argument('--kl-clip', type=float, default=0.001)
    p.add_argument('--lr', type=float, default=0.05)
    p.add_argument('--fp32', action='store_true')
    p.add_argument('--no-sgd', action='store_true', help='skip the SGD comparison run')
    return p.parse_args()


def run(args: argparse.Namespace, use_kfac: bool, dev: torch.device) -> dict:
    cfg = MODELS[args.model]
    topo = PipeModelDataParallelTopology(num_pp=1, num_mp=1, num_dp=1)
    torch.manual_seed(0)
    model = PipelineModule(
        [lambda: GPTNeoX(vocab=cfg['vocab'], hidden=cfg['hidden'], layers=cfg['layers'],
                         heads=cfg['heads'], group=None)], topo, rank=0).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9, foreach=True)
    pre = None
    if use_kfac:
        pre = GPTNeoXKFACPreconditioner(
            model, factor_update_steps=args.factor_update_steps,
            inv_update_steps=args.inv_update_steps, damping=args.damping,
            kl_clip=args.kl_clip, lr=lambda s: opt.param_groups[0]['lr'])
    g = torch.Generator(device=dev).manual_seed(1)
    pool = [torch.randint(0, cfg['vocab'], (args.micro_batch, args.seq_len + 1),
                          device=dev, generator=g) for _ in range(4)]
    counter = [0]
    amp = not args.fp32

    def step() -> None:
        tok = pool[counter[0] % len(pool)]
        counter[0] += 1
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp):
            logits = model(tok[:, :-1])
        loss = torch.nn.functional.cross_entropy(logits.float().flatten(0, 1),
                                                 tok[:, 1:].flatten())
        loss.backward()
        if pre is not None:
            pre.step()
        opt.step()

    def kind() -> str:
        if pre is None:
            return 'plain'
        if pre.steps % pre.inv_update_steps == 0:
            return 'inverse'
        if pre.steps % pre.factor_update_steps == 0:
            return 'factor'
        return 'plain'

    for _ in range(args.warmup):
        step()
    align = 0
    if pre is not None:
        while pre.steps % pre.inv_update_steps != 0:
            step()
            align += 1
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    kinds = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        kinds.append(kind())
        ev[i].record()
        step()
    ev[-1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    by = {}
    for k in ('plain', 'factor', 'inverse'):
        v = [t for t, kk in zip(per, kinds) if kk == k]
        by[k] = sum(v) / len(v) if v else 0.0
    out = {'seconds': elapsed, 'ms_per_step': elapsed / args.steps * 1e3,
           'kind_ms': {k: round(v, 3) for k, v in by.items() if v},
           'kind_counts': {k: kinds.count(k) for k in by}, 'align_steps': align}
    if pre is not None:
        inv_p, f_p = pre.inv_update_steps, pre.factor_update_steps
        n_factor = len([s for s in range(1, inv_p) if s % f_p == 0])
        n_plain = inv_p - 1 - n_factor
        tf = by['factor'] or by['plain']
        out['period_ms_per_step'] = (by['inverse'] + n_factor * tf + n_plain * by['plain']) / inv_p
        out['refresh_ms'] = by['inverse'] - by['plain']
        out['kfac_layers'] = len(pre._layers)
        out['grouped_precondition'] = pre._grouped is not None and pre._grouped._key is not None
        out['multi_apply'] = pre._multi_apply is not None and pre._multi_apply._key is not None
    del model, opt, pre
    torch.cuda.empty_cache()
    return out


def main() -> None:
    args = parse_args()
    dev = torch.device('cuda', 0)
    res = run(args, True, dev)
    base = None if args.no_sgd else run(args, False, dev)
    tokens = args.micro_batch * args.seq_len
    ms = res['period_ms_per_step']
    line = {
        'metric': f'tokens/sec, GPT-NeoX-{args.model} K-FAC training (1 GPU)',
        'value': round(tokens * 1e3 / ms, 1),
        'unit': 'tokens/s',
        'n_gpus': 1,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms, 3),
        'higher_is_better': True,
        'dtype': 'fp32' if args.fp32 else 'bf16',
        'data': 'synthetic tokens, random-init weights',
        'config': {'model': f'gpt-neox-{args.model}', **MODELS[args.model],
                   'seq_len': args.seq_len, 'micro_batch': args.micro_batch,
                   'parallelism': 'dp1 mp1',
                   'kfac': {'method': 'eigen', 'factor_update_steps': args.factor_update_steps,
                            'inv_update_steps': args.inv_update_steps,
                            'damping': args.damping, 'kl_clip': args.kl_clip}},
        'timing': 'period-averaged (see tools/bench_neox.py docstring)',
        'window_ms_per_step': round(res['ms_per_step'], 3),
        'kind_ms': res['kind_ms'],
        'kind_counts': res['kind_counts'],
        'eigen_refresh_ms': round(res['refresh_ms'], 3),
        'kfac_layers': res['kfac_layers'],
        'grouped_precondition': res['grouped_precondition'],
        'multi_apply': res['multi_apply'],
    }
    if base is not None:
        line['sgd_ms_per_step'] = round(base['ms_per_step'], 3)
        line['sgd_tokens_per_sec'] = round(tokens * 1e3 / base['ms_per_step'], 1)
        line['kfac_overhead_ms'] = round(ms - base['ms_per_step'], 3)
    print(json.dumps(line), flush=True)


if __name__ == '__main__':
    main()
