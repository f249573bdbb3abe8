"""Generate the golden fixtures of tests/test_ref_parity.py from the
reference package, on the CPU.

Runs the upstream ``kfac`` package (a scratch copy of the read-only
checkout; never committed) on a small conv net for every compute method x
eigenvalue-outer-product combination and records, per step, the input batch
and the preconditioned gradients, plus the final checkpoint factors and the
checkpoint keys -- including the ``module.`` prefix under DDP (a one-rank
gloo group).  Everything is saved as plain tensors / lists / dicts so the
test loads it with ``torch.load(weights_only=True)``.

    cp -r /root/reference/kfac /tmp/refpkg/ && \\
        python tools/make_ref_fixtures.py --reference /tmp/refpkg
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.distributed as dist

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'tests', 'data', 'ref_fixtures.pt')

CONFIGS = [
    ('eigen', True),
    ('eigen', False),
    ('inverse', True),
    ('inverse', False),
]


def make_model() -> torch.nn.Module:
    torch.manual_seed(0)
    return torch.nn.Sequential(
        torch.nn.Conv2d(3, 8, 3, padding=1, stride=2),
        torch.nn.ReLU(),
        torch.nn.Conv2d(8, 8, 3, bias=False),
        torch.nn.Flatten(),
        torch.nn.Linear(8 * 5 * 5, 10),
    )


KW = dict(factor_update_steps=1, inv_update_steps=2, lr=0.1, kl_clip=0.001,
          damping=0.003, factor_decay=0.95)


def run(ref, method: str, prediv: bool, steps: int) -> dict:  # type: ignore[no-untyped-def]
    model = make_model()
    pre = ref.preconditioner.KFACPreconditioner(
        model, compute_method=method, compute_eigenvalue_outer_product=prediv, **KW)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(7)
    rec = {'x': [], 'y': [], 'grads': []}
    for _ in range(steps):
        x = torch.randn(4, 3, 14, 14, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
        rec['x'].append(x)
        rec['y'].append(y)
        rec['grads'].append([p.grad.detach().clone() for p in model.parameters()])
        opt.step()
    sd = pre.state_dict()
    rec['factors'] = {k: {'A': v['A'].clone(), 'G': v['G'].clone()}
                      for k, v in sd['layers'].items()}
    rec['state_keys'] = sorted(sd.keys())
    return rec


def ddp_keys(ref) -> list:  # type: ignore[no-untyped-def]
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29611')
    dist.init_process_group('gloo', rank=0, world_size=1)
    model = torch.nn.parallel.DistributedDataParallel(make_model())
    pre = ref.preconditioner.KFACPreconditioner(model, **KW)
    x = torch.randn(4, 3, 14, 14)
    torch.nn.functional.cross_entropy(model(x), torch.zeros(4, dtype=torch.long)).backward()
    pre.step()
    keys = sorted(pre.state_dict()['layers'])
    dist.destroy_process_group()
    return keys


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', required=True, help='directory holding the kfac package')
    ap.add_argument('--steps', type=int, default=4)
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    import kfac as ref  # upstream package (scratch copy)

    torch.set_num_threads(1)
    data = {'source': 'upstream kfac_pytorch 0.4.1, CPU fp32', 'kwargs': KW, 'runs': {}}
    for method, prediv in CONFIGS:
        data['runs'][f'{method}-prediv{int(prediv)}'] = run(ref, method, prediv, args.steps)
    data['ddp_layer_keys'] = ddp_keys(ref)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    torch.save(data, OUT)
    print('wrote', OUT)


if __name__ == '__main__':
    main()
