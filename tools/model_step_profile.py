"""Device time of one training step by PyTorch op (torch.profiler).

    python tools/model_step_profile.py [--kfac] [--kind plain|factor] [--bf16] [--steps 5]

Builds the bench's ResNet-50 (batch 32, 224x224, channels_last, native 1x1 /
3x3 convolutions, fused SGD), runs warm eager steps, then profiles
``--steps`` steps and prints the device time per kernel grouped under the
top-level ATen / autograd op that launched it (``key_averages`` by input
shape and by stack), so library kernels such as ``reduce_kernel`` or
``CUDAFunctor_add`` are attributed to their Python call site.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

os.environ.setdefault('GPU_MAX_HW_QUEUES', '4')
_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db')
if os.path.isdir(_DB):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', _DB)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity  # noqa: E402
from torch.profiler import profile  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--kfac', action='store_true')
    ap.add_argument('--kind', default='plain', choices=['plain', 'factor'])
    ap.add_argument('--bf16', action='store_true')
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--json', default=None, help='write the table here too')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1
    from distributed_kfac_pytorch_amd.ops.conv import use_implicit_gemm_conv
    model = get_model('resnet50')
    use_gemm_conv1x1(model)
    use_implicit_gemm_conv(model)
    model = model.to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
    pre = None
    if args.kfac:
        pre = kfac.KFACPreconditioner(
            model, factor_update_steps=10, inv_update_steps=100, damping=0.001,
            factor_decay=0.95, kl_clip=0.001, lr=lambda s: opt.param_groups[0]['lr'],
            allreduce_bucket_cap_mb=25, colocate_factors=True, grad_worker_fraction=0.5)
    x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device=dev)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)

    def step() -> None:
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=args.bf16):
            loss = crit(model(x), y)
        loss.backward()
        if pre is not None:
            pre.step()
        opt.step()

    def want() -> bool:
        if pre is None:
            return True
        s = pre.steps
        if s % pre.inv_update_steps == 0:
            return False
        return (s % pre.factor_update_steps == 0) == (args.kind == 'factor')

    for _ in range(12):
        step()
    while not want():
        step()
    torch.cuda.synchronize()
    # consecutive steps from a step of the wanted kind (with K-FAC, at most
    # factor_update_steps - 1 plain steps in a row; use --steps 1 for factor)
    done = args.steps
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=False, with_stack=True) as prof:
        for _ in range(done):
            step()
        torch.cuda.synchronize()
    ev = prof.key_averages(group_by_stack_n=6)
    rows = []
    for e in ev:
        if getattr(e, 'device_type', None) != torch.autograd.DeviceType.CPU:
            continue  # kernel rows: their time is attributed to the op below
        dt = getattr(e, 'self_device_time_total', None)
        if dt is None:
            dt = getattr(e, 'self_cuda_time_total', 0)
        if dt <= 0:
            continue
        rows.append({'name': e.key, 'us_per_step': round(dt / done, 1), 'calls': e.count,
                     'stack': list(e.stack)[:6]})
    rows.sort(key=lambda r: -r['us_per_step'])
    total = sum(r['us_per_step'] for r in rows)
    print(json.dumps({'kfac': args.kfac, 'kind': args.kind, 'bf16': args.bf16,
                      'steps': done, 'device_us_per_step': round(total, 1)}))
    for r in rows[:args.top]:
        print(f"{r['us_per_step']:9.1f} us  x{r['calls']:<5d} {r['name'][:90]}")
        for s in r['stack'][:4]:
            print(f'              {s[:110]}')
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
