"""Host-side (Python + dispatch) cost of eager K-FAC steps, by function.

    python tools/host_profile.py [--kind factor|plain|inverse] [--steps 10] [--bf16]

Builds the bench configuration (ResNet-50, batch 32, 224x224, channels_last,
fused SGD, K-FAC factor 10 / inverse 100), runs every step eagerly, and
profiles the host time of ``--steps`` steps of the requested kind with
cProfile (the GPU is synchronised before and after the profiled window, not
inside).  Prints the host ms per step next to the GPU ms per step (HIP
events): when they are equal the step is host-bound.  Then the top functions
by own time and by cumulative time.
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

os.environ.setdefault('GPU_MAX_HW_QUEUES', '4')
_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db')
if os.path.isdir(_DB):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', _DB)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops.cast import enable_fused_weight_cast  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--kind', default='factor', choices=['factor', 'plain', 'inverse'])
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--bf16', action='store_true')
    ap.add_argument('--top', type=int, default=30)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = get_model('resnet50')
    # the bench's model conversions (bench.py --conv1x1 gemm --conv-kxk gemm)
    from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1, use_implicit_gemm_conv
    use_gemm_conv1x1(model)
    use_implicit_gemm_conv(model)
    model = model.to(dev).to(memory_format=torch.channels_last)
    if args.bf16:
        enable_fused_weight_cast(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
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
        pre.step()
        opt.step()

    def kind() -> str:
        s = pre.steps
        if s % pre.inv_update_steps == 0:
            return 'inverse'
        return 'factor' if s % pre.factor_update_steps == 0 else 'plain'

    for _ in range(12):  # warm: first refresh, first factor steps, tables
        step()
    torch.cuda.synchronize()
    prof = cProfile.Profile()

    def measure(profiled: bool) -> tuple[float, float]:
        host = gpu = 0.0
        done = 0
        while done < args.steps:
            if kind() != args.kind:
                step()
                continue
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            t = time.perf_counter()
            if profiled:
                prof.enable()
            step()
            if profiled:
                prof.disable()
            host += time.perf_counter() - t
            e1.record()
            torch.cuda.synchronize()
            gpu += e0.elapsed_time(e1)
            done += 1
        return host / done * 1e3, gpu / done

    h, g = measure(False)
    hp, gp = measure(True)
    print(json.dumps({'kind': args.kind, 'bf16': args.bf16, 'steps': args.steps,
                      'host_ms_per_step': round(h, 3), 'gpu_ms_per_step': round(g, 3),
                      'profiled_host_ms_per_step': round(hp, 3)}), flush=True)
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats(key).print_stats(args.top)
        print(s.getvalue())


if __name__ == '__main__':
    main()
