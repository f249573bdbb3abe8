"""Effective bandwidth of the fused BatchNorm(+ReLU) kernels at ResNet-50's
shapes (batch 32, fp32, channels_last): forward (statistics pass + finalize +
apply, as when no convolution epilogue supplied the statistics) and backward
(partials + finalize + apply, ReLU mask recomputed from x).

    python tools/bn_probe.py [--batch 32] [--reps 50] [--dtype fp32|bf16]

One JSON line per shape: ms per forward / backward and GB/s over the bytes
the passes must move (forward 3 passes of the activation: read x twice,
write y; backward 5: read x and dy twice, write dx).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402
from distributed_kfac_pytorch_amd.ops.bnact import bn_act  # noqa: E402

SHAPES = [(64, 112), (64, 56), (256, 56), (128, 56), (128, 28), (512, 28), (256, 28),
          (256, 14), (1024, 14), (512, 14), (512, 7), (2048, 7)]


def timed(fn, reps: int) -> float:  # type: ignore[no-untyped-def]
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--dtype', choices=('fp32', 'bf16'), default='fp32')
    args = ap.parse_args()
    assert _native.native() is not None, _native.load_error()
    dev = torch.device('cuda', 0)
    dt = torch.float32 if args.dtype == 'fp32' else torch.bfloat16
    # reference: a device copy of 256 MiB (read + write)
    src = torch.empty(64 * 2**20, device=dev)
    dst = torch.empty_like(src)
    cp_ms = timed(lambda: dst.copy_(src), args.reps)
    print(json.dumps({'copy_GBs': round(2 * src.numel() * 4 / cp_ms / 1e6, 0)}), flush=True)
    for c, h in SHAPES:
        bn = nn.BatchNorm2d(c).to(dev)
        x = torch.randn(args.batch, c, h, h, device=dev, dtype=dt)
        x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
        g = torch.randn_like(x)

        def fwd() -> torch.Tensor:
            with torch.no_grad():
                return bn_act(bn, x, None, True)

        y = bn_act(bn, x, None, True)

        def bwd() -> None:
            torch.autograd.grad(y, (x, bn.weight, bn.bias), g, retain_graph=True)

        f_ms, b_ms = timed(fwd, args.reps), timed(bwd, args.reps)
        nbytes = x.numel() * x.element_size()
        print(json.dumps({'C': c, 'HW': h, 'MB': round(nbytes / 2**20, 1),
                          'fwd_ms': round(f_ms, 4), 'bwd_ms': round(b_ms, 4),
                          'fwd_GBs': round(3 * nbytes / f_ms / 1e6, 0),
                          'bwd_GBs': round(5 * nbytes / b_ms / 1e6, 0)}), flush=True)


if __name__ == '__main__':
    main()
