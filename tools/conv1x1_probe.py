"""1x1 convolutions of ResNet-50 (batch 32, 224x224, channels_last): MIOpen
vs the same convolution as a GEMM on the NHWC activation matrix.

A 1x1, stride-1 convolution on a channels_last tensor is exactly
``Y[NHW, Cout] = X[NHW, Cin] @ W[Cout, Cin]^T``; its backward is
``dX = dY @ W`` and ``dW = dY^T @ X``.  This probe times forward + backward
(dX and dW) of every distinct 1x1 shape both ways, fp32 (and bf16 with
``--bf16``), and checks the results agree.

    python tools/conv1x1_probe.py [--bf16] [--batch 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db')
if os.path.isdir(_DB):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', _DB)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import _Conv1x1Gemm  # noqa: E402


def shapes(batch: int, image: int) -> list[tuple[int, int, int, int]]:
    """(H, W, Cin, Cout) of every stride-1 1x1 conv of ResNet-50."""
    m = resnet50()
    out: dict = {}
    hooks = []
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size == (1, 1) and mod.stride == (1, 1):
            def hook(mod, inp, outp, name=name):  # type: ignore[no-untyped-def]
                x = inp[0]
                out[name] = (x.shape[2], x.shape[3], mod.in_channels, mod.out_channels)
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(1, 3, image, image))
    for h in hooks:
        h.remove()
    counts: dict = {}
    for s in out.values():
        counts[s] = counts.get(s, 0) + 1
    return [(h, w, ci, co, c) for (h, w, ci, co), c in counts.items()]


def timed(fn, reps: int = 20) -> float:  # type: ignore[no-untyped-def]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--bf16', action='store_true')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    dt = torch.bfloat16 if args.bf16 else torch.float32
    tot = {'miopen': 0.0, 'gemm': 0.0, 'gemm_plain': 0.0}
    for h, w, ci, co, cnt in shapes(args.batch, args.image):
        x = torch.randn(args.batch, ci, h, w, device=dev, dtype=dt).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        wt = (torch.randn(co, ci, 1, 1, device=dev, dtype=dt) * ci ** -0.5).requires_grad_(True)
        gy = torch.randn(args.batch, co, h, w, device=dev, dtype=dt).contiguous(
            memory_format=torch.channels_last)

        def miopen() -> tuple:
            y = F.conv2d(x, wt)
            return (y,) + torch.autograd.grad(y, (x, wt), gy)

        def gemm() -> tuple:  # ops/conv.py GemmConv1x1 (slab-reduced dW)
            xm = x.permute(0, 2, 3, 1).reshape(-1, ci)
            ym = _Conv1x1Gemm.apply(xm, wt.view(co, ci), None)
            y = ym.view(args.batch, h, w, co).permute(0, 3, 1, 2)
            return (y,) + torch.autograd.grad(y, (x, wt), gy)

        def gemm_plain() -> tuple:  # one GEMM per product (dW with K = N*H*W)
            xm = x.permute(0, 2, 3, 1).reshape(-1, ci)
            ym = xm @ wt.view(co, ci).t()
            y = ym.view(args.batch, h, w, co).permute(0, 3, 1, 2)
            return (y,) + torch.autograd.grad(y, (x, wt), gy)

        a, b = miopen(), gemm()
        rel = max(float((p.detach().float() - q.detach().float()).abs().max() / q.detach().float().abs().max())
                  for p, q in zip(a, b))
        tm, tg, tp = timed(miopen), timed(gemm), timed(gemm_plain)
        tot['miopen'] += cnt * tm
        tot['gemm'] += cnt * tg
        tot['gemm_plain'] += cnt * tp
        print(json.dumps({'shape': [args.batch, ci, h, w, co], 'count': cnt, 'miopen_us': round(tm, 1),
                          'gemm_us': round(tg, 1), 'gemm_plain_us': round(tp, 1), 'maxrel': rel,
                          'y_strides_gemm': list(b[0].stride()),
                          'dx_cl': b[1].is_contiguous(memory_format=torch.channels_last)}),
              flush=True)
    print(json.dumps({'total_us': {k: round(v, 1) for k, v in tot.items()}, 'dtype': str(dt)}))


if __name__ == '__main__':
    main()
