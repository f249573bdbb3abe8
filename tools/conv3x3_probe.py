"""Per-shape MIOpen time of ResNet-50's non-1x1 convolutions (3x3 and the
7x7 stem), fp32, channels_last, batch 32, under the bench's tuned database:
forward, input gradient and weight gradient separately.  Sizes the case for
a native implicit-GEMM path.

    python tools/conv3x3_probe.py [--batch 32]
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
from tools.conv1x1_probe import timed  # noqa: E402


def shapes(image: int) -> list[tuple]:
    m = resnet50()
    out: dict = {}
    hooks = []
    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size != (1, 1):
            def hook(mod, inp, outp):  # type: ignore[no-untyped-def]
                x = inp[0]
                key = (x.shape[2], x.shape[3], mod.in_channels, mod.out_channels,
                       mod.kernel_size[0], mod.stride[0], mod.padding[0])
                out[key] = out.get(key, 0) + 1
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(1, 3, image, image))
    for h in hooks:
        h.remove()
    return [k + (c,) for k, c in out.items()]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--image', type=int, default=224)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    from distributed_kfac_pytorch_amd.ops._native import native
    lib = native()
    tot = {'fwd': 0.0, 'dgrad': 0.0, 'wgrad': 0.0, 'gflop': 0.0}
    for h, w, ci, co, k, s, p, cnt in shapes(args.image):
        x = torch.randn(args.batch, ci, h, w, device=dev).contiguous(
            memory_format=torch.channels_last)
        wt = torch.randn(co, ci, k, k, device=dev) * (ci * k * k) ** -0.5
        y = F.conv2d(x, wt, stride=s, padding=p)
        gy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
        ho, wo = y.shape[2], y.shape[3]

        def fwd() -> None:
            F.conv2d(x, wt, stride=s, padding=p)

        def dgrad() -> None:
            torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                [0, 0], 1, [True, False, False])

        def wgrad() -> None:
            torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                [0, 0], 1, [False, True, False])

        t = [timed(f) for f in (fwd, dgrad, wgrad)]
        nat = {}
        if lib is not None and ci % 32 == 0:
            wc = wt.contiguous(memory_format=torch.channels_last)
            yn = lib.gemm3_conv(x, wc, s, p)
            ref = F.conv2d(x.double(), wt.double(), stride=s, padding=p)
            nat['fwd_err'] = f'{float((yn.double() - ref).norm() / ref.norm()):.1e}'
            nat['fwd_err_miopen'] = f'{float((y.double() - ref).norm() / ref.norm()):.1e}'
            nat['fwd_us'] = round(timed(lambda: lib.gemm3_conv(x, wc, s, p)), 1)
            dw = lib.gemm3_conv_wgrad(x, gy, k, k, s, p)
            refw = torch.ops.aten.convolution_backward(
                gy.double(), x.double(), wt.double(), None, [s, s], [p, p], [1, 1], False,
                [0, 0], 1, [False, True, False])[1]
            nat['wgrad_err'] = f'{float((dw.double() - refw).norm() / refw.norm()):.1e}'
            nat['wgrad_us'] = round(timed(lambda: lib.gemm3_conv_wgrad(x, gy, k, k, s, p)), 1)
            if s == 1 and co % 32 == 0:
                def nat_dgrad() -> torch.Tensor:
                    return lib.gemm3_conv(gy, wc, 1, k - 1 - p, True)
                dx = nat_dgrad()
                refx = torch.ops.aten.convolution_backward(
                    gy.double(), x.double(), wt.double(), None, [s, s], [p, p], [1, 1], False,
                    [0, 0], 1, [True, False, False])[0]
                nat['dgrad_err'] = f'{float((dx.double() - refx).norm() / refx.norm()):.1e}'
                nat['dgrad_us'] = round(timed(nat_dgrad), 1)
        if lib is not None and ci < 4:
            # the 3-channel stem: native weight gradient on the 4-channel
            # zero-padded input (ops/conv.py _pad4) vs MIOpen's
            from distributed_kfac_pytorch_amd.ops.conv import _pad4
            xp = _pad4(x)
            dw = lib.gemm3_conv_wgrad(xp, gy, k, k, s, p)[:, :ci]
            refw = torch.ops.aten.convolution_backward(
                gy.double(), x.double(), wt.double(), None, [s, s], [p, p], [1, 1], False,
                [0, 0], 1, [False, True, False])[1]
            nat['wgrad_err'] = f'{float((dw.double() - refw).norm() / refw.norm()):.1e}'
            nat['wgrad_us'] = round(timed(lambda: lib.gemm3_conv_wgrad(xp, gy, k, k, s, p)), 1)
        gf = 2.0 * args.batch * ho * wo * co * ci * k * k / 1e9
        for key, v in zip(('fwd', 'dgrad', 'wgrad'), t):
            tot[key] += cnt * v
        tot['gflop'] += cnt * 3 * gf
        print(json.dumps({'in': [args.batch, ci, h, w], 'cout': co, 'k': k, 'stride': s,
                          'count': cnt, 'us': [round(v, 1) for v in t],
                          'tflops': [round(gf / v * 1e3, 1) for v in t], 'native': nat}),
              flush=True)
    busy = tot['fwd'] + tot['dgrad'] + tot['wgrad']
    print(json.dumps({'total_us': {k: round(v, 1) for k, v in tot.items() if k != 'gflop'},
                      'sum_us': round(busy, 1), 'gflop': round(tot['gflop'], 1),
                      'tflops': round(tot['gflop'] / busy * 1e3, 1)}))


if __name__ == '__main__':
    main()
