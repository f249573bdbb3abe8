"""1x1 convolutions of ResNet-50 as fp32 GEMMs: hipBLASLt fp32 vs the native
bf16x3 grouped GEMM (csrc/gemm3.hip, in-kernel hi/lo split).

For every distinct stride-1 1x1 shape (batch 32, 224x224, NHWC matrices)
times forward ``Y = X W^T``, ``dX = dY W`` and the slab-reduced
``dW = dY^T X`` both ways and reports the error of each against a float64
product.  Decides whether the fp32 bench's 1x1 convolutions (407 GFLOP per
step, forward + backward) should leave hipBLASLt's fp32 MFMA path.

    python tools/conv1x1_gemm3_probe.py [--batch 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import _splitk  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import _wgrad_native  # noqa: E402
from tools.conv1x1_probe import shapes  # noqa: E402
from tools.conv1x1_probe import timed  # noqa: E402


def table(lib, As, Bs, Cs, a_kc: bool, b_kc: bool):  # type: ignore[no-untyped-def]
    n = len(As)
    tab, tiles, host = lib.build_gemm_table(As, [None] * n, Bs, Cs, [None] * n, [None] * n,
                                            [None] * n, [0.0] * n, a_kc, b_kc, None, [], [])
    return tab, n, tiles, a_kc, b_kc, host


def rel(p: torch.Tensor, ref: torch.Tensor) -> float:
    return float((p.double() - ref).norm() / ref.norm())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--slab-rows', type=int, default=None)
    args = ap.parse_args()
    lib = native()
    dev = torch.device('cuda', 0)
    tot = {'lib': 0.0, 'gemm3': 0.0}
    for h, w, ci, co, cnt in shapes(args.batch, args.image):
        m = args.batch * h * w
        x = torch.randn(m, ci, device=dev)
        wt = torch.randn(co, ci, device=dev) * ci ** -0.5
        gy = torch.randn(m, co, device=dev)
        s = _splitk(m, args.slab_rows)
        y3 = torch.empty(m, co, device=dev)
        dx3 = torch.empty(m, ci, device=dev)
        part = torch.empty(s, co, ci, device=dev)
        rows = m // s
        tf = table(lib, [x], [wt], [y3], True, True)
        tx = table(lib, [gy], [wt], [dx3], True, False)
        tw = table(lib, [gy[i * rows:(i + 1) * rows] for i in range(s)],
                   [x[i * rows:(i + 1) * rows] for i in range(s)], list(part.unbind(0)),
                   False, False)

        def g3(t):  # type: ignore[no-untyped-def]
            lib.gemm3_grouped(*t[:5])

        def lib_f() -> None:
            F.linear(x, wt)

        def lib_x() -> None:
            torch.mm(gy, wt)

        def lib_w() -> None:
            torch.bmm(gy.view(s, rows, co).transpose(1, 2), x.view(s, rows, ci)).sum(0)

        def g3_f() -> None:  # the single-descriptor kernel GemmConv1x1 runs
            lib.gemm3_mm(x, wt, y3, True, True)

        def g3_x() -> None:
            lib.gemm3_mm(gy, wt, dx3, True, False)

        def g3_w() -> None:  # split-K native weight gradient (ops/conv.py)
            _wgrad_native(lib, gy, x)

        g3_f(), g3_x(), g3(tw)
        torch.cuda.synchronize()
        xd, wd, gd = x.double(), wt.double(), gy.double()
        ref = (xd @ wd.t(), gd @ wd, gd.t() @ xd)
        err_lib = [rel(F.linear(x, wt), ref[0]), rel(gy @ wt, ref[1]),
                   rel(torch.bmm(gy.view(s, rows, co).transpose(1, 2),
                                 x.view(s, rows, ci)).sum(0), ref[2])]
        err_g3 = [rel(y3, ref[0]), rel(dx3, ref[1]), rel(_wgrad_native(lib, gy, x), ref[2])]
        t_lib = [timed(f) for f in (lib_f, lib_x, lib_w)]
        t_g3 = [timed(f) for f in (g3_f, g3_x, g3_w)]
        tot['lib'] += cnt * sum(t_lib)
        tot['gemm3'] += cnt * sum(t_g3)
        print(json.dumps({'m': m, 'cin': ci, 'cout': co, 'count': cnt, 'slabs': s,
                          'lib_us': [round(t, 1) for t in t_lib],
                          'gemm3_us': [round(t, 1) for t in t_g3],
                          'err_lib': [f'{e:.1e}' for e in err_lib],
                          'err_gemm3': [f'{e:.1e}' for e in err_g3]}), flush=True)
    print(json.dumps({'total_us': {k: round(v, 1) for k, v in tot.items()}}))


if __name__ == '__main__':
    main()
