"""Time the grouped bf16x3 precondition GEMMs (csrc/gemm3.hip) on the
ResNet-50 layer set: the four chain launches separately, their total, the
effective TFLOP/s, and the accuracy vs an fp64 chain."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402
from tools.bench_gemm import LAYERS  # noqa: E402


def main() -> None:
    lib = _native.native()
    assert lib is not None, _native.load_error()
    dev = torch.device('cuda')
    torch.manual_seed(0)
    T = [[] for _ in range(4)]
    flops = 0.0
    keep = []
    for g, a, cnt in LAYERS:
        for _ in range(cnt):
            wg = torch.randn(g, a, device=dev)
            # random (not orthogonal) bases: no solver call, so the script
            # also runs under rocprofv3 --pmc
            qa = torch.randn(a, a, device=dev) / a ** 0.5
            qg = torch.randn(g, g, device=dev) / g ** 0.5
            dgda = torch.rand(g, a, device=dev)
            t1 = torch.empty(g, a, device=dev)
            t2 = torch.empty(g, a, device=dev)
            out = torch.empty(g, a, device=dev)
            T[0].append((wg, None, qa, t1, None, None, None, 0.0))
            T[1].append((qg, None, t1, t2, dgda, None, None, 0.0))
            T[2].append((qg, None, t2, t1, None, None, None, 0.0))
            T[3].append((t1, None, qa, out, None, None, None, 0.0))
            keep.append((wg, qa, qg, dgda, out))
            flops += 2 * (2 * g * g * a + 2 * g * a * a)
    flags = [(True, False), (False, False), (True, False), (True, True)]
    tabs = []
    for rows, (akc, bkc) in zip(T, flags):
        cols = list(zip(*rows))
        tab, tiles, _ = lib.build_gemm_table(*[list(c) for c in cols], akc, bkc)
        tabs.append((tab, len(rows), tiles, akc, bkc))

    def run(i: int | None = None) -> None:
        for j, (tab, n, tiles, akc, bkc) in enumerate(tabs):
            if i is None or i == j:
                lib.gemm3_grouped(tab, n, tiles, akc, bkc)

    def timeit(fn, iters: int = 20) -> float:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters

    res = {'tiles': [t[2] for t in tabs]}
    res['launch_ms'] = [round(timeit(lambda i=i: run(i)), 4) for i in range(4)]
    total = timeit(run)
    res['chain_ms'] = round(total, 4)
    res['gflop'] = round(flops / 1e9, 1)
    res['tflops'] = round(flops / total / 1e9, 1)
    run()
    torch.cuda.synchronize()
    errs = []
    for wg, qa, qg, dgda, out in keep[::7]:
        ref = qg.double() @ ((qg.double().t() @ wg.double() @ qa.double()) * dgda.double()) \
            @ qa.double().t()
        errs.append(((out.double() - ref).abs().max() / ref.abs().max()).item())
    res['max_rel_err'] = max(errs)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
