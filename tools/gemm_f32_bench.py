"""Native fp32 MFMA GEMM (csrc/gemm_f32.hip) vs torch (hipBLASLt / rocBLAS)
on the eigensolver back-transform's shapes.

    python tools/gemm_f32_bench.py [--n 4608] [--batch 3] [--nb 512]

One JSON line per shape: ms and TFLOP/s of both, max relative difference.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402


def timeit(fn, reps: int = 10) -> float:
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
    ap.add_argument('--n', type=int, default=4608)
    ap.add_argument('--batch', type=int, default=3)
    ap.add_argument('--nb', type=int, default=512)
    args = ap.parse_args()
    lib = _native.native()
    dev = torch.device('cuda', 0)
    n, c, b = args.n, args.batch, args.nb
    m = n - 1  # rows of the first block
    shapes = {  # name: (M, N, K, ta, tb)
        'VVt': (b, b, m, False, True),
        'V_X': (b, n, m, False, False),
        'T_Y': (b, n, b, False, False),
        'Vt_W': (m, n, b, True, False),
        'square': (n, n, n, False, False),
    }
    for name, (M, N, K, ta, tb) in shapes.items():
        A = torch.randn(c, *((K, M) if ta else (M, K)), device=dev)
        B = torch.randn(c, *((N, K) if tb else (K, N)), device=dev)
        C = torch.empty(c, M, N, device=dev)
        Ao = A.transpose(1, 2) if ta else A
        Bo = B.transpose(1, 2) if tb else B
        t_nat = timeit(lambda: lib.gemm_f32(A, B, C, ta, tb))
        ref = torch.bmm(Ao, Bo)
        t_lib = timeit(lambda: torch.bmm(Ao, Bo))
        err = float((C - ref).abs().max() / ref.abs().max())
        fl = 2.0 * c * M * N * K
        print(json.dumps({'shape': name, 'M': M, 'N': N, 'K': K, 'batch': c,
                          'native_ms': round(t_nat, 3), 'torch_ms': round(t_lib, 3),
                          'native_tflops': round(fl / t_nat / 1e9, 1),
                          'torch_tflops': round(fl / t_lib / 1e9, 1), 'rel_err': err}), flush=True)


if __name__ == '__main__':
    main()
