"""Accuracy and speed of the native block-Jacobi eigensolver (K-HIP-3 large
tier, csrc/eigh_block.hip) against rocSOLVER syevd and float64 references.

Factors are K-FAC-like: running averages (decay 0.95) of batch covariances
drawn from a decaying spectrum; the warm start uses the eigenbasis of the
factor 10 updates earlier while the underlying covariance drifts by a small
random rotation (what a factor sees between two second-order updates).

    python tools/bj_probe.py [--sizes 129,576,1152,2304,4608] [--mix]
Prints one JSON line per case.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402

# ResNet-50 factor dimensions (A: Cin*k*k (+1 for fc), G: Cout), one per layer
RESNET50_MIX = (
    [147, 64] + [64, 64] + [576, 64] + [64, 256] + [64, 256]  # conv1, layer1 b1 + ds
    + [256, 64, 576, 64, 64, 256] * 2  # layer1 b2, b3
    + [256, 128, 1152, 128, 128, 512, 256, 512]  # layer2 b1 + ds
    + [512, 128, 1152, 128, 128, 512] * 3
    + [512, 256, 2304, 256, 256, 1024, 512, 1024]  # layer3 b1 + ds
    + [1024, 256, 2304, 256, 256, 1024] * 5
    + [1024, 512, 4608, 512, 512, 2048, 1024, 2048]  # layer4 b1 + ds
    + [2048, 512, 4608, 512, 512, 2048] * 2
    + [2049, 1000]
)


def kfac_pair(n: int, dev: torch.device, seed: int, drift: float = 0.02):
    """(A_old, A_new): EMA factors before / after 10 more updates."""
    g = torch.Generator(device='cpu').manual_seed(seed)
    lam = torch.exp(-torch.arange(n, dtype=torch.float64) / max(n / 8, 1.0))
    u, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    k = torch.randn(n, n, generator=g, dtype=torch.float64) * drift / n ** 0.5
    rot = torch.linalg.matrix_exp(k - k.t())
    u2 = rot @ u
    m = max(32, n // 2)

    def cov(basis):
        z = torch.randn(m, n, generator=g, dtype=torch.float64) * lam.sqrt()
        x = z @ basis.t()
        return x.t() @ x / m

    a = torch.eye(n, dtype=torch.float64)
    for _ in range(20):
        a = 0.95 * a + 0.05 * cov(u)
    a_old = a.clone()
    for _ in range(10):
        a = 0.95 * a + 0.05 * cov(u2)
    return a_old.float().to(dev), a.float().to(dev)


def check(a: torch.Tensor, d: torch.Tensor, q: torch.Tensor) -> dict:
    a64 = a.double()
    ref = torch.linalg.eigvalsh(a64)
    scale = float(ref.abs().max())
    recon = q.double() @ torch.diag(d.double()) @ q.double().t()
    eye = torch.eye(a.shape[0], dtype=torch.float64, device=a.device)
    return {
        'eval_err': float((d.double() - ref).abs().max()) / scale,
        'recon_err': float((recon - a64).abs().max()) / scale,
        'orth_err': float((q.double().t() @ q.double() - eye).abs().max()),
    }


def timed(fn, reps: int = 3) -> tuple[float, object]:
    out = fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='129,300,576,1152,2304,4608')
    ap.add_argument('--configs', default='2:1e-6:4e-6:1',
                    help='comma list of inner:tol:noise:refine')
    ap.add_argument('--syevd', type=int, default=1)
    args = ap.parse_args()
    lib = _native.native()
    assert lib is not None, _native.load_error()
    dev = torch.device('cuda')
    cfgs = []
    for c in args.configs.split(','):
        i, t, nz, rf = c.split(':')
        cfgs.append((int(i), float(t), float(nz), rf == '1'))
    for n in [int(x) for x in args.sizes.split(',')]:
        a0, a1 = kfac_pair(n, dev, seed=n)
        d0, q0 = torch.linalg.eigh(a0)
        for inner, tol, noise, refine in cfgs:
            for mode in ('cold', 'warm'):
                warm = q0.unsqueeze(0).contiguous() if mode == 'warm' else None
                ms, (d, q, sw, hist) = timed(lambda: lib.block_jacobi_eigh(
                    a1.unsqueeze(0).contiguous(), warm, 20, tol, inner, noise, refine))
                rec = {'n': n, 'mode': mode, 'inner': inner, 'tol': tol, 'noise': noise,
                       'refine': refine, 'ms': round(ms, 2), 'sweeps': int(sw[0]),
                       'active': [int(x) for x in hist[0].tolist() if x]}
                rec.update(check(a1, d[0], q[0]))
                print(json.dumps(rec), flush=True)
        if args.syevd:
            ms, (d, q) = timed(lambda: lib.rocsolver_eigh(a1.unsqueeze(0).clone(), 0, 100, 1e-7))
            rec = {'n': n, 'mode': 'syevd', 'ms': round(ms, 2)}
            rec.update(check(a1, d[0], q[0]))
            print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
