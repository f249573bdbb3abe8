"""Repeatability check of the damped SPD inverse tiers (NaN scan + error vs
float64), 5 repeats per size.  Usage: python tools/spd_dbg.py"""
import sys

import torch

sys.path.insert(0, '.')
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402

for n in (64, 176, 177, 200, 255, 257, 300, 640, 2304):
    torch.manual_seed(n)
    x = torch.randn(3, n, 2 * n, device='cuda')
    f = (x @ x.transpose(1, 2) / (2 * n)).contiguous()
    ref = torch.linalg.inv(f.double() + 1e-2 * torch.eye(n, device='cuda', dtype=torch.float64))
    nans, err = 0, 0.0
    for _ in range(5):
        got = torch.stack(linalg.inverse_many(list(f), 1e-2))
        nans += int(torch.isnan(got).sum())
        err = max(err, float((got.double() - ref).abs().max() / ref.abs().max()))
    print(n, 'nan', nans, 'rel_err', f'{err:.2e}', flush=True)
