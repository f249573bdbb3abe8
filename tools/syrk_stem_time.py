"""Time the ResNet-50 stem's A-factor SYRK (fp32 patches [401408, 147], the
7x7 conv on a batch of 32) through ops.factors.cov_accumulate_."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import factors  # noqa: E402
from distributed_kfac_pytorch_amd.ops._native import native  # noqa: E402

x = torch.randn(401408, 147, device='cuda')
out = torch.zeros(147, 147, device='cuda')
for _ in range(3):
    factors.cov_accumulate_(out, x, bias=False, alpha=1.0, beta=0.0)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    factors.cov_accumulate_(out, x, bias=False, alpha=1.0, beta=0.0)
e1.record()
e1.synchronize()
ref = (x.double().t() @ x.double())
err = float((out.double() - ref).abs().max() / ref.abs().max())
print(json.dumps({'shape': [401408, 147], 'splits': int(native().syrk_default_splits(401408, 147)),
                  'ms': round(e0.elapsed_time(e1) / 20, 3), 'rel_err': err}))
