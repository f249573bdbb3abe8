"""rocSOLVER syevd on the ResNet-50 4608 bucket (3 factors), for a
kernel-level time breakdown under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402

lib = _native.native()
n = int(os.environ.get('N', '4608'))
x = torch.randn(3, n, n // 3, device='cuda')
a = (x @ x.transpose(1, 2) / n + 1e-3 * torch.eye(n, device='cuda')).contiguous()
for _ in range(2):
    lib.rocsolver_eigh(a.clone(), 0, 100, 1e-7)
torch.cuda.synchronize()
