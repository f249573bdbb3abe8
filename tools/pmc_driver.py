"""Small eager ResNet-50 K-FAC workload for rocprofv3 --pmc passes: every
step updates the factors (SYRK dense + implicit-im2col), preconditions
(grouped bf16x3 GEMM) and applies (KL clip, gradient write); step 0 and
step 4 refresh the second-order state (eigensolver tiers).  Eager (no HIP
graphs) so every dispatch is visible to the counter collection."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('MIOPEN_USER_DB_PATH', os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db'))
os.environ['KFAC_GRAPHS'] = '0'
# one issuing thread: the counter collection serialises dispatches, and the
# threaded eigensolver lanes crashed the profiled process (SIGSEGV in a lane)
os.environ['KFAC_EIGH_THREADS'] = '0'
# rocSOLVER's syevd faults under counter collection: the large factors go
# through the native block-Jacobi tier here (its kernels get counted too)
os.environ['KFAC_EIGH_LARGE'] = 'block'
os.environ['KFAC_EIGH_COLD'] = 'block'

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(0)
model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9)
method = os.environ.get('PMC_METHOD', 'eigen')
pre = kfac.KFACPreconditioner(model, factor_update_steps=1, inv_update_steps=4,
                              damping=0.001, lr=lambda s: 0.0125, grad_worker_fraction=0.5,
                              compute_method=method)
x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
for _ in range(int(os.environ.get('PMC_STEPS', '6'))):
    opt.zero_grad(set_to_none=False)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        loss = crit(model(x), y)
    loss.backward()
    pre.step()
    opt.step()
torch.cuda.synchronize()
