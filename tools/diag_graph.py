"""Diagnose graph-vs-eager differences (prints per-step max rel diff)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from tests.test_e2e_gpu import _net  # noqa: E402

cuda = torch.device('cuda')
for prediv in (True, False):
    base = _net().to(cuda).to(memory_format=torch.channels_last)
    models = [copy.deepcopy(base), copy.deepcopy(base)]
    pres = [kfac.KFACPreconditioner(m, factor_update_steps=1, inv_update_steps=4,
                                    compute_method='eigen',
                                    compute_eigenvalue_outer_product=prediv,
                                    lr=lambda s: 0.1 / (1 + s)) for m in models]
    pres[1]._graphs = None
    opts = [torch.optim.SGD(m.parameters(), lr=0.05) for m in models]
    torch.manual_seed(2)
    for step in range(10):
        x = torch.randn(8, 3, 14, 14, device=cuda).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), device=cuda)
        raw = []
        for m, p, o in zip(models, pres, opts):
            o.zero_grad(set_to_none=False)
            torch.nn.functional.cross_entropy(m(x), y).backward()
            raw.append([q.grad.clone() for q in m.parameters()])
            p.step()
        rd = max(((a - b).abs().max() / b.abs().max()).item() for a, b in zip(*raw))
        pd = max(((a.grad - b.grad).abs().max() / b.grad.abs().max()).item()
                 for a, b in zip(models[0].parameters(), models[1].parameters()))
        print(f'prediv={prediv} step={step} raw_grad_rel={rd:.3e} precond_rel={pd:.3e} '
              f'replays={pres[0]._graphs.replays}', flush=True)
        for o in opts:
            o.step()
