"""Ad-hoc CPU parity check against the read-only reference checkout at
/root/reference (not part of the test suite: the reference is absent on the
GPU box).  Trains two identical small conv nets side by side and prints the
relative gradient difference after each preconditioner step."""
import sys, copy, warnings
warnings.filterwarnings('ignore')
import torch
sys.path.insert(0, '/root/reference')
import kfac as refk
sys.path.insert(0, '/root/repo')
import distributed_kfac_pytorch_amd as mk
torch.manual_seed(0)
def make():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1, stride=2), torch.nn.ReLU(), torch.nn.Conv2d(8, 8, 3, bias=False), torch.nn.Flatten(), torch.nn.Linear(8*5*5, 10))
for method in ['eigen', 'inverse']:
  for prediv in [True, False]:
    m1 = make(); m2 = make()
    kw = dict(factor_update_steps=1, inv_update_steps=2, compute_method=method, compute_eigenvalue_outer_product=prediv, lr=0.1, kl_clip=0.001)
    p1 = refk.preconditioner.KFACPreconditioner(m1, **kw)
    p2 = mk.KFACPreconditioner(m2, **kw)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1); o2 = torch.optim.SGD(m2.parameters(), lr=0.1)
    for step in range(4):
        x = torch.randn(4, 3, 14, 14); y = torch.randint(0, 10, (4,))
        for m, p, o in ((m1, p1, o1), (m2, p2, o2)):
            o.zero_grad(); torch.nn.functional.cross_entropy(m(x), y).backward(); p.step()
        md = max((a.grad - b.grad).abs().max().item() / (a.grad.abs().max().item()+1e-12) for a, b in zip(m1.parameters(), m2.parameters()))
        o1.step(); o2.step()
        print(method, prediv, step, 'max rel grad diff', md)
    sd1 = p1.state_dict(); sd2 = p2.state_dict()
    for k in sd1['layers']:
        for f in 'AG':
            print(k, f, (sd1['layers'][k][f] - sd2['layers'][k][f]).abs().max().item())
