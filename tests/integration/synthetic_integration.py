"""Convergence integration test (reference
``tests/integration/mnist_integration_test.py``): the same small CNN trained
with Adadelta, with and without K-FAC; K-FAC must reach a higher test
accuracy.

MNIST cannot be downloaded here, so the data is a synthetic MNIST-shaped
task: 10 smooth random 28x28 class templates, each sample a randomly
shifted template plus a large shared low-rank nuisance field and pixel
noise (parity with the real-MNIST numbers is unpinned).  Run as a script for the full 5-epoch
version; pytest runs a shorter configuration.
"""
from __future__ import annotations

import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader
from torch.utils.data import TensorDataset

from distributed_kfac_pytorch_amd import KFACPreconditioner


def make_data(n: int, seed: int, nuisance: float = 3.0, noise: float = 1.0) -> TensorDataset:
    """Class templates plus a strong shared low-rank nuisance field.

    The nuisance makes the input covariance badly conditioned (what the
    K-FAC A factor whitens), so the first-order baseline stalls while K-FAC
    does not -- the property the reference test checks on MNIST.
    """
    g = torch.Generator().manual_seed(1234)  # templates shared by all splits
    templates = F.interpolate(torch.randn(10, 1, 14, 14, generator=g), size=(28, 28),
                              mode='bilinear', align_corners=False)
    common = F.interpolate(torch.randn(4, 1, 7, 7, generator=g), size=(28, 28),
                           mode='bilinear', align_corners=False)[:, 0]
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g)
    shifts = torch.randint(-3, 4, (n, 2), generator=g)
    x = torch.stack([
        torch.roll(t, (int(s[0]), int(s[1])), dims=(1, 2)) for t, s in zip(templates[y], shifts)
    ])
    c = torch.randn(n, 4, generator=g) * nuisance
    x = x + torch.einsum('nk,khw->nhw', c, common).unsqueeze(1)
    x = x + noise * torch.randn(x.shape, generator=g)
    return TensorDataset(x, y)


class Net(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(1, 4, 3, 1)
        self.conv2 = nn.Conv2d(4, 4, 3, 1)
        self.fc1 = nn.Linear(576, 64)
        self.fc2 = nn.Linear(64, 10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = F.relu(self.fc1(torch.flatten(x, 1)))
        return F.log_softmax(self.fc2(x), dim=1)


def train_and_eval(precondition: bool, epochs: int, n_train: int, n_test: int) -> float:
    torch.manual_seed(42)
    train_loader = DataLoader(make_data(n_train, 1), batch_size=64, shuffle=True)
    test = make_data(n_test, 2)
    model = Net()
    optimizer = torch.optim.Adadelta(model.parameters(), lr=0.1)
    scheduler = torch.optim.lr_scheduler.StepLR(optimizer, step_size=1, gamma=0.7)
    pre = None
    if precondition:
        pre = KFACPreconditioner(
            model, factor_update_steps=10, inv_update_steps=100,
            lr=lambda x: optimizer.param_groups[0]['lr'], update_factors_in_hook=False,
        )
    acc = 0.0
    for epoch in range(1, epochs + 1):
        model.train()
        for data, target in train_loader:
            optimizer.zero_grad(set_to_none=True)
            F.nll_loss(model(data), target).backward()
            if pre is not None:
                pre.step()
            optimizer.step()
        model.eval()
        with torch.no_grad():
            acc = 100.0 * (model(test.tensors[0]).argmax(1) == test.tensors[1]).float().mean().item()
        scheduler.step()
        print(f'  epoch {epoch}: accuracy={acc:.2f}%', flush=True)
    return acc


def run(epochs: int = 5, n_train: int = 20_000, n_test: int = 4_000) -> tuple[float, float]:
    print('Training without K-FAC:')
    base = train_and_eval(False, epochs, n_train, n_test)
    print('Training with K-FAC:')
    kfac_acc = train_and_eval(True, epochs, n_train, n_test)
    return base, kfac_acc


if __name__ == '__main__':
    t0 = time.perf_counter()
    base, kfac_acc = run()
    print(f'baseline {base:.2f}%  kfac {kfac_acc:.2f}%  ({time.perf_counter() - t0:.1f} s)')
    sys.exit(0 if kfac_acc > base else 1)
