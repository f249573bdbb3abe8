"""Small models used by the plumbing tests and the MNIST-style example
(same architectures as reference ``testing/models.py:12-66``)."""
from __future__ import annotations

import torch
import torch.nn.functional as F


class TinyModel(torch.nn.Module):
    """Linear(10->20, no bias) -> ReLU -> Linear(20->10) -> Softmax."""

    def __init__(self) -> None:
        super().__init__()
        self.linear1 = torch.nn.Linear(10, 20, bias=False)
        self.activation = torch.nn.ReLU()
        self.linear2 = torch.nn.Linear(20, 10)
        self.softmax = torch.nn.Softmax(dim=-1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.softmax(self.linear2(self.activation(self.linear1(x))))


class LeNet(torch.nn.Module):
    """LeNet-5 style CNN for 1x28x28 inputs (2 conv + 3 fc)."""

    def __init__(self, num_classes: int = 10) -> None:
        super().__init__()
        self.conv1 = torch.nn.Conv2d(1, 6, 5, padding=2)
        self.conv2 = torch.nn.Conv2d(6, 16, 5)
        self.fc1 = torch.nn.Linear(16 * 5 * 5, 120)
        self.fc2 = torch.nn.Linear(120, 84)
        self.fc3 = torch.nn.Linear(84, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = F.max_pool2d(F.relu(self.conv1(x)), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return self.fc3(x)
