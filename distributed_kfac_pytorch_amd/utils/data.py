"""Datasets for the examples (reference ``examples/vision/datasets.py``,
``examples/language/dataset.py``).

This image has no network and no torchvision / torchtext, so:

* ``SyntheticImages`` / ``SyntheticTokens``: deterministic random data of
  the real shapes (ImageNet 3x224x224 / CIFAR 3x32x32 / token streams),
  generated per index so every rank sees a different, reproducible shard.
* ``CifarBinary``: reads the CIFAR-10 *binary* release
  (``data_batch_{1..5}.bin`` / ``test_batch.bin``) when present locally --
  raw bytes, no unpickling.
* ``TokenFile``: a whitespace-tokenised text file -> fixed-length
  sequences, vocabulary built in first-seen order.
Each has a ``DistributedSampler``-friendly ``__len__`` / ``__getitem__``.
"""
from __future__ import annotations

import os

import torch
from torch.utils.data import Dataset


class SyntheticImages(Dataset):
    def __init__(self, n: int, shape: tuple[int, int, int] = (3, 224, 224),
                 num_classes: int = 1000, seed: int = 0) -> None:
        self.n, self.shape, self.num_classes, self.seed = n, shape, num_classes, seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int) -> tuple[torch.Tensor, int]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        x = torch.randn(self.shape, generator=g)
        y = int(torch.randint(0, self.num_classes, (1,), generator=g))
        return x, y


class SyntheticTokens(Dataset):
    """Random token sequences; the target is the input shifted by one."""

    def __init__(self, n: int, seq_len: int = 64, vocab: int = 33278, seed: int = 0) -> None:
        self.n, self.seq_len, self.vocab, self.seed = n, seq_len, vocab, seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int) -> tuple[torch.Tensor, torch.Tensor]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        s = torch.randint(0, self.vocab, (self.seq_len + 1,), generator=g)
        return s[:-1], s[1:]


class CifarBinary(Dataset):
    """CIFAR-10 binary format: records of 1 label byte + 3072 pixel bytes."""

    MEAN = (0.4914, 0.4822, 0.4465)
    STD = (0.2470, 0.2435, 0.2616)

    def __init__(self, root: str, train: bool = True) -> None:
        files = (
            [f'data_batch_{i}.bin' for i in range(1, 6)] if train else ['test_batch.bin']
        )
        chunks = []
        for f in files:
            path = os.path.join(root, f)
            with open(path, 'rb') as fh:
                chunks.append(torch.frombuffer(bytearray(fh.read()), dtype=torch.uint8))
        raw = torch.cat(chunks).view(-1, 3073)
        self.labels = raw[:, 0].long()
        x = raw[:, 1:].view(-1, 3, 32, 32).float() / 255.0
        mean = torch.tensor(self.MEAN).view(1, 3, 1, 1)
        std = torch.tensor(self.STD).view(1, 3, 1, 1)
        self.images = (x - mean) / std
        self.train = train

    @staticmethod
    def available(root: str) -> bool:
        return os.path.exists(os.path.join(root, 'data_batch_1.bin'))

    def __len__(self) -> int:
        return self.labels.shape[0]

    def __getitem__(self, i: int) -> tuple[torch.Tensor, int]:
        x = self.images[i]
        if self.train:  # random crop (pad 4) + horizontal flip
            if torch.rand(()) < 0.5:
                x = x.flip(-1)
            xp = torch.nn.functional.pad(x, (4, 4, 4, 4))
            dy, dx = torch.randint(0, 9, (2,)).tolist()
            x = xp[:, dy: dy + 32, dx: dx + 32]
        return x, int(self.labels[i])


class TokenFile(Dataset):
    def __init__(self, path: str, seq_len: int, vocab: dict[str, int] | None = None) -> None:
        self.vocab = {} if vocab is None else vocab
        ids = []
        with open(path, encoding='utf-8') as f:
            for line in f:
                for w in line.split() + ['<eos>']:
                    if w not in self.vocab:
                        self.vocab[w] = len(self.vocab)
                    ids.append(self.vocab[w])
        data = torch.tensor(ids, dtype=torch.long)
        n = (data.numel() - 1) // seq_len
        self.inputs = data[: n * seq_len].view(n, seq_len)
        self.targets = data[1: n * seq_len + 1].view(n, seq_len)

    def __len__(self) -> int:
        return self.inputs.shape[0]

    def __getitem__(self, i: int) -> tuple[torch.Tensor, torch.Tensor]:
        return self.inputs[i], self.targets[i]
