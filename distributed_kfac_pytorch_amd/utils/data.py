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


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
_IMG_EXT = ('.jpg', '.jpeg', '.png', '.bmp', '.webp', '.JPEG')


class ImageFolder(Dataset):
    """``root/<class>/<image>`` dataset decoded with PIL (torchvision is not
    available in this image).  Train: RandomResizedCrop(size, scale
    (0.08, 1), ratio (3/4, 4/3)) + horizontal flip; eval: resize the short
    side to ``size*8/7`` then center crop -- the standard ImageNet recipe
    the reference gets from torchvision (``examples/vision/datasets.py:
    71-151``).  Returns a normalised float CHW tensor and the class index.
    """

    def __init__(self, root: str, train: bool = True, size: int = 224) -> None:
        self.classes = sorted(
            d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))
        )
        self.samples: list[tuple[str, int]] = []
        for ci, c in enumerate(self.classes):
            for dirpath, _, files in sorted(os.walk(os.path.join(root, c))):
                for f in sorted(files):
                    if f.endswith(_IMG_EXT):
                        self.samples.append((os.path.join(dirpath, f), ci))
        self.train, self.size = train, size
        self._mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
        self._std = torch.tensor(IMAGENET_STD).view(3, 1, 1)

    def __len__(self) -> int:
        return len(self.samples)

    def _random_resized_crop(self, img):  # type: ignore[no-untyped-def]
        import math
        import random
        w, h = img.size
        area = w * h
        for _ in range(10):
            target = area * random.uniform(0.08, 1.0)
            ar = math.exp(random.uniform(math.log(3 / 4), math.log(4 / 3)))
            cw = int(round(math.sqrt(target * ar)))
            ch = int(round(math.sqrt(target / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                x0 = random.randint(0, w - cw)
                y0 = random.randint(0, h - ch)
                return img.crop((x0, y0, x0 + cw, y0 + ch))
        s = min(w, h)
        return img.crop(((w - s) // 2, (h - s) // 2, (w - s) // 2 + s, (h - s) // 2 + s))

    def __getitem__(self, i: int) -> tuple[torch.Tensor, int]:
        import random

        import numpy as np
        from PIL import Image
        path, label = self.samples[i]
        with Image.open(path) as im:
            img = im.convert('RGB')
        if self.train:
            img = self._random_resized_crop(img).resize((self.size, self.size), Image.BILINEAR)
            if random.random() < 0.5:
                img = img.transpose(Image.FLIP_LEFT_RIGHT)
        else:
            short = int(self.size * 8 / 7)
            w, h = img.size
            scale = short / min(w, h)
            img = img.resize((max(short, round(w * scale)), max(short, round(h * scale))),
                             Image.BILINEAR)
            w, h = img.size
            x0, y0 = (w - self.size) // 2, (h - self.size) // 2
            img = img.crop((x0, y0, x0 + self.size, y0 + self.size))
        x = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1)
        x = (x.float() / 255.0 - self._mean) / self._std
        return x, label
