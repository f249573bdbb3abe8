"""Language-model data (reference ``examples/language/dataset.py:40-195``).

The reference downloads PTB / WikiText through torchtext.  Here (no network,
no torchtext) a dataset is either a local directory holding the standard
split files (``train.txt``/``valid.txt``/``test.txt`` or the WikiText
``wiki.{train,valid,test}.tokens`` names), tokenised by whitespace with a
shared vocabulary, or -- when absent -- synthetic token streams with the
named dataset's vocabulary size.  Sequences are fixed ``seq_len`` chunks of
the flattened token stream, sharded per rank by ``DistributedSampler``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

from torch.utils.data import DataLoader
from torch.utils.data import Dataset
from torch.utils.data.distributed import DistributedSampler

from distributed_kfac_pytorch_amd.utils.data import SyntheticTokens
from distributed_kfac_pytorch_amd.utils.data import TokenFile

# vocabulary sizes of the reference datasets (torchtext basic_english)
VOCAB_SIZES = {'penntreebank': 9_922, 'wikitext2': 28_782, 'wikitext103': 267_735}
_SPLIT_NAMES = {
    'train': ('train.txt', 'wiki.train.tokens', 'ptb.train.txt'),
    'val': ('valid.txt', 'wiki.valid.tokens', 'ptb.valid.txt'),
    'test': ('test.txt', 'wiki.test.tokens', 'ptb.test.txt'),
}


@dataclass
class Split:
    dataset: Dataset
    sampler: DistributedSampler
    loader: DataLoader


@dataclass
class LMData:
    train: Split
    val: Split
    test: Split
    vocab_size: int
    source: str


def _find(root: str, split: str) -> str | None:
    for name in _SPLIT_NAMES[split]:
        p = os.path.join(root, name)
        if os.path.exists(p):
            return p
    return None


def get_dataset(name: str, data_dir: str | None, *, seq_len: int, batch_size: int,
                rank: int, world_size: int, cuda: bool, synthetic_tokens: int = 1_000_000
                ) -> LMData:
    paths = {s: _find(data_dir, s) for s in _SPLIT_NAMES} if data_dir else {}
    if paths and all(paths.values()):
        vocab: dict[str, int] = {}
        sets = {s: TokenFile(paths[s], seq_len, vocab) for s in ('train', 'val', 'test')}
        vocab_size, source = len(vocab), f'text:{data_dir}'
    else:
        vocab_size = VOCAB_SIZES.get(name, 33_278)
        n = max(1, synthetic_tokens // seq_len)
        sets = {
            'train': SyntheticTokens(n, seq_len, vocab_size, seed=1),
            'val': SyntheticTokens(max(1, n // 10), seq_len, vocab_size, seed=2),
            'test': SyntheticTokens(max(1, n // 10), seq_len, vocab_size, seed=3),
        }
        source = f'synthetic ({name} vocab {vocab_size})'
    out = {}
    for s, ds in sets.items():
        sampler = DistributedSampler(ds, num_replicas=world_size, rank=rank,
                                     shuffle=(s == 'train'))
        loader = DataLoader(ds, batch_size=batch_size, sampler=sampler,
                            drop_last=(s == 'train'), pin_memory=cuda)
        out[s] = Split(ds, sampler, loader)
    return LMData(out['train'], out['val'], out['test'], vocab_size, source)
