"""Transformer language model (reference ``examples/language/transformer.py``).

Token embedding (scaled by sqrt(d_model)) + sinusoidal positional encoding
-> ``nn.TransformerEncoder`` with a causal mask -> Linear decoder.  Defaults
follow the reference LM example (d_model 256, d_hid 256, 4 heads, 2 layers).

Unlike the reference (batch-first data fed to a
sequence-first encoder, mask sized by the batch) this model is batch-first
end to end: inputs are ``[batch, seq]`` token ids.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn


class PositionalEncoding(nn.Module):
    def __init__(self, d_model: int, dropout: float = 0.1, max_len: int = 5000) -> None:
        super().__init__()
        self.dropout = nn.Dropout(p=dropout)
        pos = torch.arange(max_len).unsqueeze(1)
        div = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
        pe = torch.zeros(1, max_len, d_model)
        pe[0, :, 0::2] = torch.sin(pos * div)
        pe[0, :, 1::2] = torch.cos(pos * div[: d_model // 2])
        self.register_buffer('pe', pe)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.dropout(x + self.pe[:, : x.shape[1]])


def causal_mask(seq_len: int, device: torch.device | None = None) -> torch.Tensor:
    """Additive float mask: -inf above the diagonal."""
    return torch.triu(
        torch.full((seq_len, seq_len), float('-inf'), device=device),
        diagonal=1,
    )


class TransformerLM(nn.Module):
    def __init__(
        self,
        ntoken: int,
        d_model: int = 256,
        nhead: int = 4,
        d_hid: int = 256,
        nlayers: int = 2,
        dropout: float = 0.2,
    ) -> None:
        super().__init__()
        self.d_model = d_model
        self.embedding = nn.Embedding(ntoken, d_model)
        self.pos_encoder = PositionalEncoding(d_model, dropout)
        layer = nn.TransformerEncoderLayer(
            d_model, nhead, d_hid, dropout, batch_first=True,
        )
        self.transformer_encoder = nn.TransformerEncoder(
            layer, nlayers, enable_nested_tensor=False,
        )
        self.decoder = nn.Linear(d_model, ntoken)
        r = 0.1
        self.embedding.weight.data.uniform_(-r, r)
        self.decoder.bias.data.zero_()
        self.decoder.weight.data.uniform_(-r, r)

    def forward(self, src: torch.Tensor, src_mask: torch.Tensor | None = None) -> torch.Tensor:
        if src_mask is None:
            src_mask = causal_mask(src.shape[1], src.device)
        x = self.embedding(src) * math.sqrt(self.d_model)
        x = self.pos_encoder(x)
        x = self.transformer_encoder(x, src_mask, is_causal=True)
        return self.decoder(x)
