"""GPT-NeoX-style decoder with Megatron tensor parallelism.

Used for BASELINE config #5 (GPT-NeoX 125M with model-parallel K-FAC
factors) and the TP/PP tests.  Per block (NeoX "parallel residual"):

    x = x + Attn(LN1(x)) + MLP(LN2(x))
    Attn: QKV = ColumnParallelLinear(h, 3h, gather_output=False)
          (heads split across MP ranks) -> causal SDPA ->
          dense = RowParallelLinear(h, h, input_is_parallel=True)
    MLP:  h_to_4h = ColumnParallelLinear(h, 4h, gather_output=False) -> GELU
          -> 4h_to_h = RowParallelLinear(4h, h, input_is_parallel=True)

Rotary position embeddings on the full head dim; token embedding and LM
head replicated (the reference registers only the parallel linears).
``gpt_neox_125m()`` = hidden 768, 12 layers, 12 heads, seq 2048, which gives
48 K-FAC layers with factor dims up to 3073.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.neox.tp_layers import ColumnParallelLinear
from distributed_kfac_pytorch_amd.neox.tp_layers import RowParallelLinear
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size


def _rotary(x: torch.Tensor, base: float = 10000.0) -> torch.Tensor:
    """Apply rotary embeddings to [B, H, T, D]."""
    t, d = x.shape[-2], x.shape[-1]
    inv = 1.0 / (base ** (torch.arange(0, d, 2, device=x.device, dtype=torch.float32) / d))
    ang = torch.arange(t, device=x.device, dtype=torch.float32)[:, None] * inv[None]
    cos, sin = ang.cos().to(x.dtype), ang.sin().to(x.dtype)
    x1, x2 = x[..., 0::2], x[..., 1::2]
    out = torch.stack([x1 * cos - x2 * sin, x1 * sin + x2 * cos], dim=-1)
    return out.flatten(-2)


class ParallelAttention(torch.nn.Module):
    def __init__(self, hidden: int, heads: int, group: dist.ProcessGroup | None, seed: int) -> None:
        super().__init__()
        mp = get_world_size(group)
        if heads % mp != 0:
            raise ValueError('heads must be divisible by the MP size')
        self.local_heads = heads // mp
        self.head_dim = hidden // heads
        self.query_key_value = ColumnParallelLinear(
            hidden, 3 * hidden, gather_output=False, group=group, init_seed=seed,
        )
        self.dense = RowParallelLinear(
            hidden, hidden, input_is_parallel=True, group=group, init_seed=seed + 1,
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, t, _ = x.shape
        qkv = self.query_key_value(x).view(b, t, self.local_heads, 3 * self.head_dim)
        q, k, v = qkv.permute(0, 2, 1, 3).split(self.head_dim, dim=-1)
        q, k = _rotary(q), _rotary(k)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        o = o.permute(0, 2, 1, 3).reshape(b, t, self.local_heads * self.head_dim)
        return self.dense(o)


class ParallelMLP(torch.nn.Module):
    def __init__(self, hidden: int, group: dist.ProcessGroup | None, seed: int) -> None:
        super().__init__()
        self.dense_h_to_4h = ColumnParallelLinear(
            hidden, 4 * hidden, gather_output=False, group=group, init_seed=seed,
        )
        self.dense_4h_to_h = RowParallelLinear(
            4 * hidden, hidden, input_is_parallel=True, group=group, init_seed=seed + 1,
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.dense_4h_to_h(F.gelu(self.dense_h_to_4h(x)))


class GPTNeoXBlock(torch.nn.Module):
    def __init__(self, hidden: int, heads: int, group: dist.ProcessGroup | None, seed: int) -> None:
        super().__init__()
        self.input_layernorm = torch.nn.LayerNorm(hidden)
        self.post_attention_layernorm = torch.nn.LayerNorm(hidden)
        self.attention = ParallelAttention(hidden, heads, group, seed)
        self.mlp = ParallelMLP(hidden, group, seed + 2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x + self.attention(self.input_layernorm(x)) + self.mlp(
            self.post_attention_layernorm(x),
        )


EMBED_SEED = 7919
HEAD_SEED = 7927


def _seeded_embedding(vocab: int, hidden: int, seed: int) -> torch.nn.Embedding:
    # independent of the global RNG, so a pipeline stage that builds only
    # some of the layers gets the same weights as the whole model
    e = torch.nn.Embedding(vocab, hidden)
    with torch.no_grad():
        e.weight.normal_(generator=torch.Generator().manual_seed(seed))
    return e


def _seeded_head(hidden: int, vocab: int, seed: int) -> torch.nn.Linear:
    lin = torch.nn.Linear(hidden, vocab, bias=False)
    bound = 1.0 / hidden ** 0.5
    with torch.no_grad():
        lin.weight.uniform_(-bound, bound, generator=torch.Generator().manual_seed(seed))
    return lin


class GPTNeoXEmbedding(torch.nn.Module):
    """First pipeline layer: token embedding."""

    def __init__(self, vocab: int, hidden: int) -> None:
        super().__init__()
        self.embed_in = _seeded_embedding(vocab, hidden, EMBED_SEED)

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        return self.embed_in(tokens)


class GPTNeoXHead(torch.nn.Module):
    """Last pipeline layer: final LayerNorm + LM head (logits)."""

    def __init__(self, hidden: int, vocab: int) -> None:
        super().__init__()
        self.final_layer_norm = torch.nn.LayerNorm(hidden)
        self.embed_out = _seeded_head(hidden, vocab, HEAD_SEED)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.embed_out(self.final_layer_norm(x))


class GPTNeoX(torch.nn.Module):
    def __init__(
        self,
        vocab: int = 50304,
        hidden: int = 768,
        layers: int = 12,
        heads: int = 12,
        group: dist.ProcessGroup | None = None,
    ) -> None:
        super().__init__()
        self.embed_in = _seeded_embedding(vocab, hidden, EMBED_SEED)
        self.layers = torch.nn.ModuleList(
            [GPTNeoXBlock(hidden, heads, group, seed=100 * i) for i in range(layers)],
        )
        self.final_layer_norm = torch.nn.LayerNorm(hidden)
        self.embed_out = _seeded_head(hidden, vocab, HEAD_SEED)

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        x = self.embed_in(tokens)
        for blk in self.layers:
            x = blk(x)
        return self.embed_out(self.final_layer_norm(x))


def gpt_neox_pipeline_layers(
    vocab: int = 50304,
    hidden: int = 768,
    layers: int = 12,
    heads: int = 12,
    group: dist.ProcessGroup | None = None,
) -> list:
    """Layer constructors for ``neox.pipeline.PipelineModule``: embedding,
    the blocks, the head -- weight for weight the layers of ``GPTNeoX`` with
    the same arguments, whatever the stage partition."""
    out: list = [lambda: GPTNeoXEmbedding(vocab, hidden)]
    for i in range(layers):
        out.append(lambda i=i: GPTNeoXBlock(hidden, heads, group, seed=100 * i))
    out.append(lambda: GPTNeoXHead(hidden, vocab))
    return out


def gpt_neox_125m(group: dist.ProcessGroup | None = None, vocab: int = 50304) -> GPTNeoX:
    return GPTNeoX(vocab=vocab, hidden=768, layers=12, heads=12, group=group)
