"""Transformer LM (reference ``examples/language/transformer.py``); the
model lives in :mod:`distributed_kfac_pytorch_amd.models.transformer`."""
from distributed_kfac_pytorch_amd.models.transformer import causal_mask
from distributed_kfac_pytorch_amd.models.transformer import PositionalEncoding
from distributed_kfac_pytorch_amd.models.transformer import TransformerLM

TransformerModel = TransformerLM
gen_square_subsequent_mask = causal_mask

__all__ = ['causal_mask', 'gen_square_subsequent_mask', 'PositionalEncoding',
           'TransformerLM', 'TransformerModel']
