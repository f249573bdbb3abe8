"""Embedding K-FAC (diagonal A factor) against the dense one-hot formulation."""
from __future__ import annotations

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.layers.embedding import EmbeddingModuleHelper
from distributed_kfac_pytorch_amd.layers.embedding import KFACEmbeddingEigenLayer
from distributed_kfac_pytorch_amd.layers.embedding import KFACEmbeddingInverseLayer
from distributed_kfac_pytorch_amd.models.transformer import TransformerLM
from distributed_kfac_pytorch_amd.parallel.comm import TorchDistributedCommunicator


def test_helper_factor_is_token_frequency():
    emb = torch.nn.Embedding(7, 3)
    h = EmbeddingModuleHelper(emb)
    assert h.a_factor_shape == (7, 7) and h.g_factor_shape == (3, 3)
    ids = torch.tensor([[0, 1, 1], [6, 1, 0]])
    a = h.get_a_factor(ids)
    onehot = torch.nn.functional.one_hot(ids.reshape(-1), 7).float()
    assert torch.allclose(torch.diag(a), onehot.t() @ onehot / 6)
    with pytest.raises(ValueError):
        EmbeddingModuleHelper(torch.nn.Embedding(4, 2, sparse=True))


@pytest.mark.parametrize('prediv', [True, False])
def test_eigen_embedding_matches_dense_linear(prediv):
    torch.manual_seed(0)
    v, d = 9, 4
    emb = torch.nn.Embedding(v, d)
    ids = torch.randint(0, v, (5, 6))
    out = emb(ids)
    g = torch.randn_like(out)
    out.backward(g)
    layer = KFACEmbeddingEigenLayer(
        EmbeddingModuleHelper(emb), tdc=TorchDistributedCommunicator(),
        prediv_eigenvalues=prediv,
    )
    layer.save_layer_input([ids])
    layer.save_layer_grad_output((g,))
    layer.update_a_factor(0.0)
    layer.update_g_factor(0.0)
    layer.compute_a_inv(0.1)
    layer.compute_g_inv(0.1)
    layer.preconditioned_grad(0.1)
    # dense reference: linear layer on one-hot inputs, W = E^T
    x = torch.nn.functional.one_hot(ids.reshape(-1), v).double()
    A = x.t() @ x / x.shape[0]
    gg = g.reshape(-1, d).double()
    G = gg.t() @ gg / gg.shape[0]
    da, qa = torch.linalg.eigh(A)
    dg, qg = torch.linalg.eigh(G)
    grad = emb.weight.grad.t().double()
    vv = qg.t() @ grad @ qa
    vv = vv / (torch.outer(dg.clamp(min=0), da.clamp(min=0)) + 0.1)
    ref = qg @ vv @ qa.t()
    assert torch.allclose(layer.grad.double(), ref, atol=1e-5)
    layer.update_grad()
    assert torch.allclose(emb.weight.grad.double(), ref.t(), atol=1e-5)


def test_inverse_embedding():
    emb = torch.nn.Embedding(5, 2)
    ids = torch.tensor([0, 0, 3, 4])
    out = emb(ids)
    out.sum().backward()
    layer = KFACEmbeddingInverseLayer(EmbeddingModuleHelper(emb), tdc=TorchDistributedCommunicator())
    layer.save_layer_input([ids])
    layer.save_layer_grad_output((torch.ones_like(out),))
    layer.update_a_factor(0.0)
    layer.update_g_factor(0.0)
    layer.compute_a_inv(0.5)
    layer.compute_g_inv(0.5)
    assert torch.allclose(layer.a_inv, 1 / (torch.tensor([0.5, 0, 0, 0.25, 0.25]) + 0.5))
    layer.preconditioned_grad(0.5)
    assert layer.grad.shape == (2, 5)


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
def test_lm_with_embeddings_trains(method):
    torch.manual_seed(0)
    model = TransformerLM(ntoken=50, d_model=16, nhead=2, d_hid=16, nlayers=1, dropout=0.0)
    pre = kfac.KFACPreconditioner(
        model, register_embeddings=True, compute_method=method,
        skip_layers=['self_attn'], factor_update_steps=1, inv_update_steps=2,
    )
    names = [n for n, _ in pre._layers.values()]
    assert names[0] == 'embedding' and 'decoder' in names
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    x = torch.randint(0, 50, (4, 12))
    losses = []
    for _ in range(15):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x[:, :-1]).flatten(0, 1), x[:, 1:].flatten())
        loss.backward()
        pre.step()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    sd = pre.state_dict()
    assert sd['layers']['embedding']['A'].shape == (50,)
    pre2 = kfac.KFACPreconditioner(
        TransformerLM(ntoken=50, d_model=16, nhead=2, d_hid=16, nlayers=1, dropout=0.0),
        register_embeddings=True, compute_method=method, skip_layers=['self_attn'],
    )
    pre2.load_state_dict(sd)
    assert pre2.steps == 15


def test_embeddings_off_by_default():
    model = TransformerLM(ntoken=20, d_model=8, nhead=2, d_hid=8, nlayers=1)
    pre = kfac.KFACPreconditioner(model)
    assert 'embedding' not in [n for n, _ in pre._layers.values()]
