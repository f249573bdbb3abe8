"""GPT-NeoX K-FAC on the native GPU path.

At mp=1 the tensor-parallel eigen layers run the grouped MFMA GEMM
(``GroupedPrecondition``) and the multi-tensor KL clip / apply
(``MultiLayerApply``); the result must match the CPU per-layer path.  The
model-parallel KL hook (fold partials -> one scalar all-reduce -> finalise)
is checked directly against an fp64 reference.
"""
from __future__ import annotations

import copy
import types
import warnings

import pytest
import torch

from distributed_kfac_pytorch_amd.models.gpt_neox import GPTNeoX
from distributed_kfac_pytorch_amd.neox.pipeline import PipelineModule
from distributed_kfac_pytorch_amd.neox.preconditioner import GPTNeoXKFACPreconditioner
from distributed_kfac_pytorch_amd.neox.topology import PipeModelDataParallelTopology
from distributed_kfac_pytorch_amd.ops import precondition as pops
from distributed_kfac_pytorch_amd.warnings import ExperimentalFeatureWarning

pytestmark = pytest.mark.gpu
warnings.filterwarnings('ignore', category=ExperimentalFeatureWarning)


def _model() -> torch.nn.Module:
    topo = PipeModelDataParallelTopology(num_pp=1, num_mp=1, num_dp=1)
    torch.manual_seed(0)
    return PipelineModule(
        [lambda: GPTNeoX(vocab=64, hidden=64, layers=2, heads=4, group=None)], topo, rank=0)


@pytest.mark.parametrize('prediv', [False, True])
def test_neox_grouped_gpu_matches_cpu(cuda, prediv):
    cpu = _model()
    gpu = copy.deepcopy(cpu).to(cuda)
    kw = dict(factor_update_steps=1, inv_update_steps=2, lr=0.1, kl_clip=0.01,
              compute_eigenvalue_outer_product=prediv)
    pc = GPTNeoXKFACPreconditioner(cpu, **kw)
    pg = GPTNeoXKFACPreconditioner(gpu, **kw)
    g = torch.Generator().manual_seed(3)
    for _ in range(4):
        tok = torch.randint(0, 64, (4, 17), generator=g)
        for model, pre, t in ((cpu, pc, tok), (gpu, pg, tok.to(cuda))):
            model.zero_grad(set_to_none=False)
            logits = model(t[:, :-1])
            torch.nn.functional.cross_entropy(logits.flatten(0, 1).float(),
                                              t[:, 1:].flatten()).backward()
            pre.step()
        for (name, a), b in zip(cpu.named_parameters(), gpu.parameters()):
            err = (a.grad - b.grad.cpu()).abs().max() / a.grad.abs().max().clamp_min(1e-12)
            assert err < 2e-3, (name, float(err))
        with torch.no_grad():
            for a, b in zip(cpu.parameters(), gpu.parameters()):
                a -= 0.1 * a.grad
                b -= 0.1 * b.grad
    # the native paths ran (not the per-layer torch fallback)
    assert pg._grouped is not None and pg._grouped._key is not None
    assert pg._multi_apply is not None and pg._multi_apply._key is not None


def _fake_layer(rows: int, cols: int, bias: bool, bscale: float, dev: torch.device):
    w = torch.randn(rows, cols, device=dev)
    b = torch.randn(rows, device=dev) if bias else None
    p = torch.randn(rows, cols + int(bias), device=dev)
    helper = types.SimpleNamespace(
        get_weight_grad=lambda: w, weight_grad_matrix=lambda: w,
        has_bias=lambda: bias, get_bias_grad=lambda: b)
    return types.SimpleNamespace(grad=p, module=helper, kl_bias_scale=bscale, _p=p.clone(),
                                 _w=w.clone(), _b=None if b is None else b.clone())


def test_multi_apply_mp_reduce_hook(cuda):
    torch.manual_seed(0)
    layers = [_fake_layer(96, 130, True, 0.5, cuda), _fake_layer(33, 64, False, 1.0, cuda),
              _fake_layer(257, 17, True, 1.0, cuda)]
    vg = 0.0
    for l in layers:
        vg += float((l._p[:, :l._w.shape[1]].double() * l._w.double()).sum())
        if l._b is not None:
            vg += float((l._p[:, -1].double() * l._b.double()).sum()) * l.kl_bias_scale
    seen = []

    def reduce_fn(t: torch.Tensor) -> None:  # stands in for the MP all-reduce
        seen.append(float(t))
        t.mul_(3.0)

    kl, lr = 1e-3, 0.05
    assert pops.MultiLayerApply().run(layers, kl, lr, reduce_fn=reduce_fn)
    torch.cuda.synchronize()
    assert len(seen) == 1 and abs(seen[0] - vg) <= 1e-9 * max(1.0, abs(vg))
    scale = min(1.0, (kl / abs(3.0 * vg * lr * lr)) ** 0.5)
    for l in layers:
        ncol = l._w.shape[1]
        torch.testing.assert_close(l.module.get_weight_grad(), scale * l._p[:, :ncol],
                                   rtol=1e-6, atol=1e-6)
        if l._b is not None:
            torch.testing.assert_close(l.module.get_bias_grad(), scale * l._p[:, -1],
                                       rtol=1e-6, atol=1e-6)
