"""End-to-end: the native GPU path reproduces the CPU reference math."""
from __future__ import annotations

import copy

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac

pytestmark = pytest.mark.gpu


def _net() -> torch.nn.Module:
    torch.manual_seed(0)
    return torch.nn.Sequential(
        torch.nn.Conv2d(3, 16, 3, padding=1, stride=2),
        torch.nn.ReLU(),
        torch.nn.Conv2d(16, 16, 3, bias=False),
        torch.nn.ReLU(),
        torch.nn.Conv2d(16, 32, 1),
        torch.nn.Flatten(),
        torch.nn.Linear(32 * 5 * 5, 10),
    )


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
@pytest.mark.parametrize('channels_last', [False, True])
@pytest.mark.parametrize('prediv', [True, False])
def test_gpu_matches_cpu(cuda, method, channels_last, prediv):
    cpu = _net()
    gpu = copy.deepcopy(cpu).to(cuda)
    if channels_last:
        gpu = gpu.to(memory_format=torch.channels_last)
    kw = dict(
        factor_update_steps=1,
        inv_update_steps=2,
        compute_method=method,
        compute_eigenvalue_outer_product=prediv,
        lr=0.1,
        kl_clip=0.001,
    )
    pc = kfac.KFACPreconditioner(cpu, **kw)
    pg = kfac.KFACPreconditioner(gpu, **kw)
    oc = torch.optim.SGD(cpu.parameters(), lr=0.1)
    og = torch.optim.SGD(gpu.parameters(), lr=0.1)
    torch.manual_seed(1)
    for _ in range(4):
        x = torch.randn(8, 3, 14, 14)
        y = torch.randint(0, 10, (8,))
        xg = x.to(cuda)
        if channels_last:
            xg = xg.contiguous(memory_format=torch.channels_last)
        oc.zero_grad()
        torch.nn.functional.cross_entropy(cpu(x), y).backward()
        pc.step()
        og.zero_grad()
        torch.nn.functional.cross_entropy(gpu(xg), y.to(cuda)).backward()
        pg.step()
        for a, b in zip(cpu.parameters(), gpu.parameters()):
            err = (a.grad - b.grad.cpu()).abs().max().item()
            assert err <= 2e-3 * a.grad.abs().max().item() + 1e-7
        oc.step()
        og.step()
    # checkpoints are interchangeable (reference order on both)
    sc, sg = pc.state_dict(), pg.state_dict()
    for name in sc['layers']:
        for f in 'AG':
            a = sc['layers'][name][f]
            b = sg['layers'][name][f].cpu()
            assert (a - b).abs().max().item() <= 1e-3 * a.abs().max().item()


def test_bf16_autocast_resnet_smoke(cuda):
    from distributed_kfac_pytorch_amd.models.resnet import resnet18

    model = resnet18(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
    pre = kfac.KFACPreconditioner(
        model,
        factor_update_steps=1,
        inv_update_steps=2,
        grad_worker_fraction=0.5,
    )
    x = torch.randn(4, 3, 64, 64, device=cuda).contiguous(
        memory_format=torch.channels_last,
    )
    y = torch.randint(0, 10, (4,), device=cuda)
    for _ in range(3):
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        pre.step()
        opt.step()
    assert torch.isfinite(loss).item()
    for p in model.parameters():
        assert torch.isfinite(p).all()


@pytest.mark.parametrize('prediv', [True, False])
@pytest.mark.parametrize('method', ['eigen', 'inverse'])
def test_graph_replay_matches_eager(cuda, prediv, method):
    """HIP-graph replay of precondition+apply == eager execution."""
    base = _net().to(cuda).to(memory_format=torch.channels_last)
    models = [copy.deepcopy(base), copy.deepcopy(base)]
    pres = [
        kfac.KFACPreconditioner(
            m,
            factor_update_steps=1,
            inv_update_steps=4,
            compute_method=method,
            compute_eigenvalue_outer_product=prediv,
            lr=lambda s: 0.1 / (1 + s),
        )
        for m in models
    ]
    from distributed_kfac_pytorch_amd.base_preconditioner import StepGraphs

    pres[0]._graphs = StepGraphs()  # opt-in (KFAC_GRAPHS=1)
    pres[1]._graphs = None  # eager reference
    opts = [torch.optim.SGD(m.parameters(), lr=0.05) for m in models]
    torch.manual_seed(2)
    for _ in range(10):
        x = torch.randn(8, 3, 14, 14, device=cuda).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), device=cuda)
        for m, p, o in zip(models, pres, opts):
            o.zero_grad(set_to_none=False)
            torch.nn.functional.cross_entropy(m(x), y).backward()
            p.step()
        for a, b in zip(models[0].parameters(), models[1].parameters()):
            # MIOpen backward is not bitwise deterministic (raw grads differ
            # by ~1e-6) and the bf16x3 GEMMs are accurate to ~1e-5 of the
            # largest entry: compare against the tensor's scale
            assert (a.grad - b.grad).abs().max() <= 2e-4 * b.grad.abs().max() + 1e-7
        for o in opts:
            o.step()
    assert pres[0]._graphs.replays > 0 and pres[0]._graphs.captures >= 1


def test_factor_side_stream_matches_inline(cuda, monkeypatch):
    """Factor SYRK/EMA on the hook side stream == inline on the compute
    stream; an input mutated after its hook switches to inline updates."""
    base = _net().to(cuda)
    models = [copy.deepcopy(base), copy.deepcopy(base)]
    pres = [
        kfac.KFACPreconditioner(m, factor_update_steps=1, inv_update_steps=3, lr=0.1)
        for m in models
    ]
    pres[1]._factor_stream_off = True  # inline reference
    torch.manual_seed(3)
    for _ in range(4):
        x = torch.randn(8, 3, 14, 14, device=cuda)
        y = torch.randint(0, 10, (8,), device=cuda)
        for m, p in zip(models, pres):
            m.zero_grad(set_to_none=False)
            torch.nn.functional.cross_entropy(m(x), y).backward()
            p.step()
        assert pres[0]._factor_streams, 'side stream was not used'
        for (_, la), (_, lb) in zip(pres[0]._layers.values(), pres[1]._layers.values()):
            assert torch.allclose(la.a_factor, lb.a_factor, rtol=1e-5, atol=1e-6)
            assert torch.allclose(la.g_factor, lb.g_factor, rtol=1e-5, atol=1e-6)
    x = torch.randn(8, 3, 14, 14, device=cuda)
    torch.nn.functional.cross_entropy(models[0](x), y).backward()
    x.add_(1.0)  # first layer's input changes after its forward hook
    with pytest.warns(UserWarning, match='modified in place'):
        pres[0].step()
    assert pres[0]._factor_stream_off


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
def test_embedding_kfac_gpu_matches_cpu(cuda, method):
    """nn.Embedding K-FAC (diagonal A, register_embeddings=True) on the GPU
    path (native G SYRK, grouped / per-layer preconditioning, multi-tensor
    apply) against the CPU reference math."""
    from distributed_kfac_pytorch_amd.models.transformer import TransformerLM

    torch.manual_seed(0)
    cpu = TransformerLM(ntoken=50, d_model=32, nhead=4, d_hid=32, nlayers=1, dropout=0.0)
    gpu = copy.deepcopy(cpu).to(cuda)
    kw = dict(factor_update_steps=1, inv_update_steps=2, compute_method=method, lr=0.1,
              kl_clip=0.001, register_embeddings=True, skip_layers=['self_attn'])
    pc = kfac.KFACPreconditioner(cpu, **kw)
    pg = kfac.KFACPreconditioner(gpu, **kw)
    assert any('Embedding' in type(l).__name__ for _, l in pg._layers.values())
    g = torch.Generator().manual_seed(2)
    for _ in range(4):
        tok = torch.randint(0, 50, (6, 9), generator=g)
        for model, pre, t in ((cpu, pc, tok), (gpu, pg, tok.to(cuda))):
            model.zero_grad()
            out = model(t[:, :-1])
            torch.nn.functional.cross_entropy(out.reshape(-1, 50), t[:, 1:].reshape(-1)).backward()
            pre.step()
        for a, b in zip(cpu.parameters(), gpu.parameters()):
            err = (a.grad - b.grad.cpu()).abs().max() / a.grad.abs().max().clamp_min(1e-12)
            assert err < 2e-3, float(err)
        with torch.no_grad():
            for a, b in zip(cpu.parameters(), gpu.parameters()):
                a -= 0.1 * a.grad
                b -= 0.1 * b.grad


def test_grad_scaler_unscale_on_device_no_sync(cuda):
    """With a GradScaler the G contributions are unscaled by 1/s^2 on the
    device (the scale tensor feeds the SYRK's alpha): same factors as an
    unscaled run, and the backward hooks never synchronise the host."""
    torch.manual_seed(0)
    net = _net().to(cuda)
    ref = copy.deepcopy(net)
    scaler = torch.amp.GradScaler('cuda', init_scale=2.0 ** 12)
    kw = dict(factor_update_steps=1, inv_update_steps=1000, lr=0.1, kl_clip=None)
    p_ref = kfac.KFACPreconditioner(ref, **kw)
    p_amp = kfac.KFACPreconditioner(net, grad_scaler=scaler, **kw)
    x = torch.randn(8, 3, 14, 14, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    for step in range(3):
        ref.zero_grad()
        torch.nn.functional.cross_entropy(ref(x), y).backward()
        net.zero_grad()
        loss = torch.nn.functional.cross_entropy(net(x), y)
        scaled = scaler.scale(loss)
        torch.cuda.synchronize()
        if step > 0:  # the scaler's tensor exists after the first scale()
            torch.cuda.set_sync_debug_mode('error')
        try:
            scaled.backward()
        finally:
            torch.cuda.set_sync_debug_mode('default')
        p_ref._join_factor_streams()
        p_amp._join_factor_streams()
        for (_, a), (_, b) in zip(p_ref._layers.values(), p_amp._layers.values()):
            torch.testing.assert_close(b.g_factor, a.g_factor, rtol=1e-5, atol=1e-7)
        p_ref.step()
        p_amp.step()


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
def test_early_precondition_overlap_is_exact(cuda, monkeypatch, method):
    """Preconditioning the last layers during backward on a side stream
    (KFAC_PRECOND_OVERLAP) yields bitwise the same training trajectory as
    preconditioning every layer in step()."""
    monkeypatch.setattr(torch.backends.cudnn, 'deterministic', True)  # MIOpen wrw
    runs = {}
    for flag in ('1', '0'):
        monkeypatch.setenv('KFAC_PRECOND_OVERLAP', flag)
        model = _net().to(cuda)
        pre = kfac.KFACPreconditioner(model, factor_update_steps=1, inv_update_steps=3,
                                      compute_method=method, lr=0.1, kl_clip=0.001)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        torch.manual_seed(3)
        for _ in range(7):
            x = torch.randn(8, 3, 14, 14, device=cuda)
            y = torch.randint(0, 10, (8,), device=cuda)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(model(x), y).backward()
            pre.step()
            opt.step()
        torch.cuda.synchronize()
        if flag == '1':
            assert pre._early is not None and pre._early['names'], 'no early group'
        runs[flag] = [p.detach().clone() for p in model.parameters()]
    for a, b in zip(runs['1'], runs['0']):
        assert torch.equal(a, b)
