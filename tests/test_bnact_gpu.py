"""Fused BatchNorm (+ residual) (+ ReLU) kernels (csrc/bnact.hip) vs the
PyTorch fp32 math on the same bf16 / fp32 inputs."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.ops import bnact

pytestmark = pytest.mark.gpu


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous(memory_format=torch.channels_last)


# small activations take the two-launch sliced path (csrc/bnact.hip
# sliced_plan), large ones the three-launch path: both are covered
@pytest.mark.parametrize('shape', [(4, 64, 14, 14), (2, 256, 7, 9), (3, 2048, 4, 4),
                                   (2, 16, 5, 5), (2, 24, 3, 3), (8, 128, 28, 28),
                                   (32, 512, 7, 7), (32, 1024, 14, 14), (8, 64, 56, 56),
                                   (16, 32, 32, 32)])
@pytest.mark.parametrize('relu', [True, False])
@pytest.mark.parametrize('residual', [True, False])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_bn_act_matches_reference(cuda, shape, relu, residual, dtype):
    torch.manual_seed(sum(shape))
    n, c, h, w = shape
    x = _cl((torch.randn(shape, device=cuda) * 2 + 0.5).to(dtype))
    res = _cl(torch.randn(shape, device=cuda).to(dtype)) if residual else None
    dy = _cl(torch.randn(shape, device=cuda).to(dtype))
    bn = bnact.BatchNormAct2d(c).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref_bn = torch.nn.BatchNorm2d(c).to(cuda)
    ref_bn.load_state_dict(bn.state_dict())
    assert bnact._fusable(bn, x, res)

    xa = x.clone().requires_grad_(True)
    ra = res.clone().requires_grad_(True) if residual else None
    y = bn.act(xa, residual=ra, relu=relu)
    y.backward(dy)

    xr = x.float().requires_grad_(True)
    rr = res.float().requires_grad_(True) if residual else None
    yr = ref_bn(xr)
    if residual:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    yr.backward(dy.float())

    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    fp32 = dtype == torch.float32
    tol, atol = (1e-5, 1e-5) if fp32 else (2e-2, 1e-2)
    assert (y.float() - yr).abs().max().item() <= tol * yr.abs().max().item() + atol
    gx = xr.grad.abs().max().item()
    assert (xa.grad.float() - xr.grad).abs().max().item() <= (1e-4 if fp32 else tol) * gx + 1e-5
    gtol = 1e-4 if fp32 else 1e-2
    assert torch.allclose(bn.weight.grad, ref_bn.weight.grad, rtol=gtol, atol=gtol)
    assert torch.allclose(bn.bias.grad, ref_bn.bias.grad, rtol=gtol, atol=gtol)
    if residual:
        assert (ra.grad.float() - rr.grad).abs().max().item() <= gtol * rr.grad.abs().max().item() + 1e-5
    assert torch.allclose(bn.running_mean, ref_bn.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn.running_var, ref_bn.running_var, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1


def test_resnet50_fused_vs_unfused(cuda, monkeypatch):
    """Whole ResNet-50 fwd+bwd: the fused-BN bf16 run must be at least about
    as close to an fp32 run of the same weights as the PyTorch / MIOpen bf16
    run is (the fused path rounds bn(x) + residual once, in fp32, instead of
    rounding the BN output and the sum separately)."""
    from distributed_kfac_pytorch_amd.models.resnet import resnet50

    torch.manual_seed(0)
    base = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    x = _cl(torch.randn(4, 3, 64, 64, device=cuda))
    y = torch.randint(0, 10, (4,), device=cuda)
    runs = {}
    for name, fused, amp in (('fp32', '0', False), ('fused', '1', True), ('miopen', '0', True)):
        model = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
        model.load_state_dict(base.state_dict())
        monkeypatch.setenv('KFAC_FUSED_BN', fused)
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        runs[name] = (loss.item(), model.fc.weight.grad.clone(), model)
    lr, fr, _ = runs['fp32']
    dl_f = abs(runs['fused'][0] - lr)
    dl_m = abs(runs['miopen'][0] - lr)
    assert dl_f <= 1.5 * dl_m + 2e-2 * abs(lr), (dl_f, dl_m)
    df = (runs['fused'][1] - fr).abs().max().item()
    dm = (runs['miopen'][1] - fr).abs().max().item()
    assert df <= 1.5 * dm + 1e-2 * fr.abs().max().item(), (df, dm)
    nb = [b for n, b in runs['fused'][2].named_buffers() if n.endswith('num_batches_tracked')]
    assert nb and all(int(b) == 1 for b in nb)


def test_cpp_node_matches_python_function(cuda):
    """The C++ autograd node (native().bn_act) and the Python Function
    wrapper run the same kernels: identical outputs and gradients."""
    from distributed_kfac_pytorch_amd.ops._native import native

    torch.manual_seed(1)
    shape = (4, 128, 9, 9)
    x = _cl(torch.randn(shape, device=cuda).to(torch.bfloat16))
    res = _cl(torch.randn(shape, device=cuda).to(torch.bfloat16))
    dy = _cl(torch.randn(shape, device=cuda).to(torch.bfloat16))
    outs = []
    for use_cpp in (True, False):
        bn = bnact.BatchNormAct2d(128).to(cuda)
        xa, ra = x.clone().requires_grad_(True), res.clone().requires_grad_(True)
        args = (bn.running_mean, bn.running_var, bn.num_batches_tracked)
        if use_cpp:
            y = native().bn_act(xa, bn.weight, bn.bias, ra, *args, 0.1, 1e-5, True)
        else:
            y = bnact._BNActFunction.apply(xa, bn.weight, bn.bias, *args, ra, True, 0.1, 1e-5)
        y.backward(dy)
        outs.append((y, xa.grad, ra.grad, bn.weight.grad, bn.bias.grad, bn.running_var))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize('kind', ['1x1', '3x3', '3x3s2'])
@pytest.mark.parametrize('shape', [(4, 64, 14, 14), (8, 128, 28, 28), (2, 256, 7, 9),
                                   (16, 64, 56, 56)])
@pytest.mark.parametrize('cout', [96, 64])
def test_conv_epilogue_bn_statistics(cuda, monkeypatch, kind, shape, cout):
    """A native fp32 convolution marked ``_feeds_bn`` writes the following
    BN's statistics partials from its GEMM epilogue (csrc/gemm3.hip
    bnpart); the fused BN then skips its statistics pass.  Output, running
    statistics and every gradient match the BN's own statistics pass
    (``KFAC_BN_CONV_STATS=0``) to fp32 summation-order noise, and the
    partials were actually taken."""
    from distributed_kfac_pytorch_amd.ops import conv as cops

    n, c, h, w = shape
    torch.manual_seed(7)
    if kind == '1x1':
        base = torch.nn.Conv2d(c, cout, 1, bias=False)
    else:
        base = torch.nn.Conv2d(c, cout, 3, stride=2 if kind == '3x3s2' else 1, padding=1,
                               bias=False)
    x = _cl(torch.randn(shape, device=cuda))
    runs = {}
    gys: list = []
    for stats in ('1', '0'):
        monkeypatch.setenv('KFAC_BN_CONV_STATS', stats)
        conv = _cl_module(base, cuda)
        if kind == '1x1':
            cops.use_gemm_conv1x1(conv)
        else:
            cops.use_implicit_gemm_conv(conv)
        conv[0]._feeds_bn = True
        bn = bnact.BatchNormAct2d(cout).to(cuda)
        taken = []
        orig = cops.take_bn_part

        def spy(t):  # type: ignore[no-untyped-def]
            p = orig(t)
            taken.append(p is not None)
            return p
        monkeypatch.setattr(bnact, 'take_bn_part', spy)
        xa = x.clone().requires_grad_(True)
        y = bn.act(conv(xa))
        if not gys:
            gys.append(_cl(torch.randn_like(y)))
        y.backward(gys[0])
        runs[stats] = (y.detach(), xa.grad, conv[0].weight.grad, bn.weight.grad, bn.bias.grad,
                       bn.running_mean, bn.running_var, taken)
    # a split-K convolution (small images) sums partial outputs afterwards:
    # no epilogue statistics there, the BN takes its own pass
    from distributed_kfac_pytorch_amd.ops._native import native

    single = kind == '1x1' or int(native().gemm3_conv_splits(
        n, h, w, c, cout, 3, 3, 2 if kind == '3x3s2' else 1, 1)) == 1
    assert runs['1'][-1] == [single] and runs['0'][-1] == [False]
    names = ('y', 'dx', 'dw', 'dgamma', 'dbeta', 'running_mean', 'running_var')
    for name, a, b in zip(names, runs['1'][:-1], runs['0'][:-1]):
        scale = b.abs().max().item() + 1e-12
        assert (a - b).abs().max().item() <= 1e-4 * scale, (name, (a - b).abs().max().item(), scale)


def _cl_module(base: torch.nn.Conv2d, cuda: torch.device) -> torch.nn.Sequential:
    import copy

    return torch.nn.Sequential(copy.deepcopy(base)).to(cuda).to(
        memory_format=torch.channels_last)
