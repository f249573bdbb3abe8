"""Graph-safe / GEMM 1x1 convolution modules (ops/conv.py) against
``F.conv2d``: identical forward values and gradients (CPU, float64)."""
from __future__ import annotations

import copy

import pytest
import torch
from torch import nn

from distributed_kfac_pytorch_amd.models.resnet import resnet50
from distributed_kfac_pytorch_amd.ops.conv import GemmConv1x1
from distributed_kfac_pytorch_amd.ops.conv import StridedConv1x1
from distributed_kfac_pytorch_amd.ops.conv import make_graph_safe
from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1


@pytest.mark.parametrize('cls', [StridedConv1x1, GemmConv1x1])
@pytest.mark.parametrize('stride', [1, 2])
@pytest.mark.parametrize('bias', [False, True])
@pytest.mark.parametrize('channels_last', [False, True])
def test_conv1x1_matches_conv2d(cls, stride, bias, channels_last) -> None:
    torch.manual_seed(stride + 2 * bias)
    ref = nn.Conv2d(6, 5, 1, stride=stride, bias=bias).double()
    mod = copy.deepcopy(ref)
    mod.__class__ = cls
    x = torch.randn(3, 6, 9, 8, dtype=torch.float64)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = ref(xa), mod(xb)
    assert ya.shape == yb.shape
    torch.testing.assert_close(yb, ya, rtol=1e-12, atol=1e-12)
    g = torch.randn_like(ya)
    ga = torch.autograd.grad(ya, [xa] + list(ref.parameters()), g)
    gb = torch.autograd.grad(yb, [xb] + list(mod.parameters()), g)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(b, a, rtol=1e-12, atol=1e-12)


def test_resnet50_projections_are_graph_safe() -> None:
    m = resnet50()
    strided = [n for n, mm in m.named_modules() if isinstance(mm, StridedConv1x1)]
    assert strided == ['layer2.0.downsample.0', 'layer3.0.downsample.0',
                       'layer4.0.downsample.0']
    # same state dict keys as torchvision's layout
    assert 'layer2.0.downsample.0.weight' in m.state_dict()
    # graph-safe (default 'strided'): only the strided 1x1 conv is switched
    plain = nn.Sequential(nn.Conv2d(4, 8, 1, stride=2), nn.Conv2d(8, 8, 1), nn.Conv2d(8, 8, 3))
    assert make_graph_safe(plain, 'strided') == 1
    assert type(plain[0]) is StridedConv1x1 and type(plain[1]) is nn.Conv2d
    assert type(plain[2]) is nn.Conv2d
    # 'gemm': every 1x1 conv becomes a GEMM conv, other kernels stay
    plain = nn.Sequential(nn.Conv2d(4, 8, 1, stride=2), nn.Conv2d(8, 8, 1), nn.Conv2d(8, 8, 3))
    assert make_graph_safe(plain, 'gemm') == 2
    assert type(plain[0]) is GemmConv1x1 and type(plain[1]) is GemmConv1x1
    assert type(plain[2]) is nn.Conv2d
    with pytest.raises(ValueError):
        make_graph_safe(plain, 'nope')


def test_use_gemm_conv1x1_switches_every_1x1() -> None:
    m = resnet50()
    n1 = sum(1 for mm in m.modules() if isinstance(mm, nn.Conv2d) and mm.kernel_size == (1, 1))
    assert use_gemm_conv1x1(m) == n1
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    m = m.to(memory_format=torch.channels_last)
    assert torch.isfinite(m(x)).all()


@pytest.mark.parametrize('shape', [(4, 16, 56, 56, 32, True), (2, 8, 7, 7, 16, False),
                                   (8, 64, 28, 28, 128, True)])
def test_gemm_conv1x1_slab_weight_grad_matches_conv(shape) -> None:
    """``GemmConv1x1``'s weight gradient, reduced in ``_splitk`` slabs,
    equals the convolution's (float64)."""
    from distributed_kfac_pytorch_amd.ops.conv import _splitk

    n, c, h, w, co, bias = shape
    torch.manual_seed(0)
    a = nn.Conv2d(c, co, 1, bias=bias).double()
    b = nn.Conv2d(c, co, 1, bias=bias).double()
    b.load_state_dict(a.state_dict())
    b.__class__ = GemmConv1x1
    x = torch.randn(n, c, h, w, dtype=torch.float64).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    x2 = x.detach().clone().contiguous(memory_format=torch.channels_last).requires_grad_()
    ya, yb = a(x), b(x2)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(yb, ya, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(x2.grad, x.grad, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(b.weight.grad, a.weight.grad, rtol=1e-10, atol=1e-10)
    if bias:
        torch.testing.assert_close(b.bias.grad, a.bias.grad, rtol=1e-10, atol=1e-10)
    m = n * h * w
    s = _splitk(m)
    assert m % s == 0 and (s == 1 or m // s >= 2048)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(32, 64, 56, 56, 256), (32, 1024, 14, 14, 256)])
def test_gemm_conv1x1_bf16_weight_grad(cuda, shape) -> None:
    """Under bf16 autocast the slab partials of ``GemmConv1x1``'s weight
    gradient are fp32 (one rounding to bf16 at the end): the result matches
    the float64 weight gradient of the same bf16 operands to bf16 precision,
    and is at least as close as MIOpen's bf16 convolution."""
    n, c, h, w, co = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(c, co, 1, bias=False).to(cuda)
    gem = nn.Conv2d(c, co, 1, bias=False).to(cuda)
    gem.load_state_dict(conv.state_dict())
    gem.__class__ = GemmConv1x1
    x = torch.randn(n, c, h, w, device=cuda).contiguous(memory_format=torch.channels_last)
    g = torch.randn(n, co, h, w, device=cuda).contiguous(memory_format=torch.channels_last)
    grads = []
    for m in (gem, conv):
        m.weight.grad = None
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = m(x)
        y.backward(g.to(y.dtype))
        grads.append(m.weight.grad.double().view(co, c))
    xb = x.to(torch.bfloat16).double().permute(0, 2, 3, 1).reshape(-1, c)
    gb = g.to(torch.bfloat16).double().permute(0, 2, 3, 1).reshape(-1, co)
    ref = gb.t() @ xb
    err_gemm = float((grads[0] - ref).norm() / ref.norm())
    err_miopen = float((grads[1] - ref).norm() / ref.norm())
    assert err_gemm < 4e-3, (err_gemm, err_miopen)
    assert err_gemm <= 1.5 * err_miopen + 1e-4, (err_gemm, err_miopen)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,stride', [((32, 64, 56, 56, 256), 1), ((8, 256, 28, 28, 512), 2),
                                          ((32, 1024, 14, 14, 256), 1), ((4, 100, 9, 9, 36), 1)])
def test_gemm_conv1x1_fp32_native_matches_float64(cuda, shape, stride, monkeypatch) -> None:
    """fp32 ``GemmConv1x1`` computes its forward and input gradient on the
    native bf16x3 GEMM (``gemm3_mm``): output, input and weight gradients
    match the float64 convolution to fp32-class accuracy (~5e-6), and the
    native kernel really runs (a call counter on the binding)."""
    from distributed_kfac_pytorch_amd.ops import _native

    lib = _native.native()
    assert lib is not None, _native.load_error()
    calls = []
    real = lib.gemm3_mm

    class Spy:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(lib, name)

        def gemm3_mm(self, *a):  # type: ignore[no-untyped-def]
            calls.append(a[0].shape)
            return real(*a)

    monkeypatch.setattr(_native, 'native', lambda: Spy())
    monkeypatch.setenv('KFAC_CONV1X1_MATH', 'bf16x3')
    n, c, h, w, co = shape
    torch.manual_seed(0)
    gem = nn.Conv2d(c, co, 1, stride=stride, bias=False).to(cuda)
    gem.__class__ = GemmConv1x1
    x = torch.randn(n, c, h, w, device=cuda).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = gem(x)
    g = torch.randn_like(y)
    y.backward(g)
    assert calls, 'the native bf16x3 GEMM did not run'
    xd, wd = x.detach().double(), gem.weight.detach().double()
    xd.requires_grad_(True)
    wd.requires_grad_(True)
    yd = torch.nn.functional.conv2d(xd, wd, stride=stride)
    yd.backward(g.double())

    def rel(a: torch.Tensor, b: torch.Tensor) -> float:
        return float((a.double() - b).norm() / b.norm())

    assert rel(y, yd) < 2e-5, rel(y, yd)
    assert rel(x.grad, xd.grad) < 2e-5, rel(x.grad, xd.grad)
    assert rel(gem.weight.grad, wd.grad) < 2e-5, rel(gem.weight.grad, wd.grad)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,stride,k', [((8, 64, 56, 56, 64), 1, 3), ((8, 128, 56, 56, 128), 2, 3),
                                            ((32, 512, 7, 7, 512), 1, 3),
                                            ((2, 96, 11, 13, 40), 1, 3),
                                            ((4, 3, 64, 64, 64), 2, 7),
                                            ((4, 256, 14, 14, 256), 1, 3)])
def test_implicit_gemm_conv_matches_float64(cuda, shape, stride, k, monkeypatch) -> None:
    """fp32 ``ImplicitGemmConv2d`` (3x3 pad 1, and the 7x7 stride-2 stem
    with its 3 channels padded to 4): forward on the native implicit GEMM
    (split-K on small images), stride-1 input gradient as the native
    convolution of dy with the flipped kernel, strided input gradient as dy .
    W + col2im and every weight gradient native (KFAC_CONV_DETERMINISTIC,
    the default) -- output and both gradients match float64 to fp32-class
    accuracy, and the native kernel runs."""
    from distributed_kfac_pytorch_amd.ops import _native
    from distributed_kfac_pytorch_amd.ops.conv import ImplicitGemmConv2d

    lib = _native.native()
    assert lib is not None, _native.load_error()
    calls = []
    real = lib.gemm3_conv

    class Spy:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(lib, name)

        def gemm3_conv(self, *a):  # type: ignore[no-untyped-def]
            calls.append(tuple(a[0].shape))
            return real(*a)

    monkeypatch.setattr(_native, 'native', lambda: Spy())
    monkeypatch.setenv('KFAC_CONV_KXK_MATH', 'bf16x3')
    n, c, h, w, co = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(c, co, k, stride=stride, padding=k // 2, bias=True).to(cuda)
    conv = conv.to(memory_format=torch.channels_last)
    conv.__class__ = ImplicitGemmConv2d
    x = torch.randn(n, c, h, w, device=cuda).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = conv(x)
    g = torch.randn_like(y)
    y.backward(g)
    assert len(calls) == 1 + (stride == 1 and co % 32 == 0 and c % 4 == 0), calls
    xd = x.detach().double().requires_grad_(True)
    wd = conv.weight.detach().double().requires_grad_(True)
    bd = conv.bias.detach().double().requires_grad_(True)
    yd = torch.nn.functional.conv2d(xd, wd, bd, stride=stride, padding=k // 2)
    yd.backward(g.double())

    def rel(a: torch.Tensor, b: torch.Tensor) -> float:
        return float((a.double() - b).norm() / b.norm())

    assert rel(y, yd) < 2e-5, rel(y, yd)
    assert rel(x.grad, xd.grad) < 2e-5, rel(x.grad, xd.grad)
    assert rel(conv.weight.grad, wd.grad) < 2e-5, rel(conv.weight.grad, wd.grad)
    assert rel(conv.bias.grad, bd.grad) < 2e-5, rel(conv.bias.grad, bd.grad)


@pytest.mark.gpu
def test_implicit_gemm_conv_wgrad_falls_back_past_kernel_limit(cuda, monkeypatch) -> None:
    """An input with N*Ho*Wo >= 2^22 output pixels (here 16 x 512 x 512)
    is past the native weight gradient's index range: the backward takes
    MIOpen's weight gradient instead of failing the binding's check."""
    from distributed_kfac_pytorch_amd.ops import _native
    from distributed_kfac_pytorch_amd.ops.conv import ImplicitGemmConv2d

    lib = _native.native()
    assert lib is not None, _native.load_error()
    called = []

    class Spy:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(lib, name)

        def gemm3_conv_wgrad(self, *a):  # type: ignore[no-untyped-def]
            called.append(tuple(a[0].shape))
            return lib.gemm3_conv_wgrad(*a)

    monkeypatch.setattr(_native, 'native', lambda: Spy())
    monkeypatch.setenv('KFAC_CONV_KXK_MATH', 'bf16x3')
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 8, 3, padding=1, bias=False).to(cuda).to(memory_format=torch.channels_last)
    conv.__class__ = ImplicitGemmConv2d
    for n, native in ((15, True), (16, False)):  # 15*512*512 < 2^22 <= 16*512*512
        x = torch.randn(n, 3, 512, 512, device=cuda).contiguous(memory_format=torch.channels_last)
        called.clear()
        conv.weight.grad = None
        y = conv(x)
        g = torch.randn_like(y)
        y.backward(g)
        assert bool(called) == native, (n, called)
        wd = torch.nn.grad.conv2d_weight(x.double(), conv.weight.shape, g.double(), padding=1)
        err = float((conv.weight.grad.double() - wd).norm() / wd.norm())
        assert err < 2e-5, (n, err)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,stride,k,stem', [((32, 128, 56, 56, 128), 2, 3, False),
                                                 ((32, 512, 14, 14, 512), 2, 3, False),
                                                 ((3, 12, 9, 11, 40), 2, 3, False),
                                                 ((2, 8, 10, 10, 40), 3, 5, False),
                                                 ((16, 64, 56, 56, 64), 1, 3, False),
                                                 ((32, 3, 224, 224, 64), 2, 7, True)])
def test_deterministic_conv_backward(cuda, shape, stride, k, stem, monkeypatch) -> None:
    """``KFAC_CONV_DETERMINISTIC=1`` (the default): a strided input gradient
    is ``dy . W`` on gemm3 plus the native fixed-order col2im, a 64-channel
    weight gradient and the 3-channel stem's (``StemConv2d``: MIOpen
    forward) run on the native split-K kernel.  Gradients match float64 to
    fp32-class accuracy, the native kernels run, MIOpen's backward does not,
    and two backward passes are bit-identical."""
    from distributed_kfac_pytorch_amd.ops import _native
    from distributed_kfac_pytorch_amd.ops import conv as cops

    lib = _native.native()
    assert lib is not None, _native.load_error()
    calls: list = []

    class Spy:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(lib, name)

        def col2im_nhwc(self, *a):  # type: ignore[no-untyped-def]
            calls.append('col2im')
            return lib.col2im_nhwc(*a)

        def gemm3_conv_wgrad(self, *a):  # type: ignore[no-untyped-def]
            calls.append('wgrad')
            return lib.gemm3_conv_wgrad(*a)

    real_cb = torch.ops.aten.convolution_backward

    class Aten:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(torch.ops.aten, name)

        def convolution_backward(self, *a):  # type: ignore[no-untyped-def]
            calls.append('miopen')
            return real_cb(*a)

    monkeypatch.setattr(_native, 'native', lambda: Spy())
    monkeypatch.setattr(cops.torch.ops, 'aten', Aten(), raising=False)
    monkeypatch.setenv('KFAC_CONV_KXK_MATH', 'bf16x3')
    monkeypatch.setenv('KFAC_CONV_DETERMINISTIC', '1')
    n, c, h, w, co = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(c, co, k, stride=stride, padding=k // 2, bias=False).to(cuda)
    conv = conv.to(memory_format=torch.channels_last)
    assert cops.use_implicit_gemm_conv(conv) == 1
    assert type(conv) is (cops.StemConv2d if stem else cops.ImplicitGemmConv2d)
    x = torch.randn(n, c, h, w, device=cuda).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(not stem)
    y = conv(x)
    g = torch.randn_like(y)
    grads = []
    for _ in range(2):
        calls.clear()
        conv.weight.grad = None
        x.grad = None
        y = conv(x)
        y.backward(g)
        grads.append((None if stem else x.grad.clone(), conv.weight.grad.clone()))
        assert 'miopen' not in calls, calls
        assert 'wgrad' in calls, calls
        assert ('col2im' in calls) == (stride > 1 and not stem), calls
    assert stem or torch.equal(grads[0][0], grads[1][0])
    assert torch.equal(grads[0][1], grads[1][1])
    xd = x.detach().double().requires_grad_(not stem)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = torch.nn.functional.conv2d(xd, wd, None, stride=stride, padding=k // 2)
    yd.backward(g.double())

    def rel(a: torch.Tensor, b: torch.Tensor) -> float:
        return float((a.double() - b).norm() / b.norm())

    assert rel(y, yd) < 2e-5, rel(y, yd)
    assert rel(conv.weight.grad, wd.grad) < 2e-5, rel(conv.weight.grad, wd.grad)
    if not stem:
        assert rel(x.grad, xd.grad) < 2e-5, rel(x.grad, xd.grad)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,stride,k,stem', [((32, 64, 56, 56, 64), 1, 3, False),
                                                 ((32, 128, 56, 56, 128), 2, 3, False),
                                                 ((32, 512, 7, 7, 512), 1, 3, False),
                                                 ((3, 16, 9, 11, 40), 2, 3, False),
                                                 ((8, 3, 224, 224, 64), 2, 7, True)])
def test_deterministic_conv_backward_bf16(cuda, shape, stride, k, stem, monkeypatch) -> None:
    """``KFAC_CONV_DETERMINISTIC_BF16=1`` (opt-in): under bf16 autocast the
    3x3 convolutions and the stem run as bf16 GEMMs -- forward ``im2col(x) .
    W^T``, input gradient ``dy . W`` + the native bf16 col2im, weight gradient
    ``dy^T . patches`` -- with no MIOpen backward call.  Two passes are
    bit-identical and output and gradients match float64 of the same bf16
    operands to bf16 accuracy."""
    from distributed_kfac_pytorch_amd.ops import _native
    from distributed_kfac_pytorch_amd.ops import conv as cops

    lib = _native.native()
    assert lib is not None, _native.load_error()
    calls: list = []

    class Spy:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(lib, name)

        def col2im_nhwc(self, *a):  # type: ignore[no-untyped-def]
            calls.append('col2im')
            return lib.col2im_nhwc(*a)

    real_cb = torch.ops.aten.convolution_backward

    class Aten:
        def __getattr__(self, name):  # type: ignore[no-untyped-def]
            return getattr(torch.ops.aten, name)

        def convolution_backward(self, *a):  # type: ignore[no-untyped-def]
            calls.append('miopen')
            return real_cb(*a)

    monkeypatch.setattr(_native, 'native', lambda: Spy())
    monkeypatch.setattr(cops.torch.ops, 'aten', Aten(), raising=False)
    monkeypatch.setenv('KFAC_CONV_DETERMINISTIC_BF16', '1')
    n, c, h, w, co = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(c, co, k, stride=stride, padding=k // 2, bias=False).to(cuda)
    conv = conv.to(memory_format=torch.channels_last)
    assert cops.use_implicit_gemm_conv(conv) == 1
    x = torch.randn(n, c, h, w, device=cuda).contiguous(memory_format=torch.channels_last)
    x = x.to(torch.bfloat16).requires_grad_(not stem)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = conv(x)
    assert y.dtype == torch.bfloat16
    g = torch.randn_like(y)
    grads = []
    for _ in range(2):
        calls.clear()
        conv.weight.grad = None
        x.grad = None
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = conv(x)
        y.backward(g)
        grads.append((None if stem else x.grad.clone(), conv.weight.grad.clone(), y.detach()))
        assert 'miopen' not in calls, calls
        assert ('col2im' in calls) == (not stem), calls
    assert stem or torch.equal(grads[0][0], grads[1][0])
    assert torch.equal(grads[0][1], grads[1][1]) and torch.equal(grads[0][2], grads[1][2])
    xd = x.detach().double().requires_grad_(not stem)
    wd = conv.weight.detach().to(torch.bfloat16).double().requires_grad_(True)
    yd = torch.nn.functional.conv2d(xd, wd, None, stride=stride, padding=k // 2)
    yd.backward(g.double())

    def rel(a: torch.Tensor, b: torch.Tensor) -> float:
        return float((a.detach().double() - b).norm() / b.norm())

    assert rel(y, yd) < 1e-2, rel(y, yd)
    assert rel(conv.weight.grad, wd.grad) < 1e-2, rel(conv.weight.grad, wd.grad)
    if not stem:
        assert rel(x.grad, xd.grad) < 1e-2, rel(x.grad, xd.grad)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(32, 3, 224, 224), (2, 5, 7, 9), (64, 3, 7, 7), (1, 1, 3, 3)])
def test_pad_channels4_native_exact(cuda, shape) -> None:
    """``pad_channels4`` (csrc/subsample.hip): the channels_last input
    zero-padded to a multiple of 4 channels in one pass, equal to torch's
    cat with zeros, channels_last."""
    from distributed_kfac_pytorch_amd.ops import _native
    from distributed_kfac_pytorch_amd.ops.conv import _pad4

    lib = _native.native()
    assert lib is not None, _native.load_error()
    x = torch.randn(*shape, device=cuda).contiguous(memory_format=torch.channels_last)
    c = shape[1]
    ref = torch.cat([x, x.new_zeros(shape[0], (4 - c % 4) % 4, *shape[2:])], 1)
    got = lib.pad_channels4(x)
    assert torch.equal(got, ref)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(_pad4(x), ref)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,s', [((32, 256, 56, 56), 2), ((3, 12, 7, 9), 2), ((2, 8, 10, 10), 3)])
def test_subsample_native_exact(cuda, shape, s) -> None:
    """The strided 1x1 convolutions' subsample and its adjoint on the native
    kernels (csrc/subsample.hip) equal the slicing reference bit for bit."""
    from distributed_kfac_pytorch_amd.ops import _native
    from distributed_kfac_pytorch_amd.ops.conv import _subsample

    assert _native.native() is not None, _native.load_error()
    x = torch.randn(*shape, device=cuda).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = _subsample(x, s, s)
    ref = x.detach()[:, :, ::s, ::s]
    assert torch.equal(y, ref) and y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(y)
    y.backward(g)
    gx = torch.zeros_like(x)
    gx[:, :, ::s, ::s] = g
    assert torch.equal(x.grad, gx)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(7, 256, 64), (256, 64, 256), (3, 5, 7), (1, 8, 4),
                                   (64, 64, 576), (37, 16, 36), (128, 4, 8)])
def test_sum_splits_matches_torch(cuda, shape) -> None:
    """The split-K partial sum kernel (csrc/subsample.hip ``sum_splits``,
    fixed order; lane-grouped when few outputs meet many splits) equals
    ``part.sum(0)`` to fp32 rounding and repeats bit for bit, with the torch
    fallback for element counts that are not a multiple of 4."""
    from distributed_kfac_pytorch_amd.ops import _native

    lib = _native.native()
    assert lib is not None, _native.load_error()
    part = torch.randn(*shape, device=cuda)
    got = lib.sum_splits(part)
    ref = part.double().sum(0)
    assert got.shape == ref.shape
    assert float((got.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)) < 1e-5
    out = torch.empty(shape[1:], device=cuda)
    assert lib.sum_splits(part, out).data_ptr() == out.data_ptr()
    assert torch.equal(out, got)  # fixed summation order
