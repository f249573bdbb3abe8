"""Probe: ResNet-50 BatchNorm(+ReLU) cost on MI355X by backend.

For each distinct ResNet-50 BN shape at batch 32 (bf16, channels_last),
times forward + backward of BN followed by ReLU with (a) MIOpen BN (torch's
default on ROCm) and (b) PyTorch's native channels-last BN kernels (cudnn
flag off around the BN call).  Then times a whole SGD step of ResNet-50
with each backend.  JSON lines on stdout.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops import bnact  # noqa: E402

SHAPES = [(64, 112), (64, 56), (256, 56), (128, 56), (128, 28), (512, 28), (256, 28),
          (256, 14), (1024, 14), (512, 14), (512, 7), (2048, 7)]


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def bn_relu(x, w, b, rm, rv, native):
    with torch.backends.cudnn.flags(enabled=not native):
        y = F.batch_norm(x, rm, rv, w, b, training=True, momentum=0.1, eps=1e-5)
    return F.relu(y)


def main() -> None:
    dev = torch.device('cuda')
    for c, hw in SHAPES:
        x = torch.randn(32, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        w = torch.ones(c, device=dev, requires_grad=True)
        b = torch.zeros(c, device=dev, requires_grad=True)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        g = torch.randn_like(x)
        row = {'C': c, 'HW': hw, 'MB': round(x.numel() * 2 / 1e6, 1)}
        for native in (False, True):
            def step():
                y = bn_relu(x, w, b, rm, rv, native)
                y.backward(g)
            row['native_us' if native else 'miopen_us'] = round(timed(step), 1)
        bn = bnact.BatchNormAct2d(c).to(dev)

        def fused():
            bn.act(x).backward(g)
        row['fused_us'] = round(timed(fused), 1)
        print(json.dumps(row), flush=True)
    # whole SGD step
    for fused in ('1', '0'):
        os.environ['KFAC_FUSED_BN'] = fused
        model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, foreach=True)
        xb = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
        yb = torch.randint(0, 1000, (32,), device=dev)

        def sgd2():
            opt.zero_grad(set_to_none=True)
            with torch.autocast('cuda', dtype=torch.bfloat16):
                loss = F.cross_entropy(model(xb), yb)
            loss.backward()
            opt.step()
        ms = timed(sgd2, reps=30) / 1e3
        print(json.dumps({'sgd_step_ms': round(ms, 3), 'bn': 'fused' if fused == '1' else 'miopen(model)'}),
              flush=True)
    os.environ['KFAC_FUSED_BN'] = '0'
    orig = torch.nn.BatchNorm2d.forward
    for native in (False, True):
        if native:
            def fwd(self, inp, _orig=orig):
                with torch.backends.cudnn.flags(enabled=False):
                    return _orig(self, inp)
            torch.nn.BatchNorm2d.forward = fwd
        model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, foreach=True)
        xb = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
        yb = torch.randint(0, 1000, (32,), device=dev)

        def sgd():
            opt.zero_grad(set_to_none=True)
            with torch.autocast('cuda', dtype=torch.bfloat16):
                loss = F.cross_entropy(model(xb), yb)
            loss.backward()
            opt.step()
        ms = timed(sgd, reps=30) / 1e3
        print(json.dumps({'sgd_step_ms': round(ms, 3), 'bn': 'native' if native else 'miopen'}),
              flush=True)
        torch.nn.BatchNorm2d.forward = orig


if __name__ == '__main__':
    main()
