"""One-off MI355X probe: sizes the K-FAC design against the real hardware.

Times (1) ResNet-50 fwd+bwd at batch 32 bf16, (2) torch.linalg.eigh / inv /
cholesky at the ResNet-50 factor sizes, (3) fp32 / bf16 GEMMs of the
precondition and factor shapes.  Output: one JSON per line on stdout.
"""
from __future__ import annotations

import json
import sys
import time

import torch

sys.path.insert(0, '.')
from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402


def timeit(fn, iters=10, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    dev = torch.device('cuda:0')
    emit(device=torch.cuda.get_device_name(0),
         props=str(torch.cuda.get_device_properties(0)))
    try:
        emit(linalg_lib=str(torch.backends.cuda.preferred_linalg_library()))
    except Exception as e:  # noqa: BLE001
        emit(linalg_lib_err=str(e))

    # (1) ResNet-50
    for cl in (True, False):
        model = resnet50().to(dev)
        if cl:
            model = model.to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
        x = torch.randn(32, 3, 224, 224, device=dev)
        if cl:
            x = x.to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (32,), device=dev)

        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast('cuda', dtype=torch.bfloat16):
                loss = torch.nn.functional.cross_entropy(model(x), y)
            loss.backward()
            opt.step()

        ms = timeit(step, iters=20, warmup=5)
        emit(what='resnet50_b32_bf16', channels_last=cl, ms=ms,
             img_s=32 / ms * 1e3)
        del model, opt

    # (2) linalg
    for n in (64, 147, 256, 512, 576, 1024, 1152, 2048, 2304, 4608):
        a = torch.randn(n, n, device=dev)
        a = a @ a.t() / n + torch.eye(n, device=dev)
        it = 3 if n >= 2048 else 5
        ms_e = timeit(lambda: torch.linalg.eigh(a), iters=it, warmup=1)
        ms_i = timeit(lambda: torch.linalg.inv(a), iters=it, warmup=1)
        ms_c = timeit(lambda: torch.linalg.cholesky(a), iters=it, warmup=1)
        emit(what='linalg', n=n, eigh_ms=ms_e, inv_ms=ms_i, chol_ms=ms_c)

    # (3) GEMMs
    for (m, k, n) in ((512, 4608, 4608), (2048, 2048, 4608), (4608, 4608, 4608),
                      (256, 2304, 2304), (64, 576, 576)):
        a = torch.randn(m, k, device=dev)
        b = torch.randn(k, n, device=dev)
        ms = timeit(lambda: a @ b, iters=10)
        emit(what='gemm_fp32', m=m, k=k, n=n, ms=ms,
             tflops=2 * m * n * k / ms / 1e9)
    for (rows, d) in ((100352, 576), (25088, 1152), (6272, 2304), (1568, 4608),
                      (401408, 147), (100352, 64), (100352, 256)):
        x = torch.randn(rows, d, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: x.t() @ x, iters=10)
        xf = x.float()
        ms32 = timeit(lambda: xf.t() @ xf, iters=10)
        emit(what='syrk_as_gemm', rows=rows, d=d, bf16_ms=ms, fp32_ms=ms32,
             bf16_tflops=2 * rows * d * d / ms / 1e9,
             fp32_tflops=2 * rows * d * d / ms32 / 1e9)


if __name__ == '__main__':
    main()
