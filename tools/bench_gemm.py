"""Time the ResNet-50 precondition GEMM shapes under torch.mm (fp32) at the
three float32 matmul precisions, with accuracy vs fp64.  One JSON line per
(shape, precision)."""
from __future__ import annotations

import json

import torch

# (g, a) factor dims of the distinct ResNet-50 layers and their counts
LAYERS = [(64, 147, 1), (64, 64, 3), (64, 576, 3), (256, 64, 4), (64, 256, 2),
          (128, 256, 1), (128, 1152, 4), (512, 128, 4), (512, 256, 1), (128, 512, 3),
          (256, 512, 1), (256, 2304, 6), (1024, 256, 6), (1024, 512, 1), (256, 1024, 5),
          (512, 1024, 1), (512, 4608, 3), (2048, 512, 3), (2048, 1024, 1), (512, 2048, 2),
          (1000, 2049, 1)]


def timeit(fn, iters: int = 20) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main() -> None:
    dev = torch.device('cuda')
    total = {}
    for prec in ('highest', 'high', 'medium'):
        torch.set_float32_matmul_precision(prec)
        tot_ms = 0.0
        for g, a, cnt in LAYERS:
            grad = torch.randn(g, a, device=dev)
            qa = torch.linalg.qr(torch.randn(a, a, device=dev))[0]
            qg = torch.linalg.qr(torch.randn(g, g, device=dev))[0]
            t1 = torch.empty(g, a, device=dev)
            t2 = torch.empty(g, a, device=dev)

            def chain() -> None:
                torch.mm(grad, qa, out=t1)
                torch.mm(qg.t(), t1, out=t2)
                torch.mm(qg, t2, out=t1)
                torch.mm(t1, qa.t(), out=t2)

            ms = timeit(chain)
            ref = (qg.double() @ (qg.double().t() @ (grad.double() @ qa.double())) @ qa.double().t())
            chain()
            err = ((t2.double() - ref).abs().max() / ref.abs().max()).item()
            flops = 2 * (2 * g * g * a + 2 * g * a * a)
            tot_ms += ms * cnt
            print(json.dumps({'prec': prec, 'g': g, 'a': a, 'count': cnt, 'ms': round(ms, 4),
                              'tflops': round(flops / ms / 1e9, 1), 'rel_err': err}), flush=True)
        total[prec] = round(tot_ms, 3)
    print(json.dumps({'total_chain_ms_per_step': total}), flush=True)


if __name__ == '__main__':
    main()
