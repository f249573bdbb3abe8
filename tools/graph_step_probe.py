"""Probe: how launch-bound is the ResNet-50 b32 training step?  Times the
plain SGD step eagerly and as one captured HIP graph (forward + backward +
foreach SGD), same model / data / dtype as bench.py.  One JSON line."""
from __future__ import annotations

import json
import os
import sys
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('MIOPEN_USER_DB_PATH', os.path.join(_ROOT, 'miopen_db'))
import torch  # noqa: E402

sys.path.insert(0, _ROOT)
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402


def main() -> None:
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9,
                          weight_decay=5e-5, foreach=True)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device=dev)

    def step() -> None:
        opt.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
            loss = crit(model(x), y)
        loss.backward()
        opt.step()

    def timed(fn, n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(5):
            step()
    torch.cuda.current_stream().wait_stream(side)
    row = {'eager_ms': round(timed(step, 50), 3)}
    g = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=True)
    try:
        with torch.cuda.graph(g):
            with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
                loss = crit(model(x), y)
            loss.backward()
            opt.step()
        row['graph_ms'] = round(timed(g.replay, 50), 3)
        row['eager_again_ms'] = round(timed(g.replay, 1) * 0 + timed(step, 50), 3)
    except Exception as e:  # noqa: BLE001
        row['capture_error'] = str(e)[:400]
    print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
