"""Would an eigen refresh overlapped with training steps pay off?

Snapshots real step-100 ResNet-50 factors (tools/refresh_probe.py), then
times, on one GPU:
  (a) N graph-replayed ResNet-50 SGD training steps alone,
  (b) the refresh (ops.linalg.eigh_many, warm-tested) alone,
  (c) both at once: the refresh issued from a background thread on its own
      streams while the main thread replays the N steps.
Prints JSON: the steps' time with and without the concurrent refresh and the
wall time until both finish."""
from __future__ import annotations

import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from refresh_probe import snapshot  # noqa: E402

from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402


def main() -> None:
    n_steps = int(os.environ.get('N_STEPS', '40'))
    mats, warm = snapshot(100)
    dev = torch.device('cuda')
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss()
    x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device=dev)
    main_s = torch.cuda.Stream()
    with torch.cuda.stream(main_s):
        for _ in range(3):
            opt.zero_grad(set_to_none=False)
            with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
                crit(model(x), y).backward()
            opt.step()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s):
            opt.zero_grad(set_to_none=False)
            with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
                crit(model(x), y).backward()
            opt.step()
    torch.cuda.synchronize()

    def steps() -> float:
        with torch.cuda.stream(main_s):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n_steps):
                g.replay()
            e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1)

    side = torch.cuda.Stream()

    def refresh() -> None:
        with torch.cuda.stream(side):
            linalg.eigh_many([m.clone() for m in mats], list(warm))

    for rep in range(3):
        steps()
        t_steps = steps()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        refresh()
        torch.cuda.synchronize()
        t_ref = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = threading.Thread(target=refresh)
        th.start()
        t_steps_conc = steps()
        th.join()
        torch.cuda.synchronize()
        t_both = (time.perf_counter() - t0) * 1e3
        print(json.dumps({'rep': rep, 'n_steps': n_steps, 'steps_ms': round(t_steps, 1),
                          'refresh_ms': round(t_ref, 1),
                          'sequential_ms': round(t_steps + t_ref, 1),
                          'steps_ms_concurrent': round(t_steps_conc, 1),
                          'both_done_ms': round(t_both, 1)}), flush=True)


if __name__ == '__main__':
    main()
