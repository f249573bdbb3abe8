"""Is a captured ResNet-50 forward + backward replayed correctly (no K-FAC,
no optimizer)?  Compares the parameter gradients of each replay with an
eager forward + backward of the same input, replay by replay.

    python tools/graph_sgd_probe.py [--nchw] [--nodet] [--no-cudnn]
                                    [--side-warmup N] [--replays 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--nchw', action='store_true')
    ap.add_argument('--nodet', action='store_true')
    ap.add_argument('--no-cudnn', action='store_true')
    ap.add_argument('--side-warmup', type=int, default=0)
    ap.add_argument('--replays', type=int, default=4)
    ap.add_argument('--batch', type=int, default=8)
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = not args.nodet
    torch.backends.cudnn.enabled = not args.no_cudnn
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = resnet50(num_classes=10).to(dev)
    fmt = torch.contiguous_format if args.nchw else torch.channels_last
    model = model.to(memory_format=fmt)
    x = torch.randn(args.batch, 3, 64, 64, device=dev).contiguous(memory_format=fmt)
    y = torch.randint(0, 10, (args.batch,), device=dev)
    params = list(model.parameters())
    names = [n for n, _ in model.named_parameters()]

    def fb() -> torch.Tensor:
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        return loss.detach()

    for _ in range(2):  # eager warmup + reference
        model.zero_grad(set_to_none=False)
        fb()
    ref = [p.grad.clone() for p in params]
    model.zero_grad(set_to_none=False)
    fb()
    eager_rep = max(float((p.grad - r).abs().max() / r.abs().max().clamp_min(1e-30))
                    for p, r in zip(params, ref))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(args.side_warmup):
            model.zero_grad(set_to_none=False)
            fb()
    torch.cuda.current_stream().wait_stream(side)
    model.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    side2 = torch.cuda.Stream()
    side2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side2):
        with torch.cuda.graph(g, stream=side2):
            fb()
    torch.cuda.current_stream().wait_stream(side2)
    grads = [p.grad for p in params]
    out = {'args': vars(args), 'eager_repeat_maxrel': eager_rep, 'replays': []}
    for r in range(args.replays):
        g.replay()
        torch.cuda.synchronize()
        diffs = [float((gg - rr).abs().max() / rr.abs().max().clamp_min(1e-30))
                 for gg, rr in zip(grads, ref)]
        worst = sorted(zip(diffs, names), reverse=True)[:4]
        out['replays'].append({'replay': r, 'maxrel': max(diffs),
                               'n_bad': sum(d > 1e-4 for d in diffs),
                               'worst': [(round(d, 6), n) for d, n in worst]})
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
