"""Which MIOpen op replays wrongly from a HIP graph in channels_last?

Each case captures ONE op (forward + backward of a small module on fixed
inputs) and replays it several times, comparing outputs and gradients with
an eager run of the same inputs.  tools/graph_sgd_probe.py showed the full
ResNet-50 forward + backward replaying wrongly from the second replay on in
channels_last with MIOpen, and correctly in NCHW or without MIOpen.

    python tools/miopen_graph_probe.py
"""
from __future__ import annotations

import json

import torch


def case(name: str, make, x_shape, fmt, replays: int = 4) -> dict:  # type: ignore[no-untyped-def]
    dev = torch.device('cuda')
    torch.manual_seed(0)
    mod = make().to(dev).to(memory_format=fmt)
    x = torch.randn(*x_shape, device=dev).contiguous(memory_format=fmt).requires_grad_(True)
    w = torch.randn_like(mod(x)).contiguous(memory_format=fmt)

    def run() -> list[torch.Tensor]:
        out = mod(x)
        (out * w).sum().backward()
        return [out.detach()]

    for _ in range(2):
        mod.zero_grad(set_to_none=False)
        x.grad = None
        ref_out = run()
    ref = ref_out + [x.grad.clone()] + [p.grad.clone() for p in mod.parameters()]
    mod.zero_grad(set_to_none=True)
    x.grad = None
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            outs = run()
    torch.cuda.current_stream().wait_stream(s)
    got = outs + [x.grad] + [p.grad for p in mod.parameters()]
    res = []
    for _ in range(replays):
        g.replay()
        torch.cuda.synchronize()
        res.append(max(float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
                       for a, b in zip(got, ref)))
    return {'case': name, 'fmt': 'cl' if fmt == torch.channels_last else 'nchw', 'maxrel': res}


def main() -> None:
    torch.backends.cudnn.deterministic = True
    cases = [
        ('conv3x3', lambda: torch.nn.Conv2d(64, 64, 3, padding=1, bias=False), (8, 64, 16, 16)),
        ('conv1x1', lambda: torch.nn.Conv2d(256, 64, 1, bias=False), (8, 256, 16, 16)),
        ('conv1x1_s2', lambda: torch.nn.Conv2d(256, 512, 1, stride=2, bias=False), (8, 256, 16, 16)),
        ('conv7x7_s2', lambda: torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), (8, 3, 64, 64)),
        ('bn', lambda: torch.nn.BatchNorm2d(256), (8, 256, 16, 16)),
        ('bn_small', lambda: torch.nn.BatchNorm2d(64), (8, 64, 32, 32)),
        ('bn_relu', lambda: torch.nn.Sequential(torch.nn.BatchNorm2d(256), torch.nn.ReLU()),
         (8, 256, 16, 16)),
        ('maxpool', lambda: torch.nn.MaxPool2d(3, 2, 1), (8, 64, 32, 32)),
    ]
    for fmt in (torch.channels_last, torch.contiguous_format):
        for name, make, shape in cases:
            for rep in range(2):
                print(json.dumps(case(f'{name}#{rep}', make, shape, fmt)), flush=True)


if __name__ == '__main__':
    main()
