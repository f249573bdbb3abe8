"""Which MIOpen convolution solvers give inconsistent HIP-graph replays?

    python tools/conv_replay_probe.py [--bf16] [--conv1x1 gemm|miopen] [--db tuned|fresh|<dir>]

For every convolution of ResNet-50 (bench shape: batch 32, 224x224,
channels_last) that still runs through MIOpen, one graph is captured of
``y = conv(x)`` plus ``dX, dW = grad(sum(y^2))`` on fixed inputs, then:

* ``eager``: the same op run eagerly twice -> solver noise (atomics);
* ``replay``: two back-to-back replays -> replay noise;
* ``interleaved``: a replay after the WHOLE model ran one eager forward +
  backward (every other convolution's solver ran on the same MIOpen handle
  in between) -> does the graph depend on state some other solver call
  overwrites (handle-owned scratch, a workspace not re-zeroed in the graph)?
* ``vs_eager``: replay against the eager result.

Each is a relative Frobenius difference per output (y, dX, dW).  A solver
whose ``interleaved`` or ``vs_eager`` difference is far above its eager noise
is unsafe inside a captured step.  One JSON line per convolution.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import zlib

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _db_from_argv() -> None:
    db = 'tuned'
    for i, a in enumerate(sys.argv):
        if a == '--db' and i + 1 < len(sys.argv):
            db = sys.argv[i + 1]
        elif a.startswith('--db='):
            db = a.split('=', 1)[1]
    if db == 'tuned':
        os.environ['MIOPEN_USER_DB_PATH'] = os.path.join(_ROOT, 'miopen_db')
    elif db == 'fresh':
        os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='miopen_fresh_')
    else:
        os.environ['MIOPEN_USER_DB_PATH'] = os.path.abspath(db)


_db_from_argv()

import torch  # noqa: E402

sys.path.insert(0, _ROOT)

from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import GemmConv1x1  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1  # noqa: E402


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double(), b.double()
    if not bool(torch.isfinite(a).all()) or not bool(torch.isfinite(b).all()):
        return float('inf')
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--bf16', action='store_true')
    ap.add_argument('--conv1x1', default='gemm', choices=['gemm', 'miopen'])
    ap.add_argument('--db', default='tuned')
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--only', default='', help='comma list of conv names')
    ap.add_argument('--deterministic', type=int, default=0,
                    help='torch.backends.cudnn.deterministic (the twin test sets it)')
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = bool(args.deterministic)
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    if args.conv1x1 == 'gemm':
        use_gemm_conv1x1(model)
    amp = args.bf16
    x = torch.randn(args.batch, 3, args.image, args.image, device=dev).contiguous(
        memory_format=torch.channels_last)
    yl = torch.randint(0, 1000, (args.batch,), device=dev)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)

    def ac():  # type: ignore[no-untyped-def]
        return torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp, cache_enabled=False)

    def whole() -> None:
        model.zero_grad(set_to_none=True)
        with ac():
            loss = crit(model(x), yl)
        loss.backward()

    whole()
    torch.cuda.synchronize()
    shapes: dict = {}
    hooks = []
    for nm, mm in model.named_modules():
        if isinstance(mm, torch.nn.Conv2d) and not isinstance(mm, GemmConv1x1):
            def rec(mod, inp, out, nm=nm) -> None:  # type: ignore[no-untyped-def]
                shapes.setdefault(nm, tuple(inp[0].shape))
            hooks.append(mm.register_forward_hook(rec))
    with torch.no_grad(), ac():
        model(x)
    for h in hooks:
        h.remove()
    only = {s for s in args.only.split(',') if s}
    summary = {'db': os.environ['MIOPEN_USER_DB_PATH'], 'bf16': amp, 'convs': len(shapes)}
    print(json.dumps(summary), flush=True)
    worst = 0.0
    for nm, mm in model.named_modules():
        if nm not in shapes or (only and nm not in only):
            continue
        gen = torch.Generator(device=dev).manual_seed(zlib.crc32(nm.encode()))
        xin = torch.randn(shapes[nm], device=dev, generator=gen).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)

        def fn(mm=mm, xin=xin) -> list:  # type: ignore[no-untyped-def]
            with ac():
                z = mm(xin)
            gx, gw = torch.autograd.grad(z.float().square().sum(), [xin, mm.weight])
            return [z, gx, gw]

        e1 = [t.detach().clone() for t in fn()]
        e2 = [t.detach().clone() for t in fn()]
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()  # warm on the capture stream
            with torch.cuda.graph(g, stream=side):
                outs = fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()

        def replay() -> list:
            g.replay()
            torch.cuda.synchronize()
            return [o.detach().clone() for o in outs]

        r1 = replay()
        r2 = replay()
        whole()  # every solver of the model runs eagerly in between
        torch.cuda.synchronize()
        r3 = replay()
        names = ('y', 'dx', 'dw')
        rec = {'conv': nm, 'in': list(shapes[nm]), 'k': list(mm.kernel_size),
               'stride': list(mm.stride), 'cout': mm.out_channels}
        for key, (a, b) in {'eager': (e1, e2), 'replay': (r1, r2),
                            'interleaved': (r3, r1), 'vs_eager': (r1, e1)}.items():
            rec[key] = {n: rel(p, q) for n, p, q in zip(names, a, b)}
        noise = max(max(rec['eager'].values()), 1e-6)
        bad = max(max(rec['interleaved'].values()), max(rec['vs_eager'].values()))
        rec['flag'] = bool(bad > max(1e-2, 100 * noise))
        worst = max(worst, bad)
        print(json.dumps(rec), flush=True)
        del g, outs
    print(json.dumps({'done': True, 'worst': worst}), flush=True)


if __name__ == '__main__':
    main()
