"""Bisect which part of a captured ResNet-50 step reads free global memory.

Companion of ``tools/graph_oop_audit.py``: after one eager training step,
each stage below is captured into its own HIP graph (private pool, side
stream, like ``GraphedTrainStep``) and replayed three times from the same
saved state -- twice clean, once after every free block of the caching
allocator's global pool has been filled with 0xFF.  A stage whose poisoned
replay differs from its clean replays reads memory that neither its pool nor
a live tensor owns.

    python tools/graph_oop_bisect.py [--bf16] [--stages conv1,stem,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

if '--miopen-db' in sys.argv:
    # the tuned MIOpen database bench.py uses (must be set before MIOpen
    # initialises)
    os.environ.setdefault('MIOPEN_USER_DB_PATH', os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db'))

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402


def unsafe(model: nn.Module) -> None:
    """Undo ops/conv.py: plain nn.Conv2d strided 1x1 shortcuts."""
    from distributed_kfac_pytorch_amd.ops.conv import StridedConv1x1
    for mm in model.modules():
        if type(mm) is StridedConv1x1:
            mm.__class__ = nn.Conv2d


def free_global_blocks() -> list[tuple[int, int]]:
    out = []
    for s in torch.cuda.memory_snapshot():
        if tuple(s.get('segment_pool_id', (0, 0))) != (0, 0):
            continue
        addr = s['address']
        for b in s['blocks']:
            ba = b.get('address', addr)
            if b['state'] == 'inactive':
                out.append((ba, b['size']))
            addr = ba + b['size']
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--bf16', action='store_true')
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--stages', default='conv1,conv1_bwd,stem,layer1,fwd,loss,fwd_bwd,full')
    ap.add_argument('--eager-steps', type=int, default=1)
    ap.add_argument('--stages-quiet', type=int, default=0, help='print only failing stages')
    ap.add_argument('--miopen-db', action='store_true', help="use the repo's tuned MIOpen db")
    ap.add_argument('--deterministic', type=int, default=1)
    ap.add_argument('--fused-bn', type=int, default=1)
    ap.add_argument('--graph-safe', type=int, default=1,
                    help='0: plain nn.Conv2d for the strided 1x1 shortcuts (reproduces the bug)')
    args = ap.parse_args()
    if not args.fused_bn:
        os.environ['KFAC_FUSED_BN'] = '0'
    torch.backends.cudnn.deterministic = bool(args.deterministic)
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    lib = _native.native()
    assert lib is not None and hasattr(lib, 'memset_raw'), _native.load_error()
    torch.manual_seed(0)
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    if not args.graph_safe:
        unsafe(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
    x = torch.randn(args.batch, 3, args.image, args.image, device=dev).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    amp = args.bf16

    def ac():  # type: ignore[no-untyped-def]
        return torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp, cache_enabled=False)

    for _ in range(args.eager_steps):
        opt.zero_grad(set_to_none=False)
        with ac():
            loss = crit(model(x), y)
        loss.backward()
        opt.step()
    # no autograd graph (and its AccumulateGrad nodes) may outlive the eager
    # steps: captured backwards would reuse nodes bound to the eager stream
    del loss
    torch.cuda.synchronize()
    m = model

    def st_conv1():  # type: ignore[no-untyped-def]
        with ac():
            return [m.conv1(x)]

    def st_conv1_bwd():  # type: ignore[no-untyped-def]
        with ac():
            z = m.conv1(x)
        gw, = torch.autograd.grad(z.float().square().sum(), [m.conv1.weight])
        return [z, gw]

    def st_stem():  # type: ignore[no-untyped-def]
        with ac():
            return [m.maxpool(m.bn1.act(m.conv1(x)))]

    def st_layer1():  # type: ignore[no-untyped-def]
        with ac():
            return [m.layer1(m.maxpool(m.bn1.act(m.conv1(x))))]

    def st_fwd():  # type: ignore[no-untyped-def]
        with ac():
            return [m(x)]

    def st_loss():  # type: ignore[no-untyped-def]
        with ac():
            return [crit(m(x), y)]

    def st_fwd_bwd():  # type: ignore[no-untyped-def]
        opt.zero_grad(set_to_none=True)
        with ac():
            loss = crit(m(x), y)
        loss.backward()
        return [loss.detach()] + [p.grad for p in m.parameters()]

    def st_full():  # type: ignore[no-untyped-def]
        opt.zero_grad(set_to_none=True)
        with ac():
            loss = crit(m(x), y)
        loss.backward()
        opt.step()
        return [loss.detach()] + [p.grad for p in m.parameters()] + list(m.parameters())

    params = list(m.parameters())
    feat = torch.randn(args.batch, 2048, device=dev)
    l4in = torch.randn(args.batch, 1024, args.image // 16, args.image // 16, device=dev).contiguous(
        memory_format=torch.channels_last)

    def st_grad_api():  # type: ignore[no-untyped-def]
        with ac():
            loss = crit(m(x), y)
        return list(torch.autograd.grad(loss, params))

    def _bwd(loss: torch.Tensor, mods: list) -> list:
        opt.zero_grad(set_to_none=True)
        loss.backward()
        return [p.grad for mm in mods for p in mm.parameters()]

    def st_fc_bwd():  # type: ignore[no-untyped-def]
        with ac():
            loss = crit(m.fc(feat), y)
        return _bwd(loss, [m.fc])

    def st_stem_bwd():  # type: ignore[no-untyped-def]
        with ac():
            z = m.maxpool(m.bn1.act(m.conv1(x)))
        return _bwd(z.float().square().mean(), [m.conv1, m.bn1])

    def st_layer4_bwd():  # type: ignore[no-untyped-def]
        with ac():
            z = m.layer4(l4in)
        return _bwd(z.float().square().mean(), [m.layer4])

    def st_head_bwd():  # type: ignore[no-untyped-def]
        with ac():
            loss = crit(m.fc(torch.flatten(m.avgpool(m.layer4(l4in)), 1)), y)
        return _bwd(loss, [m.layer4, m.fc])

    # every conv on its own: backward data + weight from a fixed input
    conv_in: dict = {}
    def rec(nm: str):  # type: ignore[no-untyped-def]
        def hook(mod, inp, out) -> None:  # type: ignore[no-untyped-def]
            conv_in.setdefault(nm, tuple(inp[0].shape))
        return hook
    hooks = [mm.register_forward_hook(rec(nm))
             for nm, mm in m.named_modules() if isinstance(mm, torch.nn.Conv2d)]
    with torch.no_grad(), ac():
        m(x)
    for h in hooks:
        h.remove()
    conv_stages = {}
    for nm, mm in m.named_modules():
        if not isinstance(mm, torch.nn.Conv2d):
            continue
        xin = torch.randn(conv_in[nm], device=dev).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)

        def st(mm=mm, xin=xin):  # type: ignore[no-untyped-def]
            with ac():
                z = mm(xin)
            return list(torch.autograd.grad(z.float().square().sum(), [xin, mm.weight]))
        conv_stages['conv:' + nm] = st

    stages = {'grad_api': st_grad_api, 'fc_bwd': st_fc_bwd, 'stem_bwd': st_stem_bwd,
              'layer4_bwd': st_layer4_bwd, 'head_bwd': st_head_bwd,
              'conv1': st_conv1, 'conv1_bwd': st_conv1_bwd, 'stem': st_stem,
              'layer1': st_layer1, 'fwd': st_fwd, 'loss': st_loss, 'fwd_bwd': st_fwd_bwd,
              'full': st_full, **conv_stages}
    args.stages = ','.join(','.join(conv_stages) if t == 'convs' else t
                           for t in args.stages.split(','))
    state = list(m.parameters()) + list(m.buffers()) + [
        opt.state[p]['momentum_buffer'] for p in m.parameters()
        if opt.state.get(p, {}).get('momentum_buffer') is not None]
    saved = [t.detach().cpu().clone() for t in state]

    def restore() -> None:
        with torch.no_grad():
            for t, s in zip(state, saved):
                t.copy_(s)
        torch.cuda.synchronize()

    for name in args.stages.split(','):
        fn = stages[name]
        restore()
        warm = fn()  # eager run of the stage (lazy state, workspaces)
        del warm
        torch.cuda.synchronize()
        restore()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                outs = fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()

        def run() -> list[torch.Tensor]:
            restore()
            g.replay()
            torch.cuda.synchronize()
            return [o.detach().float().cpu() for o in outs if o is not None]

        c1 = run()
        c2 = run()
        det = sum(int(not torch.equal(a, b)) for a, b in zip(c1, c2))
        restore()
        blocks = free_global_blocks()
        for a, n in blocks:
            lib.memset_raw(a, n, 0xFF)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        p = [o.detach().float().cpu() for o in outs if o is not None]
        bad = sum(int(not torch.equal(a, b)) for a, b in zip(c1, p))
        first = next((i for i, (a, b) in enumerate(zip(c1, p)) if not torch.equal(a, b)), None)

        def rel(a: torch.Tensor, b: torch.Tensor) -> float:
            if not bool(torch.isfinite(b).all()):
                return float('inf')
            return float((a - b).abs().max() / a.abs().max().clamp_min(1e-30))
        # atomics-based (non-deterministic) kernels differ run to run at the
        # 1e-6 level; a read of poisoned (0xFF) memory is far larger
        noise = max([rel(a, b) for a, b in zip(c1, c2)] or [0.0])
        gross = [i for i, (a, b) in enumerate(zip(c1, p)) if rel(a, b) > max(1e-3, 100 * noise)]
        if args.stages_quiet and not gross:
            del g, outs
            continue
        print(json.dumps({'stage': name, 'outputs': len(c1), 'nondet': det,
                          'noise_rel': noise, 'gross_outputs': gross,
                          'poisoned_differs': bad, 'first_bad_output': first,
                          'free_blocks': len(blocks),
                          'free_mb': round(sum(b[1] for b in blocks) / 2**20, 1)}), flush=True)
        del g, outs
        torch.cuda.synchronize()


if __name__ == '__main__':
    main()
