"""Find memory that a captured whole-step graph reads but does not own.

A HIP graph replays fixed addresses.  Memory it reads must stay allocated
for the graph's life: either in the graph's private pool, or held by a live
tensor.  A block that lives in the caching allocator's global pool and is
*free* after the capture can be handed to any later eager allocation, and
the next replay then reads (or writes) someone else's data.

Two independent probes, in one process, on the bench configuration
(ResNet-50, channels_last, fused SGD, optional K-FAC / bf16 autocast):

1. allocator history (``torch.cuda.memory._record_memory_history``) around
   the capture: every block that was allocated BEFORE the capture began and
   freed DURING it (the graph may still read it), and every block allocated
   during the capture outside the private pool, with Python stacks;
2. poison: after the capture, fill every free block of the global pool with
   0xFF bytes (NaN in fp32 / bf16) and replay once from a saved state; if the
   result differs from a clean replay from the same state the graph reads
   free global memory.  The poisoned set is bisected down to the culprit
   block(s), whose alloc/free history is printed.

    python tools/graph_oop_audit.py [--bf16] [--no-kfac] [--image 224 --batch 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

if '--miopen-db' in sys.argv:
    # the tuned MIOpen database bench.py uses (before MIOpen initialises)
    os.environ.setdefault('MIOPEN_USER_DB_PATH', os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'miopen_db'))

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402
from distributed_kfac_pytorch_amd.ops.cast import enable_fused_weight_cast  # noqa: E402

_S0 = 7777 * 512  # sentinel allocation sizes marking the capture window
_S1 = 7779 * 512


def unsafe(model: nn.Module) -> None:
    """Undo ops/conv.py: plain nn.Conv2d strided 1x1 shortcuts."""
    from distributed_kfac_pytorch_amd.ops.conv import StridedConv1x1
    for mm in model.modules():
        if type(mm) is StridedConv1x1:
            mm.__class__ = nn.Conv2d


def _frames(fr: list, n: int = 8) -> list[str]:
    out = []
    for f in fr:
        fn = f.get('filename', '')
        if 'torch/' in fn and 'nn/modules' not in fn:
            continue
        out.append(f"{os.path.basename(fn)}:{f.get('line')} {f.get('name')}")
        if len(out) >= n:
            break
    return out


def build(args: argparse.Namespace, dev: torch.device):  # type: ignore[no-untyped-def]
    torch.manual_seed(0)
    model = get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    if not args.graph_safe:
        unsafe(model)
    amp = args.bf16
    if amp and args.fused_cast:
        enable_fused_weight_cast(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          **({'fused': True} if args.fused_sgd else {'foreach': True}))
    pre = None
    if not args.no_kfac:
        pre = kfac.KFACPreconditioner(
            model, factor_update_steps=args.factor_steps, inv_update_steps=args.inv_steps,
            damping=0.001, factor_decay=0.95, kl_clip=0.001,
            lr=lambda s: opt.param_groups[0]['lr'], allreduce_bucket_cap_mb=25,
            colocate_factors=True, grad_worker_fraction=0.5)
    x = torch.randn(args.batch, 3, args.image, args.image, device=dev).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)

    def fb() -> torch.Tensor:
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            loss = crit(model(x), y)
        loss.backward()
        return loss

    runner = GraphedTrainStep(fb, opt, pre, warmup=1, enabled=True, conv_mode=args.conv_mode)
    return model, opt, pre, runner


def _state(model, opt) -> list[torch.Tensor]:  # type: ignore[no-untyped-def]
    ts = list(model.parameters()) + [b for b in model.buffers()]
    for p in model.parameters():
        st = opt.state.get(p, {})
        if st.get('momentum_buffer') is not None:
            ts.append(st['momentum_buffer'])
    return ts


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--bf16', action='store_true')
    ap.add_argument('--conv-mode', default=None, choices=[None, 'strided', 'gemm'],
                    help="GraphedTrainStep conv_mode (bench: 'gemm' under bf16)")
    ap.add_argument('--no-kfac', action='store_true')
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--fused-sgd', type=int, default=1)
    ap.add_argument('--fused-cast', type=int, default=1)
    ap.add_argument('--factor-steps', type=int, default=10)
    ap.add_argument('--inv-steps', type=int, default=100)
    ap.add_argument('--steps', type=int, default=4, help='steps before the audit (>= capture)')
    ap.add_argument('--max-report', type=int, default=40)
    ap.add_argument('--miopen-db', action='store_true', help="use the repo's tuned MIOpen db")
    ap.add_argument('--deterministic', type=int, default=1)
    ap.add_argument('--graph-safe', type=int, default=1,
                    help='0: plain nn.Conv2d for the strided 1x1 shortcuts (reproduces the bug)')
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = bool(args.deterministic)
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    lib = _native.native()
    assert lib is not None and hasattr(lib, 'memset_raw'), _native.load_error()

    torch.cuda.memory._record_memory_history(enabled='all', context='all', stacks='python',
                                             max_entries=1_000_000)
    # sentinels around every capture
    orig_begin = torch.cuda.CUDAGraph.capture_begin
    orig_end = torch.cuda.CUDAGraph.capture_end

    def begin(self, *a, **k):  # type: ignore[no-untyped-def]
        t = torch.empty(_S0, dtype=torch.uint8, device=dev)
        del t
        return orig_begin(self, *a, **k)

    def end(self, *a, **k):  # type: ignore[no-untyped-def]
        r = orig_end(self, *a, **k)
        t = torch.empty(_S1, dtype=torch.uint8, device=dev)
        del t
        return r

    torch.cuda.CUDAGraph.capture_begin = begin
    torch.cuda.CUDAGraph.capture_end = end

    model, opt, pre, runner = build(args, dev)
    for i in range(args.steps):
        runner()
    torch.cuda.synchronize()
    report: dict = {'config': vars(args), 'captures': runner.captures,
                    'replays': runner.replays, 'kinds': sorted(runner.graphs)}
    snap = torch.cuda.memory._snapshot()
    trace = snap['device_traces'][dev.index]
    segs = snap['segments']

    def pool_of(addr: int):  # type: ignore[no-untyped-def]
        for s in segs:
            if s['address'] <= addr < s['address'] + s['total_size']:
                return tuple(s.get('segment_pool_id', (0, 0)))
        return None

    # ---------------------------------------------------- 1. history
    wins = []
    start = None
    for i, e in enumerate(trace):
        if e['action'] == 'alloc' and e['size'] == _S0:
            start = i
        elif e['action'] == 'alloc' and e['size'] == _S1 and start is not None:
            wins.append((start, i))
            start = None
    report['capture_windows'] = len(wins)
    last_alloc: dict[int, int] = {}
    suspects = []
    outside_allocs = []
    wi = 0
    for i, e in enumerate(trace):
        a = e.get('addr')
        act = e['action']
        inwin = any(s < i < t for s, t in wins)
        if act == 'alloc':
            last_alloc[a] = i
            if inwin:
                pid = pool_of(a)
                if pid is not None and pid == (0, 0):
                    outside_allocs.append({'size': e['size'], 'stream': e['stream'],
                                           'frames': _frames(e.get('frames', []))})
        elif act == 'free_requested' and inwin:
            j = last_alloc.get(a)
            win = next(((s, t) for s, t in wins if s < i < t), None)
            if j is not None and win is not None and j < win[0]:
                suspects.append({'addr': hex(a), 'size': e['size'], 'stream': e['stream'],
                                 'alloc_frames': _frames(trace[j].get('frames', [])),
                                 'free_frames': _frames(e.get('frames', []))})
    report['freed_during_capture_allocated_before'] = suspects[:args.max_report]
    report['n_freed_during_capture_allocated_before'] = len(suspects)
    report['allocated_during_capture_in_global_pool'] = outside_allocs[:args.max_report]
    report['n_allocated_during_capture_in_global_pool'] = len(outside_allocs)
    print(json.dumps({'history': report}), flush=True)

    # ---------------------------------------------------- 2. poison
    kind = 'plain' if 'plain' in runner.graphs else next(iter(runner.graphs))
    g = runner.graphs[kind]
    grads = runner.grads[kind]
    st = _state(model, opt)
    saved = [t.detach().cpu().clone() for t in st]

    def restore() -> None:
        for t, s in zip(st, saved):
            t.data.copy_(s)
        torch.cuda.synchronize()

    def outcome() -> list[torch.Tensor]:
        g.replay()
        torch.cuda.synchronize()
        return [t.detach().float().cpu() for t in list(model.parameters())] + \
            [t.detach().float().cpu() for t in grads if t is not None]

    def rel(x: torch.Tensor, y: torch.Tensor) -> float:
        if not bool(torch.isfinite(y).all()):
            return float('inf')
        return float((x - y).abs().max() / x.abs().max().clamp_min(1e-30))

    noise = [0.0]

    def differs(a: list, b: list) -> int:
        # exact with deterministic kernels; otherwise only differences far
        # above the run-to-run noise of atomics-based kernels count
        if args.deterministic:
            return sum(int(not torch.equal(x, y)) for x, y in zip(a, b))
        return sum(int(rel(x, y) > max(1e-3, 100 * noise[0])) for x, y in zip(a, b))

    restore()
    clean = outcome()
    restore()
    clean2 = outcome()
    noise[0] = max([rel(x, y) for x, y in zip(clean, clean2)] or [0.0])
    det = differs(clean, clean2)
    free_blocks = []
    snap2 = torch.cuda.memory._snapshot()
    for s in snap2['segments']:
        if tuple(s.get('segment_pool_id', (0, 0))) != (0, 0):
            continue
        addr = s['address']
        for b in s['blocks']:
            ba = b.get('address', addr)
            if b['state'] == 'inactive':
                free_blocks.append((ba, b['size']))
            addr = ba + b['size']
    pres = {'kind': kind, 'nondeterministic_tensors': det, 'noise_rel': noise[0],
            'free_global_blocks': len(free_blocks),
            'free_global_mb': round(sum(b[1] for b in free_blocks) / 2**20, 1)}

    def poisoned(blocks: list) -> int:
        restore()
        for a, n in blocks:
            lib.memset_raw(a, n, 0xFF)
        torch.cuda.synchronize()
        return differs(clean, outcome())

    full = poisoned(free_blocks)
    pres['poison_all_differs'] = full
    culprits = []
    if full and not det:
        cand = list(free_blocks)
        while len(cand) > 1:
            h = len(cand) // 2
            lo, hi = cand[:h], cand[h:]
            if poisoned(lo):
                cand = lo
            elif poisoned(hi):
                cand = hi
            else:
                break
        for a, n in cand[:8]:
            hist = []
            for e in trace:
                ea = e.get('addr')
                if ea is None or e['action'] not in ('alloc', 'free_requested'):
                    continue
                if ea <= a < ea + e['size'] or a <= ea < a + n:
                    hist.append({'action': e['action'], 'addr': hex(ea), 'size': e['size'],
                                 'stream': e['stream'], 'frames': _frames(e.get('frames', []))})
            culprits.append({'addr': hex(a), 'size': n, 'history_tail': hist[-6:]})
    pres['culprits'] = culprits
    print(json.dumps({'poison': pres}), flush=True)
    torch.cuda.memory._record_memory_history(enabled=None)


if __name__ == '__main__':
    main()
