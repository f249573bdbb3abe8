"""Host-side audit of every device pointer baked into the K-FAC descriptor
tables of freshly captured step graphs (nothing is replayed or launched).

Decodes each cached table's staging bytes (csrc/descs.h layouts) and checks
that every pointer lies inside an ACTIVE block of the caching allocator
(``torch.cuda.memory_snapshot``).  A pointer into a free block means a graph
would read or write memory the allocator can hand to someone else.

    python tools/graph_ptr_audit.py [--fp32]
"""
from __future__ import annotations

import argparse
import bisect
import json
import os
import struct
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from graph_nan_probe import build  # noqa: E402

from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402

# (record bytes, pointer field names) per descriptor type (csrc/descs.h)
LAYOUTS = {
    'gemm3s': (128, ['A', 'B', 'C', 'S', 'dg', 'da']),
    'split': (72, ['src', 'extra', 'dst']),
    'apply': (80, ['p', 'w', 'b']),
}


def active_blocks() -> tuple[list[int], list[tuple[int, int, str]]]:
    blocks = []
    for seg in torch.cuda.memory_snapshot():
        addr = seg['address']
        for b in seg['blocks']:
            blocks.append((addr, addr + b['size'], b['state']))
            addr += b['size']
    blocks.sort()
    return [b[0] for b in blocks], blocks


def lookup(starts: list[int], blocks: list, p: int) -> str:
    i = bisect.bisect_right(starts, p) - 1
    if i < 0 or p >= blocks[i][1]:
        return 'unmapped'
    return blocks[i][2]


def audit(pre, label: str) -> None:  # type: ignore[no-untyped-def]
    torch.cuda.synchronize()
    starts, blocks = active_blocks()
    report = {'at': label, 'bad': [], 'checked': 0}
    caches = [('grouped', pre._grouped._cache)] if pre._grouped is not None else []
    if pre._multi_apply is not None:
        caches.append(('apply', pre._multi_apply._tables))
    for owner, cache in caches:
        for key, (value, _slots, _ev) in cache._d.items():
            sticky = key in cache._sticky
            if owner == 'grouped':
                ents = [(e[0], e[1], e[2], e[-1]) for e in value if e is not None]
            else:
                ents = [('apply', value[0], len(key), value[2])]
            for kind, dev, n, host in ents:
                layout = 'split' if kind == 'split' else ('apply' if kind == 'apply' else 'gemm3s')
                rec, fields = LAYOUTS[layout]
                raw = bytes(host[: rec * n].numpy())
                st = lookup(starts, blocks, dev.data_ptr())
                report['checked'] += 1
                if st != 'active_allocated':
                    report['bad'].append({'table': kind, 'sticky': sticky, 'field': 'TABLE',
                                          'state': st})
                for i in range(n):
                    for j, f in enumerate(fields):
                        (p,) = struct.unpack_from('<Q', raw, i * rec + 8 * j)
                        if p == 0:
                            continue
                        report['checked'] += 1
                        s = lookup(starts, blocks, p)
                        if s != 'active_allocated':
                            report['bad'].append({'table': kind, 'sticky': sticky, 'rec': i,
                                                  'field': f, 'ptr': hex(p), 'state': s})
    print(json.dumps(report), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--fp32', action='store_true')
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = True
    dev = torch.device('cuda')
    torch.manual_seed(0)
    base = resnet50(num_classes=10)
    model, opt, pre, x, y, runner = build(base, dev, True, not args.fp32, True)
    gen = torch.Generator(device='cpu').manual_seed(1)
    x.copy_(torch.randn(8, 3, 64, 64, generator=gen))
    y.copy_(torch.randint(0, 10, (8,), generator=gen))
    runner()  # step 0 (eager refresh)
    runner()  # step 1 (eager: warmup after the signature is first seen)
    audit(pre, 'eager tables after step 1')
    runner.signature = runner._signature()
    runner._capture('plain')
    audit(pre, 'after plain capture')
    runner._capture('factor')
    audit(pre, 'after factor capture')
    # grads of each graph must be live
    starts, blocks = active_blocks()
    for k, gl in runner.grads.items():
        bad = [lookup(starts, blocks, g.data_ptr()) for g in gl if g is not None]
        print(json.dumps({'grads': k, 'not_active': [b for b in bad if b != 'active_allocated']}))


if __name__ == '__main__':
    main()
