"""Per-phase time of the grouped preconditioning GEMMs (gemm3s) on the
ResNet-50 layer set, split-K on vs off (``KFAC_G3S_SPLITK``).

Runs a few K-FAC steps of ResNet-50 (batch 32, fp32) so every layer has
eigenbases, then rebuilds the grouped tables under each setting and times
each phase's launch (T1, T2, T3, T4; the split-K combine counted with its
GEMM) with HIP events over ``--reps`` repetitions.  One JSON line per
setting.

    python tools/g3s_splitk_probe.py --reps 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import resnet50
from distributed_kfac_pytorch_amd.ops import precondition as pops
from distributed_kfac_pytorch_amd.ops._native import native


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--batch', type=int, default=32)
    args = ap.parse_args()
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = resnet50().to(dev).to(memory_format=torch.channels_last)
    pre = kfac.KFACPreconditioner(model, factor_update_steps=1, inv_update_steps=2, lr=0.1)
    pre._graphs = None
    x = torch.randn(args.batch, 3, 224, 224, device=dev).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    for _ in range(3):
        model.zero_grad(set_to_none=False)
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
    torch.cuda.synchronize()
    g = pre._grouped
    assert isinstance(g, pops.SplitGroupedPrecondition), type(g)
    layers, damping = g._layers, pre.damping
    lib = native()
    for setting in ('1', '0', '1'):
        os.environ['KFAC_G3S_SPLITK'] = setting
        g._cache = pops._TableCache(slots_per_entry=6)
        g._key = None
        assert g.prepare(layers, damping)
        times: dict[str, float] = {}
        for _ in range(3):
            g.launch()
        torch.cuda.synchronize()
        for entry in g._tables:
            name = entry[0]
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(args.reps):
                if name == 'split':
                    _, tab, n, blocks, _ = entry
                    lib.split_pad_multi(tab, n, blocks)
                else:
                    _, tab, n, tiles, (amc, bmc, osplit), _, (ncomb, cblocks) = entry
                    lib.gemm3s_grouped(tab, n, tiles, amc, bmc, osplit)
                    if ncomb:
                        lib.gemm3s_combine(tab, n, ncomb, cblocks, osplit)
            ev1.record()
            torch.cuda.synchronize()
            times[name] = round(ev0.elapsed_time(ev1) * 1000 / args.reps, 1)
        splits = {e[0]: e[6][0] for e in g._tables if e[0] != 'split'}
        print(json.dumps({'splitk': setting, 'us': times, 'total_us': round(sum(times.values()), 1),
                          'split_layers': splits}), flush=True)


if __name__ == '__main__':
    main()
