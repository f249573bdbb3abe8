"""Eigen-refresh wall time for the ResNet-50 factor set (108 SPD matrices,
n = 64..4608) under three schedules:
  bucketed  -- current eigh_many (size buckets, side streams, one thread)
  streams   -- one rocSOLVER call per matrix, K streams, one host thread
  threads   -- one call per matrix, K streams each driven by its own host
               thread (binding releases the GIL)."""
from __future__ import annotations

import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.ops import _native  # noqa: E402
from distributed_kfac_pytorch_amd.ops import linalg  # noqa: E402
from tools.bench_gemm import LAYERS  # noqa: E402


def spd(n: int, dev: torch.device) -> torch.Tensor:
    x = torch.randn(n, n, device=dev)
    return x @ x.t() / n + 0.01 * torch.eye(n, device=dev)


def main() -> None:
    lib = _native.native()
    dev = torch.device('cuda')
    torch.manual_seed(0)
    sizes = []
    for g, a, cnt in LAYERS:
        sizes += [g] * cnt + [a] * cnt
    mats = [spd(n, dev) for n in sizes]
    torch.cuda.synchronize()

    def run_bucketed() -> None:
        linalg.eigh_many(mats)

    def sched(k: int) -> list[list[torch.Tensor]]:
        lanes = [[] for _ in range(k)]
        load = [0.0] * k
        for m in sorted(mats, key=lambda m: -m.shape[0]):
            j = load.index(min(load))
            lanes[j].append(m)
            load[j] += float(m.shape[0]) ** 3
        return lanes

    def one(m: torch.Tensor) -> None:
        if m.shape[0] <= linalg.JACOBI_MAX_N:
            linalg.eigh_many([m])
        else:
            lib.rocsolver_eigh(m.clone().unsqueeze(0), 0, 100, 1e-7)

    def run_streams(k: int) -> None:
        main_s = torch.cuda.current_stream()
        streams = [torch.cuda.Stream() for _ in range(k)]
        for s, lane in zip(streams, sched(k)):
            s.wait_stream(main_s)
            with torch.cuda.stream(s):
                for m in lane:
                    one(m)
        for s in streams:
            main_s.wait_stream(s)

    def run_threads(k: int) -> None:
        main_s = torch.cuda.current_stream()
        streams = [torch.cuda.Stream() for _ in range(k)]
        lanes = sched(k)

        def work(s: torch.cuda.Stream, lane: list) -> None:
            with torch.cuda.stream(s):
                for m in lane:
                    one(m)

        for s in streams:
            s.wait_stream(main_s)
        ts = [threading.Thread(target=work, args=(s, lane)) for s, lane in zip(streams, lanes)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for s in streams:
            main_s.wait_stream(s)

    def run_hybrid(k: int, split_n: int = 1024) -> None:
        # size buckets (batched calls); big buckets split per matrix; LPT over
        # k host threads, each with its own stream
        buckets: dict[int, list] = {}
        for m in mats:
            buckets.setdefault(m.shape[0], []).append(m)
        items = []
        for n, ms in buckets.items():
            if n >= split_n:
                items += [(n, [m]) for m in ms]
            else:
                items.append((n, ms))
        cost = lambda it: float(it[0]) ** 3 * (len(it[1]) if it[0] >= 256 else 1 + 0.1 * len(it[1]))
        lanes = [[] for _ in range(k)]
        load = [0.0] * k
        for it in sorted(items, key=lambda it: -cost(it)):
            j = load.index(min(load))
            lanes[j].append(it)
            load[j] += cost(it)
        main_s = torch.cuda.current_stream()
        streams = [torch.cuda.Stream() for _ in range(k)]

        def work(s: torch.cuda.Stream, lane: list) -> None:
            with torch.cuda.stream(s):
                for n, ms in lane:
                    linalg.eigh_many(ms) if n <= linalg.JACOBI_MAX_N else \
                        lib.rocsolver_eigh(torch.stack(ms), 0, 100, 1e-7)

        for s in streams:
            s.wait_stream(main_s)
        ts = [threading.Thread(target=work, args=(s, lane)) for s, lane in zip(streams, lanes)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for s in streams:
            main_s.wait_stream(s)

    def timeit(fn) -> float:
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    res = {'n_mats': len(mats), 'bucketed_ms': round(timeit(run_bucketed), 1)}
    for k in (4, 8, 12):
        res[f'hybrid{k}_ms'] = round(timeit(lambda: run_hybrid(k)), 1)
    for k in (8,):
        res[f'hybrid{k}_split2048_ms'] = round(timeit(lambda: run_hybrid(k, 2048)), 1)
        res[f'hybrid{k}_split512_ms'] = round(timeit(lambda: run_hybrid(k, 512)), 1)
    for k in (12,):
        res[f'threads{k}_ms'] = round(timeit(lambda: run_threads(k)), 1)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
