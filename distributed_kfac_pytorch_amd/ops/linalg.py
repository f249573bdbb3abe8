"""Second-order linear algebra: batched symmetric eigensolver and SPD inverse.

``eigh_many(mats)`` decomposes a list of symmetric fp32 matrices of mixed
sizes (all K-FAC factors a rank owns; the reference solves them one by one
with ``torch.linalg.eigh``, ``kfac/layers/eigen.py:294-347``).  Matrices are
bucketed by size; each bucket is one batched solve, and the buckets run
concurrently on a few HIP streams ("lanes", one host thread each, joined
back into the caller's stream with events).  Tiers, by size ``n``:

* ``n <= 128``: the LDS-resident parallel Jacobi kernel
  (csrc/eigh_jacobi.hip), one matrix per workgroup (``jacobi``);
* ``129 <= n <= 8192``: the native one-stage Householder tridiagonalisation
  (csrc/sytrd.hip).  Buckets are grouped into chains by size
  (``KFAC_SYTRD_SPLIT``, default n >= 4000 / >= 1000 / rest); a chain
  advances every member one column per launch pair on its own lane and is
  issued in segments ending where each bucket ends, so that bucket's tail --
  native divide and conquer on T (csrc/tridiag.hip, ``ops.tridiag``) and the
  blocked back-transform ``apply_q_blocked`` -- runs on another lane while
  the chain reduces the larger factors.  The largest chain and its tail run
  on high-priority lanes (``sytrd+dc``);
* buckets of many equal-size factors (n >= 700, >= 8 factors, count x n >=
  ``KFAC_TWOSTAGE_BUCKET_ROWS`` = 18000 rows, e.g. GPT-NeoX's 12 x 3072):
  the native two-stage solver (``ops.twostage``: dense -> band -> tridiagonal
  bulge chasing -> divide and conquer -> two back-transforms), whose bulge
  chase runs one workgroup per matrix and fills the chip with a large batch
  where one chain would be a single latency-bound sequence
  (``KFAC_EIGH_LARGE=twostage`` sends every factor above the Jacobi tier
  there);
* ``n`` above the native limits: rocSOLVER ``syevd`` through the native
  extension (no host synchronisation, unlike ``torch.linalg.eigh``).

CPU tensors, or ``KFAC_EIGH=torch``, use ``torch.linalg.eigh``.  Results
match ``torch.linalg.eigh``: ascending eigenvalues, eigenvectors in columns
(unique up to sign / rotation inside degenerate eigenspaces, which K-FAC's
``Q f(D) Q^T`` does not see).  Every result is checked for finiteness once
per call (``_repair_nonfinite``).

Other knobs: ``KFAC_EIGH_STREAMS`` (lanes, default 8, capped at
``GPU_MAX_HW_QUEUES``), ``KFAC_EIGH_THREADS=0`` (issue every lane from the
calling thread), ``KFAC_SYTRD_GRAPHS`` (replay chain segments from captured
HIP graphs), ``KFAC_SYTRD_WAVES`` / ``KFAC_SYTRD_SU`` (symv launch size /
loads in flight per row), ``KFAC_JACOBI_SWEEPS`` / ``KFAC_JACOBI_TOL``.
"""
from __future__ import annotations

import logging
import os
from collections import defaultdict
from typing import Any

import torch

from distributed_kfac_pytorch_amd.ops import twostage
from distributed_kfac_pytorch_amd.ops._native import load_error as _native_error
from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native

# largest n sent to the LDS Jacobi kernel (its hard limit is jacobi_max_n());
# everything above goes to the native tridiagonalisation
JACOBI_MAX_N = 128

logger = logging.getLogger(__name__)
_streams: list[torch.cuda.Stream] = []
# per-call statistics: last_stats['tiers'] = [(tier, n, count)] (tests, probes)
last_stats: dict[str, Any] = {}


def jacobi_max_n() -> int:
    lib = native()
    return int(lib.jacobi_max_n()) if lib is not None else 0


def _side_streams(device: torch.device) -> list[torch.cuda.Stream]:
    n = int(os.environ.get('KFAC_EIGH_STREAMS', '8'))
    global _streams
    if len(_streams) < n or _streams[0].device != device:
        _streams = [torch.cuda.Stream(device=device) for _ in range(n)]
    return _streams[:n]


def twostage_bucket_rows() -> int:
    """Size buckets of n >= 700 holding >= 8 factors and >= this many matrix
    rows in total (count x n; ``KFAC_TWOSTAGE_BUCKET_ROWS``, default 18000)
    go to the two-stage solver: its bulge chase runs one workgroup per
    matrix, so a large batch of equal-size factors fills the chip where a
    one-stage chain over the same bucket is one long latency-bound sequence.
    GPT-NeoX-125M (12 x 2304 / 3072 / 3073 = 27.6k-36.9k rows, 36 x 769,
    24 x 768 = 18.4k): eigen refresh 667 ms on the chains, 405 ms two-stage
    (profiles/neox_twostage_r3.txt).  ResNet-50's largest bucket has 14.3k
    rows (14 x 1024) and stays on the chains, which win there
    (profiles/twostage_r3.md)."""
    return int(os.environ.get('KFAC_TWOSTAGE_BUCKET_ROWS', '18000'))


def twostage_sizes(counts: dict) -> set:
    """Factor sizes the bucket-population rule sends to the two-stage solver,
    from ``{n: number of factors of size n}``."""
    rows = twostage_bucket_rows()
    return {n for n, c in counts.items() if n >= 700 and c >= 8 and c * n >= rows}


def large_algo() -> str:
    """``KFAC_EIGH_LARGE``: sytrd (default: one-stage chains, with the
    bucket-population rule's sizes on the two-stage solver) | twostage (every
    factor above the Jacobi tier)."""
    return os.environ.get('KFAC_EIGH_LARGE', 'sytrd')


def _use_twostage(n: int, ts_sizes: set) -> bool:
    """Native two-stage solver for this factor size (``ts_sizes``: this
    call's bucket-population rule result)."""
    if not JACOBI_MAX_N < n <= twostage.max_n():
        return False
    return large_algo() == 'twostage' or n in ts_sizes


def _use_sytrd(n: int) -> bool:
    """Native one-stage chain tier for factors of size n."""
    lib = native()
    return lib is not None and JACOBI_MAX_N < n <= int(lib.sytrd_max_n())


def _tier(name: str, n: int, count: int) -> None:
    """Record which solver handled a bucket (``last_stats['tiers']``)."""
    last_stats.setdefault('tiers', []).append((name, int(n), int(count)))


def _gpu_bucket(stack: torch.Tensor, ts_sizes: set) -> tuple[torch.Tensor, torch.Tensor]:
    """One size bucket on the current stream (everything but the chains)."""
    n = stack.shape[-1]
    lib = native()
    if n <= JACOBI_MAX_N:
        _tier('jacobi', n, stack.shape[0])
        return lib.jacobi_eigh(stack.contiguous(), int(os.environ.get('KFAC_JACOBI_SWEEPS', '15')),
                               float(os.environ.get('KFAC_JACOBI_TOL', '1e-7')))
    if _use_twostage(n, ts_sizes):
        _tier('twostage', n, stack.shape[0])
        if twostage.graphs_enabled():
            return twostage.eigh_twostage_graphed(stack)
        w, x, _, _ = twostage.eigh_twostage(stack)
        return w, x
    # above every native limit: rocSOLVER's divide and conquer
    _tier('syevd', n, stack.shape[0])
    return lib.rocsolver_eigh(stack.contiguous(), 0, 100, 1e-7)


def _bucket_cost(n: int, count: int) -> float:
    return float(count) * float(n) ** 3


def eigh_many(mats: list[torch.Tensor]) -> list[tuple[torch.Tensor, torch.Tensor]]:
    """Eigendecompose each symmetric matrix; returns ``[(evals, evecs)]``."""
    last_stats['tiers'] = []  # this call's buckets only
    out: list[tuple[torch.Tensor, torch.Tensor] | None] = [None] * len(mats)
    buckets: dict[tuple, list[int]] = defaultdict(list)
    for i, m in enumerate(mats):
        buckets[(m.shape[0], m.device)].append(i)
    gpu = [(k, v) for k, v in buckets.items() if k[1].type == 'cuda']
    host = [(k, v) for k, v in buckets.items() if k[1].type != 'cuda']
    if gpu and (os.environ.get('KFAC_EIGH', 'auto') == 'torch'
                or not use_native(*[mats[idxs[0]] for _, idxs in gpu])):
        host += gpu
        gpu = []
    for _, idxs in host:
        evals, evecs = torch.linalg.eigh(torch.stack([mats[i].to(torch.float32) for i in idxs]))
        for k, i in enumerate(idxs):
            out[i] = (evals[k], evecs[k])
    if gpu:
        dev = gpu[0][0][1]
        counts: dict[int, int] = defaultdict(int)
        for key, idxs in gpu:
            counts[key[0]] += len(idxs)
        stacks = {key: torch.stack([mats[i].to(torch.float32) for i in idxs])
                  for key, idxs in gpu}
        res = _launch_jobs(gpu, stacks, dev, twostage_sizes(counts))
        for i, r in res.items():
            out[i] = r
        _repair_nonfinite(mats, out, list(res))
    return [o for o in out if o is not None]


def _repair_nonfinite(mats: list[torch.Tensor], out: list, idxs: list[int]) -> None:
    """A failed solve must never be installed silently (rocSOLVER reports
    failures only in a device ``info`` flag; the bulge chase has a timeout
    flag).  One fused finiteness check over every result -- ONE host
    read-back per refresh, after the whole refresh has been enqueued; a
    non-finite factor is re-solved by torch's float64 eigh (the reference's
    routine, kfac/layers/eigen.py:294-347) and logged."""
    if not idxs:
        return
    # results are views of a few per-bucket stacks: check each stack once
    bases: dict[int, torch.Tensor] = {}
    for i in idxs:
        for t in out[i]:
            b = t._base if t._base is not None else t
            bases.setdefault(id(b), b)
    ok = torch.stack([torch.isfinite(b).all() for b in bases.values()]).all()
    if bool(ok):
        return
    flags = torch.stack([
        torch.isfinite(out[i][0]).all() & torch.isfinite(out[i][1]).all() for i in idxs
    ])
    bad = [i for i, good in zip(idxs, flags.tolist()) if not good]
    if not bad:
        return
    # a non-finite FACTOR (NaN / Inf gradients upstream) cannot be repaired
    # here: its results stay non-finite, as torch's eigh would fail on it
    fin = torch.stack([torch.isfinite(mats[i]).all() for i in bad]).tolist()
    fixable = [i for i, f in zip(bad, fin) if f]
    logger.warning('eigendecomposition: %d non-finite result(s) (sizes %s), %d of them '
                   'from non-finite factors; re-solving the others with torch float64 '
                   'eigh', len(bad), sorted({int(mats[i].shape[0]) for i in bad}),
                   len(bad) - len(fixable))
    for i in fixable:
        d, q = torch.linalg.eigh(mats[i].double())
        out[i] = (d.float(), q.float())


def _run_lane(stream: torch.cuda.Stream, jobs: list, stacks: dict, ts_sizes: set) -> list:
    with _lane_lock(stream), torch.cuda.stream(stream):
        return [_gpu_bucket(stacks[key], ts_sizes) for key, _ in jobs]


def _launch_jobs(
    gpu: list,
    stacks: dict,
    dev: torch.device,
    ts_sizes: set,
) -> dict[int, tuple[torch.Tensor, torch.Tensor]]:
    """Run the size buckets on the lanes and join them back into the
    current stream.  With chain members (the default for n > 128) the
    chains drive the schedule (``_launch_sytrd``); otherwise the buckets are
    spread over the lanes by LPT on n^3.  One host thread per lane: the
    native calls release the GIL, so the lanes' launches are enqueued
    concurrently (ResNet-50 mix: 410 ms with 8 threaded lanes vs 506-516 ms
    from one thread, profiles/eigh_lanes_mi355x.jsonl)."""
    main = torch.cuda.current_stream(dev)
    out: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
    chain_keys = {k for k, _ in gpu if _use_sytrd(k[0]) and not _use_twostage(k[0], ts_sizes)
                  and k[0] > JACOBI_MAX_N}
    ready = torch.cuda.Event()
    ready.record(main)
    if os.environ.get('KFAC_REFRESH_SYNC', '1') == '1':
        # The host is usually many steps ahead of the GPU (graph replays and
        # eager steps enqueue faster than they run; ~28 ResNet-50 steps, bounded
        # by the hardware queue's ring).  Lane work enqueued now would sit on
        # the other hardware queues behind a barrier on `ready` for all those
        # steps, and while it waits the queued steps ran 2.5x slower (13.3 ->
        # 33 ms per plain step for the 28 steps before every refresh: 1605
        # img/s over 300 steps vs 1979 with this wait, 1997 vs 1990 over 20;
        # profiles/r6/refresh_sync/).  So the lanes are issued once the
        # factors are ready on the GPU; the host has nothing better to do.
        ready.synchronize()
    streams = _side_streams(dev)
    big = [(k, v) for k, v in gpu if k in chain_keys]
    rest = [(k, v) for k, v in gpu if k not in chain_keys]
    if big:
        out.update(_launch_sytrd(big, rest, stacks, main, ready, streams, ts_sizes))
        return out
    jobs = sorted(rest, key=lambda j: -_bucket_cost(j[0][0], len(j[1])))
    # one lane per hardware queue: streams beyond GPU_MAX_HW_QUEUES share a
    # queue, and a lane queued behind another lane's long kernel (a two-stage
    # bulge chase runs for tens of ms on one CU) waits for all of it
    hwq = int(os.environ.get('GPU_MAX_HW_QUEUES', '4'))
    streams = streams[:max(1, min(len(streams), hwq))]
    lanes: list[list] = [[] for _ in streams]
    loads = [0.0] * len(streams)
    for job in jobs:
        k = loads.index(min(loads))
        loads[k] += _bucket_cost(job[0][0], len(job[1]))
        lanes[k].append(job)
    active = [(s, ln) for s, ln in zip(streams, lanes) if ln]
    for s, _ in active:
        s.wait_event(ready)
    if len(active) > 1 and _threads_enabled():
        pool = _executor(len(active))
        futs = [pool.submit(_run_lane, s, ln, stacks, ts_sizes) for s, ln in active]
        results = [f.result() for f in futs]
    else:
        results = [_run_lane(s, ln, stacks, ts_sizes) for s, ln in active]
    for (s, ln), res in zip(active, results):
        main.wait_stream(s)
        for (key, idxs), (evals, evecs) in zip(ln, res):
            # produced on a lane stream, consumed on the main stream
            evals.record_stream(main)
            evecs.record_stream(main)
            for k, i in enumerate(idxs):
                out[i] = (evals[k], evecs[k])
    return out


_lane_locks: dict[int, Any] = {}


def _lane_lock(stream: torch.cuda.Stream) -> Any:
    """One host thread at a time per lane: the rocSOLVER handle (and its
    workspace) is cached per stream and is not thread-safe."""
    import threading

    return _lane_locks.setdefault(stream.cuda_stream, threading.Lock())


def _tail_job(stream: torch.cuda.Stream, ev: torch.cuda.Event, red: torch.Tensor,
              d: torch.Tensor, e: torch.Tensor, tau: torch.Tensor
              ) -> tuple[torch.Tensor, torch.Tensor]:
    """Finish one reduced bucket on ``stream`` once the chain reached it:
    eigenpairs of T (native divide and conquer), then X = Q Z."""
    with _lane_lock(stream), torch.cuda.stream(stream):
        stream.wait_event(ev)
        for t in (red, d, e, tau):  # produced on the chain lane
            t.record_stream(stream)
        _tier('sytrd+dc', red.shape[-1], red.shape[0])
        n = d.shape[-1]
        w, z = native().tridiag_eigh_dc(d, e[:, :max(n - 1, 0)])
        return w, apply_q_blocked(red, tau, z)


def _chain_groups(keys: list) -> list[list]:
    """Split the sytrd-tier buckets into independent chains (one lane
    each) at the sizes in ``KFAC_SYTRD_SPLIT`` (comma-separated).  Each chain costs ~24 us
    of kernel-boundary latency per column of its largest matrix, so two
    chains on two hardware queues overlap each other's gaps, while the
    smaller matrices no longer add their symv traffic to the largest chain."""
    cuts = sorted((int(c) for c in os.environ.get('KFAC_SYTRD_SPLIT', '4000,1000').split(',')
                   if c), reverse=True)
    groups, left = [], list(keys)
    for c in cuts:
        groups.append([k for k in left if k[0] >= c])
        left = [k for k in left if k[0] < c]
    groups.append(left)
    return [g for g in groups if g]


def _chain_waves(group: int) -> int:
    """Waves each symv launch of chain ``group`` (0 = the largest) is sized
    to: ``KFAC_SYTRD_WAVES``, comma-separated per group, the last entry
    repeating; 0 = the whole chip (3 blocks per CU)."""
    vals = [int(v) for v in os.environ.get('KFAC_SYTRD_WAVES', '0').split(',') if v]
    return vals[min(group, len(vals) - 1)] if vals else 0


_chain_cache: dict[tuple, dict] = {}
_hi: list[torch.cuda.Stream] = []


def _hi_streams(device: torch.device) -> list[torch.cuda.Stream]:
    """High-priority lanes for the largest chain and its tail."""
    global _hi
    if not _hi or _hi[0].device != device:
        lo, hi_prio = torch.cuda.Stream.priority_range()
        _hi = [torch.cuda.Stream(device=device, priority=hi_prio) for _ in range(2)]
    return _hi


def _chain_graphs_enabled(group: int = 0) -> bool:
    """``KFAC_SYTRD_GRAPHS``: 0 (default: chains launched eagerly), 1 (every
    chain replays captured graphs) or first (only the largest chain).

    Replay enqueues a whole chain at once, so a lane that HIP maps onto the
    same hardware queue waits behind all of it; eager launches interleave.
    In the bench process (alternating runs, one box) replay gave 470 / 351 ms
    refresh steps, first 364 / 368, eager 353 / 360
    (profiles/sytrd_graphs_ab_r2.txt): the replay's host saving does not
    pay for the outlier risk."""
    mode = os.environ.get('KFAC_SYTRD_GRAPHS', '0')
    return mode == '1' or (mode == 'first' and group == 0)


def _chain_entry(sig: tuple, keys: list, stacks: dict, waves: int = 0) -> dict:
    """Persistent operands + one captured HIP graph per segment for a chain
    signature (the sizes and counts of its buckets), built on first use.

    A refresh is bound by the HOST's launch rate, not the GPU: ~45k kernel
    launches (the 4608 chain alone issues ~9.3k) complete only ~5 ms after
    the last one is enqueued (profiles/refresh_variance_r2.jsonl).  A
    replayed segment is one host call; the matrices are copied into the
    persistent operands first (a D2D copy)."""
    ent = _chain_cache.get(sig)
    if ent is not None:
        return ent
    lib = native()
    nb = int(lib.sytrd_nb())
    bufs = [torch.empty_like(stacks[k]) for k in keys]
    state = lib.sytrd_begin(bufs)
    sizes = [k[0] for k in keys for _ in range(stacks[k].shape[0])]
    graphs: list = []
    k0 = 0
    for key in keys:
        k1 = -(-key[0] // nb) * nb
        g = None
        if k1 > k0:
            g = torch.cuda.CUDAGraph()
            # no torch.cuda.graph(): its entry synchronises the device and
            # empties the cache while the other lanes are running
            g.capture_begin(capture_error_mode='thread_local')
            lib.sytrd_advance(state[0], sizes, k0, k1, waves)
            g.capture_end()
            k0 = k1
        graphs.append(g)
    ent = {'bufs': bufs, 'state': state, 'graphs': graphs}
    _chain_cache[sig] = ent
    return ent


def _run_chain(stream: torch.cuda.Stream, keys: list, stacks: dict,
               tail_lane: dict, pool: Any, group: int = 0) -> list:
    """Issue one chain (ascending n) in segments; after each bucket's last
    panel, hand that bucket's tail to its lane behind an event.  Segments
    replay from captured HIP graphs (``_chain_entry``; ``KFAC_SYTRD_GRAPHS=0``
    launches them eagerly)."""
    lib = native()
    nb = int(lib.sytrd_nb())
    keys = sorted(keys, key=lambda k: k[0])
    out = []
    waves = _chain_waves(group)
    with torch.cuda.stream(stream):
        if _chain_graphs_enabled(group):
            sig = (str(stream.device), tuple((k[0], stacks[k].shape[0]) for k in keys))
            ent = _chain_entry(sig + (waves,), keys, stacks, waves)
            for buf, k in zip(ent['bufs'], keys):
                buf.copy_(stacks[k])
            state, reds, graphs = ent['state'], ent['bufs'], ent['graphs']
        else:
            reds = [stacks[k] for k in keys]
            state = lib.sytrd_begin(reds)
            graphs = None
        descs = state[0]
        sizes = [k[0] for k in keys for _ in range(stacks[k].shape[0])]
        k0 = 0
        for j, key in enumerate(keys):
            if graphs is not None:
                if graphs[j] is not None:
                    graphs[j].replay()
            else:
                k1 = -(-key[0] // nb) * nb
                if k1 > k0:
                    lib.sytrd_advance(descs, sizes, k0, k1, waves)
                    k0 = k1
            ev = torch.cuda.Event()
            ev.record(stream)
            d, e, tau = state[2 + 3 * j:5 + 3 * j]
            args = (tail_lane[key], ev, reds[j], d, e, tau)
            out.append((key, pool.submit(_tail_job, *args) if pool else _tail_job(*args)))
        if graphs is None:
            for t in state[:2]:
                t.record_stream(stream)
        for k in keys:
            stacks[k].record_stream(stream)
    return out


def _launch_sytrd(
    big: list,
    rest: list,
    stacks: dict,
    main: torch.cuda.Stream,
    ready: torch.cuda.Event,
    streams: list[torch.cuda.Stream],
    ts_sizes: set,
) -> dict[int, tuple[torch.Tensor, torch.Tensor]]:
    """Large buckets: native tridiagonalisation chains (``_chain_groups``),
    one lane each, issued in segments that end where each bucket's size
    ends.  As soon as a segment is enqueued, an event marks it and that
    bucket's tail (native divide and conquer + back-transform, ``_tail_job``) is issued on
    another lane behind the event, so tails run while the chains are still
    reducing the larger factors.  The small buckets' syevd share the
    non-chain lanes.  Only as many lanes as the process has hardware queues
    (``GPU_MAX_HW_QUEUES``, HIP's default 4) are used: streams beyond that
    share a queue with a chain lane, and work queued behind a chain waits
    for it in order."""
    hwq = int(os.environ.get('GPU_MAX_HW_QUEUES', '4'))
    streams = streams[:max(2, min(len(streams), hwq))]
    for s in streams:
        s.wait_event(ready)
    groups = _chain_groups([k for k, _ in big])
    nchain = min(len(groups), len(streams) - 1)
    if nchain < len(groups):  # too few lanes: one chain
        groups = [sum(groups, [])]
        nchain = 1
    chains = streams[:nchain]
    others = streams[nchain:]
    hi = _hi_streams(streams[0].device)
    if hi:
        # the largest chain and its tail are the critical path: high-priority
        # queues get the CUs first, the other lanes fill in around them
        # (276 vs 301 ms on the step-100 ResNet-50 mix).  Giving the second
        # chain a high-priority lane as well measured worse (334 ms): the two
        # chains are both bandwidth-bound and slow each other down
        # (profiles/refresh_trace_r2.txt)
        for h in hi:
            h.wait_event(ready)
        chains = [hi[0]] + chains[1:]
    small_jobs = sorted(rest, key=lambda j: -_bucket_cost(j[0][0], len(j[1])))
    lanes: list[list] = [[] for _ in others]
    loads = [0.0] * len(others)
    for job in small_jobs:
        k = loads.index(min(loads))
        loads[k] += _bucket_cost(job[0][0], len(job[1]))
        lanes[k].append(job)
    tail_lane = {}
    for key in sorted((k for k, _ in big), key=lambda k: -_bucket_cost(
            k[0], stacks[k].shape[0])):
        k = loads.index(min(loads))
        loads[k] += _bucket_cost(key[0], stacks[key].shape[0]) / 4  # tail only
        tail_lane[key] = others[k]
    if hi:
        tail_lane[max(groups[0], key=lambda k: k[0])] = hi[1]
    threads = _threads_enabled()
    pool = _executor(len(others) + nchain + len(big)) if threads else None
    active = [(s, ln) for s, ln in zip(others, lanes) if ln]
    futs = [pool.submit(_run_lane, s, ln, stacks, ts_sizes) for s, ln in active] if pool else []
    cf = [pool.submit(_run_chain, c, g, stacks, tail_lane, pool, gi) if pool else
          _run_chain(c, g, stacks, tail_lane, None, gi)
          for gi, (c, g) in enumerate(zip(chains, groups))]
    results = [f.result() for f in futs] if pool else [
        _run_lane(s, ln, stacks, ts_sizes) for s, ln in active]
    tails = [(key, f.result() if pool else f)
             for key, f in sum((c.result() if pool else c for c in cf), [])]
    out: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
    for s in streams + hi:  # every lane's work is enqueued by now
        main.wait_stream(s)
    for (s, ln), res in zip(active, results):
        for (key, idxs), (evals, evecs) in zip(ln, res):
            evals.record_stream(main)
            evecs.record_stream(main)
            for k, i in enumerate(idxs):
                out[i] = (evals[k], evecs[k])
    idx_of = dict(big)
    for key, (evals, evecs) in tails:
        evals.record_stream(main)
        evecs.record_stream(main)
        for k, i in enumerate(idx_of[key]):
            out[i] = (evals[k], evecs[k])
    return out


def apply_q_blocked(red: torch.Tensor, tau: torch.Tensor, z: torch.Tensor,
                    nb: int = 512) -> torch.Tensor:
    """``Q Z`` for the reflectors the native tridiagonalisation left in
    ``red`` (reflector k in ROW k: v[k+1] = 1 implicit, v[k+2:] stored;
    Q = H_0 H_1 ... H_{n-2}, H_k = I - tau_k v_k v_k^T) -- the back-transform
    of the eigenvectors ``z`` of T (columns) into eigenvectors of A.

    rocSOLVER's ormtr applies the reflectors in 32-wide panels with ~10
    small kernels each; here ``nb`` reflectors form one UT block
    ``I - V T V^T`` with ``T = (striu(V^T V) + diag(1/tau))^-1`` (the
    identity behind LAPACK's larft), so each block costs three batched fp32
    GEMMs over every factor of the size at once and one small triangular
    solve.  Blocks run last to first; block p touches rows p+1..n-1 only.
    tau = 0 (nothing to annihilate: H = I) zeroes the reflector.  No host
    synchronisation.  Returns X [cnt, n, n], eigenvectors in columns."""
    c, n, _ = red.shape
    x = z.contiguous().clone() if z.is_contiguous() else z.contiguous()
    if n < 2:
        return x
    vt = torch.triu(red, diagonal=2)
    idx = torch.arange(n - 1, device=red.device)
    vt[:, idx, idx + 1] = 1.0
    live = (tau != 0).to(red.dtype)
    vt.mul_(live.unsqueeze(-1))
    lib = native() if red.is_cuda and red.dtype == torch.float32 else None
    if red.is_cuda and red.dtype == torch.float32 and lib is None:
        raise RuntimeError(f'native extension missing: {_native_error()}')
    eye = torch.eye(nb, device=red.device, dtype=red.dtype)
    for p in reversed(range(0, n - 1, nb)):
        q = min(p + nb, n - 1)
        b = q - p
        v = vt[:, p:q, p + 1:]  # [c, b, m]: V_b^T restricted to rows >= p+1
        t_ = tau[:, p:q]
        dinv = torch.where(t_ == 0, torch.ones_like(t_), 1.0 / torch.where(
            t_ == 0, torch.ones_like(t_), t_))
        xs = x[:, p + 1:, :]
        if lib is not None:
            # native fp32 MFMA GEMMs + blocked triangular inverse
            # (csrc/gemm_f32.hip): no library GEMM in the refresh
            g = torch.empty(c, b, b, device=red.device, dtype=red.dtype)
            lib.gemm_f32(v, v, g, False, True)
            tm = torch.triu(g, diagonal=1) + torch.diag_embed(dinv)
            lib.trinv_upper_(tm)
            y = torch.empty(c, b, n, device=red.device, dtype=red.dtype)
            lib.gemm_f32(v, xs, y, False, False)
            w = torch.empty_like(y)
            lib.gemm_f32(tm, y, w, False, False)
            lib.gemm_f32(v, w, xs, True, False, -1.0, 1.0)
            continue
        g = torch.bmm(v, v.transpose(1, 2))
        u = torch.triu(g, diagonal=1) + torch.diag_embed(dinv)
        tm = torch.linalg.solve_triangular(u, eye[:b, :b].expand(c, b, b), upper=True)
        w = torch.bmm(tm, torch.bmm(v, xs))
        xs.baddbmm_(v.transpose(1, 2), w, alpha=-1.0)
    return x


def _threads_enabled() -> bool:
    return os.environ.get('KFAC_EIGH_THREADS', '1') != '0'


_pool: Any = None


def _executor(n: int) -> Any:
    global _pool
    if _pool is None or _pool._max_workers < n:
        from concurrent.futures import ThreadPoolExecutor

        _pool = ThreadPoolExecutor(max_workers=n, thread_name_prefix='kfac-eigh')
    return _pool


def eigh(mat: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Single-matrix convenience wrapper around ``eigh_many``."""
    return eigh_many([mat])[0]


def inverse_many(mats: list[torch.Tensor], damping: float) -> list[torch.Tensor]:
    """``(F + damping I)^-1`` for every symmetric factor, fp32, batched by
    size (K-HIP-5, csrc/spdinv_chol.hip): blocked Cholesky, triangular
    inverse and W^T W on fp32 MFMA tiles, every factor of a size in one
    launch per block step; exactly symmetric results.

    Cholesky has LU's backward stability at half the flops (a Gauss-Jordan
    inverse without exchanges, tried in round 1, was 50x less accurate than
    fp32 LU on rank-deficient factors at the reference damping).

    Robustness: a factor whose Cholesky pivots fail (non-positive or
    non-finite), or whose result is not finite, is re-solved with a pivoted
    LU (``torch.linalg.inv``, the reference's routine) -- never installed as
    NaN.  That check costs one host read-back per size bucket per
    second-order update.  CPU tensors use the PyTorch math."""
    out: list[torch.Tensor | None] = [None] * len(mats)
    buckets: dict[tuple[int, torch.device], list[int]] = defaultdict(list)
    for i, m in enumerate(mats):
        buckets[(m.shape[0], m.device)].append(i)
    for (_, dev), idxs in buckets.items():
        n = mats[idxs[0]].shape[0]
        if dev.type == 'cuda' and use_native(mats[idxs[0]]):
            stack = torch.stack([mats[i].to(torch.float32) for i in idxs]).contiguous()
            # every Cholesky pivot positive and finite => finite result
            inv, fail = native().spd_inverse_blocked(stack, float(damping))
            bad = fail != 0
            failed = bad.nonzero().flatten().tolist()
            if failed:
                logger.warning('damped inverse: %d factor(s) of n=%d failed the '
                               'no-pivoting elimination; using LU', len(failed), n)
                for k in failed:
                    a = stack[k] + damping * torch.eye(n, device=dev, dtype=torch.float32)
                    x = torch.linalg.inv(a.double()).float()
                    inv[k] = 0.5 * (x + x.t())
            for k, i in enumerate(idxs):
                out[i] = inv[k]
        else:
            for i in idxs:
                out[i] = _damped_inverse_torch(mats[i], damping)
    return [o for o in out if o is not None]


def damped_inverse(mat: torch.Tensor, damping: float) -> torch.Tensor:
    """``(mat + damping*I)^-1`` computed in fp32 (reference inverse.py:
    185-212); single-matrix wrapper around ``inverse_many``."""
    return inverse_many([mat], damping)[0]


def _damped_inverse_torch(mat: torch.Tensor, damping: float) -> torch.Tensor:
    """PyTorch math (CPU): the damped factor is SPD, so a Cholesky
    factorisation plus ``cholesky_inverse`` replaces the general LU inverse
    (half the flops, no pivoting); if the factorisation fails (indefinite
    input) it falls back to ``torch.linalg.inv``."""
    a = mat.to(torch.float32)
    a = a + damping * torch.eye(a.shape[-1], dtype=a.dtype, device=a.device)
    chol, info = torch.linalg.cholesky_ex(a)
    if bool((info != 0).any()):
        return torch.linalg.inv(a)
    return torch.cholesky_inverse(chol)
