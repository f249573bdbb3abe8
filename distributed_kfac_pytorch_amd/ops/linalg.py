"""Second-order linear algebra: batched symmetric eigensolver and SPD inverse.

``eigh_many(mats)`` decomposes a list of symmetric fp32 matrices of mixed
sizes (all K-FAC factors a rank owns) with as little latency as possible:

* matrices are bucketed by size; each bucket is ONE batched call;
* n <= 64: the LDS-resident parallel Jacobi kernel (csrc/eigh_jacobi.hip),
  one matrix per workgroup;
* with ``KFAC_EIGH=sytrd``, n >= ``KFAC_SYTRD_MIN_N``: the native batched
  tridiagonalisation (csrc/sytrd.hip): every such factor of every bucket
  advances one column per launch pair in ONE chain, then each matrix is
  finished by rocSOLVER ``stedc`` + ``ormtr`` (the second half of syevd) on
  the lanes below.  Opt-in: on MI355X it is correct to ~1e-6 and its
  3 x 4608 chain now matches rocSOLVER's (164 vs 165 ms,
  profiles/sytrd_per_column_trace_r2.txt), but the refresh of the real
  step-100 ResNet-50 factors is still slower than the default (375 ms at
  n >= 4000, 411 ms at n >= 2000, vs 353 ms for warm-tested syevd:
  profiles/refresh_probe_r2_sytrd_tier.jsonl) -- the chain pays ~16 us of
  kernel-boundary floor per column, and its stedc + ormtr tail follows it;
* other n: direct batched rocSOLVER ``syevd`` calls from C++
  (csrc/solver.cpp) which, unlike ``torch.linalg.eigh``, never synchronise
  the host;
* the buckets run concurrently on a small pool of HIP streams (joined back
  into the caller's stream with events), so latency-bound small/medium
  decompositions overlap the bandwidth-bound large ones.

Results match ``torch.linalg.eigh``: ascending eigenvalues, eigenvectors in
columns.  Eigenvectors are unique only up to sign (and rotation inside
degenerate eigenspaces); K-FAC only uses them through ``Q f(D) Q^T``, which
is invariant to that freedom.

Environment knobs: ``KFAC_EIGH`` = auto | torch | syevd | syevj | syevdj
(force one algorithm for n > 64; sytrd = native tridiagonalisation tier),
``KFAC_SYTRD_MIN_N`` (smallest n for the sytrd tier), ``KFAC_EIGH_STREAMS`` (lanes, default 8),
``KFAC_EIGH_THREADS`` (0: issue every lane from the calling thread),
``KFAC_EIGH_SPLIT_N`` (factors at least this large are solved one per job),
``KFAC_JACOBI_SWEEPS`` / ``KFAC_JACOBI_TOL`` (small-n kernel).
"""
from __future__ import annotations

import logging
import os
from collections import defaultdict
from typing import Any

import torch

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native

JACOBI_SWEEPS = int(os.environ.get('KFAC_JACOBI_SWEEPS', '15'))
JACOBI_TOL = float(os.environ.get('KFAC_JACOBI_TOL', '1e-7'))
_ALGOS = {'syevd': 0, 'syevj': 1, 'syevdj': 2}
# n above which auto picks syevd over syevj (Jacobi sweeps are O(n^3) each)
# largest n sent to the LDS Jacobi kernel (its hard limit is jacobi_max_n())
JACOBI_MAX_N = int(os.environ.get('KFAC_JACOBI_MAX_N', '128'))


def sytrd_min_n() -> int:
    """Smallest factor dimension sent to the native tridiagonalisation."""
    return int(os.environ.get('KFAC_SYTRD_MIN_N', '512'))


logger = logging.getLogger(__name__)
_streams: list[torch.cuda.Stream] = []


def jacobi_max_n() -> int:
    lib = native()
    return int(lib.jacobi_max_n()) if lib is not None else 0


def _side_streams(device: torch.device) -> list[torch.cuda.Stream]:
    n = int(os.environ.get('KFAC_EIGH_STREAMS', '8'))
    global _streams
    if len(_streams) < n or _streams[0].device != device:
        _streams = [torch.cuda.Stream(device=device) for _ in range(n)]
    return _streams[:n]


def _algo_for(n: int) -> str:
    mode = os.environ.get('KFAC_EIGH', 'auto')
    if mode != 'auto':
        return mode
    # Measured on MI355X (tools/bench_eigh.py): batched syevd beats syevj /
    # syevdj at every size >= 128 and matches torch's eigh accuracy; the
    # native Jacobi kernel wins for n <= 64.
    return 'syevd'


def block_jacobi_enabled() -> bool:
    """Native warm-started block Jacobi (csrc/eigh_block.hip) for every
    factor above the LDS Jacobi tier (``KFAC_EIGH_BLOCK=0``: rocSOLVER)."""
    return os.environ.get('KFAC_EIGH_BLOCK', '1') != '0' and os.environ.get(
        'KFAC_EIGH', 'auto') == 'auto'


def cold_algo() -> str:
    """Solver for a factor with no previous eigenbasis (first refresh,
    checkpoint load): ``KFAC_EIGH_COLD`` = block | syevd."""
    return os.environ.get('KFAC_EIGH_COLD', 'block')


BJ_MAX_SWEEPS_WARM = int(os.environ.get('KFAC_BJ_SWEEPS', '10'))
BJ_MAX_SWEEPS_COLD = int(os.environ.get('KFAC_BJ_SWEEPS_COLD', '20'))
BJ_TOL = float(os.environ.get('KFAC_BJ_TOL', '1e-6'))
BJ_INNER = int(os.environ.get('KFAC_BJ_INNER', '2'))
BJ_NOISE = float(os.environ.get('KFAC_BJ_NOISE', '4e-6'))
BJ_REFINE = os.environ.get('KFAC_BJ_REFINE', '1') != '0'
# per-call statistics of the block-Jacobi tier (bench / tests read them)
last_stats: dict[str, Any] = {}


def _block_jacobi(stack: torch.Tensor, warm: torch.Tensor | None) -> tuple[torch.Tensor, torch.Tensor]:
    lib = native()
    sweeps_max = BJ_MAX_SWEEPS_WARM if warm is not None else BJ_MAX_SWEEPS_COLD
    evals, evecs, sweeps, _ = lib.block_jacobi_eigh(
        stack.contiguous(), warm, sweeps_max, BJ_TOL, BJ_INNER, BJ_NOISE, BJ_REFINE)
    sw = sweeps.tolist()  # host tensor: the solver already synchronised
    n = stack.shape[-1]
    last_stats.setdefault('sweeps', []).extend((n, s) for s in sw)
    bad = [i for i, s in enumerate(sw) if s < 0]
    if bad:
        # not converged within the sweep budget: rocSOLVER for those
        logger.warning('block Jacobi did not converge for %d factor(s) of n=%d; '
                       'using syevd', len(bad), n)
        idx = torch.tensor(bad, device=stack.device)
        e2, v2 = lib.rocsolver_eigh(stack.index_select(0, idx).contiguous(), 0, 100, 1e-7)
        evals = evals.clone()
        evecs = evecs.clone()
        evals.index_copy_(0, idx, e2)
        evecs.index_copy_(0, idx, v2.contiguous())
    return evals, evecs


WARM_ACCEPT_TOL = float(os.environ.get('KFAC_EIGH_ACCEPT_TOL', '1e-6'))
# the acceptance GEMM sits on the critical path of a lane: the largest
# (A) factors essentially never pass, so they go straight to the solver
WARM_ACCEPT_MAX_N = int(os.environ.get('KFAC_EIGH_ACCEPT_MAX_N', '2048'))


def _accept_warm(stack: torch.Tensor, warm: torch.Tensor
                 ) -> tuple[list[int], torch.Tensor, torch.Tensor]:
    """Factors the previous eigenbasis still diagonalises.

    With Q0 the previous basis, the Rayleigh quotients r = diag(Q0^T A Q0)
    and the residual ||A Q0 - Q0 diag(r)||_F = off(Q0^T A Q0)_F cost ONE
    batched GEMM; a factor whose residual is below KFAC_EIGH_ACCEPT_TOL *
    ||A||_F (the block-Jacobi convergence test: no rotation would be
    applied) keeps Q0 with the fresh eigenvalues r.  On real ResNet-50
    factors about a third of the factors (most G factors) pass at the
    step-100 refresh (profiles/refresh_probe_r2_resnet50_step100.jsonl).
    Returns (accepted indices, their sorted evals, their evecs)."""
    aq = torch.bmm(stack, warm)
    r = (warm * aq).sum(1)
    res = (aq - warm * r.unsqueeze(1)).flatten(1).norm(dim=1)
    fro = stack.flatten(1).norm(dim=1)
    ok = (res <= WARM_ACCEPT_TOL * fro).tolist()
    idx = [i for i, v in enumerate(ok) if v]
    if not idx:
        return [], r[:0], warm[:0]
    sel = torch.tensor(idx, device=stack.device)
    rs, order = r.index_select(0, sel).sort(dim=1)
    q = warm.index_select(0, sel)
    q = q.gather(2, order.unsqueeze(1).expand(-1, q.shape[1], -1))
    return idx, rs, q


def large_algo() -> str:
    """Solver for factors above the LDS Jacobi tier that the warm-start
    acceptance test did not settle: ``KFAC_EIGH_LARGE`` = syevd | block.

    Default syevd: on the real ResNet-50 step-100 refresh the native block
    Jacobi (warm) needs 6-12 sweeps on the large A factors (the step-0
    basis of a rank-deficient early factor is a poor start) and the mix
    takes 1002 ms against 395 ms for syevd at equal accuracy
    (profiles/refresh_probe_r2_resnet50_step100.jsonl)."""
    return os.environ.get('KFAC_EIGH_LARGE', 'syevd')


def _large_bucket(stack: torch.Tensor, warm: torch.Tensor | None
                  ) -> tuple[torch.Tensor, torch.Tensor]:
    n = stack.shape[-1]
    if block_jacobi_enabled() and (
        large_algo() == 'block' and (warm is not None or cold_algo() == 'block')
    ):
        return _block_jacobi(stack, warm)
    algo = _algo_for(n)
    if algo in ('sytrd', 'auto'):
        algo = 'syevd'
    if algo == 'torch':
        return torch.linalg.eigh(stack)
    evals, evecs = native().rocsolver_eigh(stack.contiguous(), _ALGOS[algo], 100, 1e-7)
    return evals, evecs


def _gpu_bucket(stack: torch.Tensor, warm: torch.Tensor | None = None
                ) -> tuple[torch.Tensor, torch.Tensor]:
    n = stack.shape[-1]
    lib = native()
    if n <= JACOBI_MAX_N:
        return lib.jacobi_eigh(stack.contiguous(), JACOBI_SWEEPS, JACOBI_TOL)
    if warm is not None and block_jacobi_enabled() and n <= WARM_ACCEPT_MAX_N:
        idx, r, q = _accept_warm(stack, warm)
        last_stats.setdefault('accepted', []).extend([n] * len(idx))
        if len(idx) == stack.shape[0]:
            return r, q
        if idx:
            rest = [i for i in range(stack.shape[0]) if i not in set(idx)]
            sel = torch.tensor(rest, device=stack.device)
            e2, v2 = _large_bucket(stack.index_select(0, sel).contiguous(),
                                   warm.index_select(0, sel).contiguous())
            evals = torch.empty(stack.shape[:2], dtype=e2.dtype, device=stack.device)
            evecs = torch.empty_like(stack)
            evals.index_copy_(0, torch.tensor(idx, device=stack.device), r)
            evecs.index_copy_(0, torch.tensor(idx, device=stack.device), q)
            evals.index_copy_(0, sel, e2)
            evecs.index_copy_(0, sel, v2.contiguous())
            return evals, evecs
    return _large_bucket(stack, warm)


def _bucket_cost(n: int, count: int) -> float:
    return float(count) * float(n) ** 3


def eigh_many(
    mats: list[torch.Tensor],
    warm: list[torch.Tensor | None] | None = None,
) -> list[tuple[torch.Tensor, torch.Tensor]]:
    """Eigendecompose each symmetric matrix; returns ``[(evals, evecs)]``.

    ``warm[i]``, when given, is a previous eigenbasis of ``mats[i]``'s factor
    (eigenvectors in columns); the block-Jacobi tier starts from it.  Size
    buckets are split into warm and cold sub-buckets."""
    out: list[tuple[torch.Tensor, torch.Tensor] | None] = [None] * len(mats)
    buckets: dict[tuple, list[int]] = defaultdict(list)
    for i, m in enumerate(mats):
        w = warm[i] if warm is not None else None
        ok = (
            w is not None and isinstance(w, torch.Tensor) and w.shape == m.shape
            and w.dtype == torch.float32 and w.device == m.device
        )
        if warm is not None and not ok and w is not None:
            warm[i] = None
        buckets[(m.shape[0], m.device, bool(ok))].append(i)
    gpu = [(k, v) for k, v in buckets.items() if k[1].type == 'cuda']
    cpu = [(k, v) for k, v in buckets.items() if k[1].type != 'cuda']
    for (n, _, _), idxs in cpu:
        stack = torch.stack([mats[i].to(torch.float32) for i in idxs])
        evals, evecs = torch.linalg.eigh(stack)
        for k, i in enumerate(idxs):
            out[i] = (evals[k], evecs[k])
    if gpu:
        dev = gpu[0][0][1]
        if not use_native(*[mats[idxs[0]] for _, idxs in gpu]):
            for key, idxs in gpu:
                evals, evecs = torch.linalg.eigh(
                    torch.stack([mats[i].to(torch.float32) for i in idxs]))
                for k, i in enumerate(idxs):
                    out[i] = (evals[k], evecs[k])
        else:
            stacks = {
                key: torch.stack([mats[i].to(torch.float32) for i in idxs])
                for key, idxs in gpu
            }
            warms = {
                key: torch.stack([warm[i] for i in idxs])  # type: ignore[index]
                for key, idxs in gpu if key[2]
            }
            for i, r in _launch_jobs(gpu, stacks, dev, warms).items():
                out[i] = r
    return [o for o in out if o is not None]


def _use_sytrd(n: int) -> bool:
    if os.environ.get('KFAC_EIGH', 'auto') != 'sytrd' or n < sytrd_min_n():
        return False
    lib = native()
    return lib is not None and n <= int(lib.sytrd_max_n())


def _jobs(gpu: list) -> list[tuple[tuple, list[int], int, int]]:
    """Split the size buckets into solver jobs ``(key, idxs, lo, hi)``.
    By default every bucket is one batched call: rocSOLVER's strided-batched
    kernels cover all matrices of a bucket per launch, which measured faster
    than one job per matrix even with threaded lanes (ResNet-50 mix on
    MI355X: 410 ms batched vs 564 ms split at n >= 1024, 8 lanes).  Factors
    with n >= ``KFAC_EIGH_SPLIT_N`` become one job each."""
    split_n = int(os.environ.get('KFAC_EIGH_SPLIT_N', '1000000'))
    jobs = []
    for key, idxs in gpu:
        if key[0] >= split_n and key[0] > JACOBI_MAX_N:
            jobs += [(key, idxs, k, k + 1) for k in range(len(idxs))]
        else:
            jobs.append((key, idxs, 0, len(idxs)))
    return jobs


def _run_lane(stream: torch.cuda.Stream, jobs: list, stacks: dict,
              warms: dict | None = None) -> list:
    with torch.cuda.stream(stream):
        res = []
        for key, _, lo, hi in jobs:
            w = warms.get(key) if warms else None
            res.append(_gpu_bucket(stacks[key][lo:hi], None if w is None else w[lo:hi]))
        return res


def _launch_jobs(
    gpu: list,
    stacks: dict,
    dev: torch.device,
    warms: dict | None = None,
) -> dict[int, tuple[torch.Tensor, torch.Tensor]]:
    """Run the solver jobs on ``KFAC_EIGH_STREAMS`` lanes (LPT on n^3), one
    host thread per lane, and join the lanes back into the current stream.

    rocSOLVER's syevd is a one-stage tridiagonalisation that issues ~5 tiny
    kernels per column (~22k launches and ~110 ms of dependent small kernels
    for n = 4608: profiles/rocprof_eigh4608_syevd_stats.csv).  Issued from
    one thread the call is bound by host enqueue rate, so buckets on
    different streams barely overlap (ResNet-50 mix: 4 streams 530 ms vs 1
    stream 573 ms).  The native call releases the GIL, so one thread per
    lane enqueues the independent chains concurrently and the GPU runs them
    side by side.  Measured on the ResNet-50 mix (tools/eigh_lanes_probe.py,
    profiles/eigh_lanes_mi355x.jsonl): 410 ms with 8 threaded lanes vs
    506-516 ms from one thread on one box, 412 vs 419 ms on another -- the
    floor is the 3 x 4608 bucket alone (242 ms).

    HIP graphs do not remove this bound: syevd fails under stream capture
    (it synchronises the host internally), and its stages captured one by
    one (sytrd, then stedc + ormtr; possible only with rocBLAS's hipBLASLt
    backend disabled) replay no faster than they run eagerly (3 x 4608:
    sytrd 165 ms eager / 169 ms replayed; profiles/
    eigh_rocsolver_stages_capture.jsonl) -- the reduction is a chain of
    dependent tiny kernels on the GPU as well.
    """
    main = torch.cuda.current_stream(dev)
    ready = torch.cuda.Event()
    ready.record(main)
    streams = _side_streams(dev)
    big = [(k, v) for k, v in gpu if _use_sytrd(k[0])]
    rest = [(k, v) for k, v in gpu if not _use_sytrd(k[0])]
    out: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
    if big:
        out.update(_launch_sytrd(big, rest, stacks, main, ready, streams))
        return out
    jobs = sorted(_jobs(gpu), key=lambda j: -_bucket_cost(j[0][0], j[3] - j[2]))
    lanes: list[list] = [[] for _ in streams]
    loads = [0.0] * len(streams)
    for job in jobs:
        k = loads.index(min(loads))
        loads[k] += _bucket_cost(job[0][0], job[3] - job[2])
        lanes[k].append(job)
    active = [(s, ln) for s, ln in zip(streams, lanes) if ln]
    for s, _ in active:
        s.wait_event(ready)
    if len(active) > 1 and _threads_enabled():
        pool = _executor(len(active))
        futs = [pool.submit(_run_lane, s, ln, stacks, warms) for s, ln in active]
        results = [f.result() for f in futs]
    else:
        results = [_run_lane(s, ln, stacks, warms) for s, ln in active]
    for (s, ln), res in zip(active, results):
        main.wait_stream(s)
        for (key, idxs, lo, hi), (evals, evecs) in zip(ln, res):
            # produced on a lane stream, consumed on the main stream
            evals.record_stream(main)
            evecs.record_stream(main)
            for k in range(hi - lo):
                out[idxs[lo + k]] = (evals[k], evecs[k])
    return out


def _sytrd_lane(stream: torch.cuda.Stream, keys: list, stacks: dict) -> list:
    with torch.cuda.stream(stream):
        return native().sytrd_reduce([stacks[k] for k in keys])


def _tridiag_lane(stream: torch.cuda.Stream, jobs: list, stacks: dict,
                  red: dict) -> list:
    with torch.cuda.stream(stream):
        res = []
        for key, _, lo, hi in jobs:
            d, e, tau = red[key]
            for t in (d, e, tau):  # allocated on lane 0, read here
                t.record_stream(stream)
            res.append(native().tridiag_eigvecs(
                stacks[key][lo:hi], d[lo:hi], e[lo:hi], tau[lo:hi]))
        return res


def _launch_sytrd(
    big: list,
    rest: list,
    stacks: dict,
    main: torch.cuda.Stream,
    ready: torch.cuda.Event,
    streams: list[torch.cuda.Stream],
) -> dict[int, tuple[torch.Tensor, torch.Tensor]]:
    """Large buckets: ONE native tridiagonalisation chain on lane 0 while the
    other lanes run the small buckets' syevd; then every large matrix is
    finished (stedc + ormtr) as its own job, LPT over all lanes."""
    for s in streams:
        s.wait_event(ready)
    keys = [k for k, _ in big]
    small_jobs = sorted(_jobs(rest), key=lambda j: -_bucket_cost(j[0][0], j[3] - j[2]))
    lanes: list[list] = [[] for _ in streams[1:]]
    loads = [0.0] * len(lanes)
    for job in small_jobs:
        k = loads.index(min(loads))
        loads[k] += _bucket_cost(job[0][0], job[3] - job[2])
        lanes[k].append(job)
    active = [(s, ln) for s, ln in zip(streams[1:], lanes) if ln]
    if _threads_enabled() and active:
        pool = _executor(len(active) + 1)
        fut_red = pool.submit(_sytrd_lane, streams[0], keys, stacks)
        futs = [pool.submit(_run_lane, s, ln, stacks) for s, ln in active]
        flat = fut_red.result()
        results = [f.result() for f in futs]
    else:
        flat = _sytrd_lane(streams[0], keys, stacks)
        results = [_run_lane(s, ln, stacks) for s, ln in active]
    red = {k: tuple(flat[3 * i:3 * i + 3]) for i, k in enumerate(keys)}
    reduced = torch.cuda.Event()
    reduced.record(streams[0])
    # phase 2: per-matrix stedc + ormtr jobs over every lane
    tjobs = [(key, idxs, b, b + 1) for key, idxs in big for b in range(len(idxs))]
    tjobs.sort(key=lambda j: -_bucket_cost(j[0][0], 1))
    tl: list[list] = [[] for _ in streams]
    tload = [0.0] * len(streams)
    for job in tjobs:
        k = tload.index(min(tload))
        tload[k] += _bucket_cost(job[0][0], 1)
        tl[k].append(job)
    tactive = [(s, ln) for s, ln in zip(streams, tl) if ln]
    for s, _ in tactive:
        s.wait_event(reduced)
    if _threads_enabled() and len(tactive) > 1:
        pool = _executor(len(tactive))
        tf = [pool.submit(_tridiag_lane, s, ln, stacks, red) for s, ln in tactive]
        tres = [f.result() for f in tf]
    else:
        tres = [_tridiag_lane(s, ln, stacks, red) for s, ln in tactive]
    out: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
    for (s, ln), res in list(zip(active, results)) + list(zip(tactive, tres)):
        main.wait_stream(s)
        for (key, idxs, lo, hi), (evals, evecs) in zip(ln, res):
            evals.record_stream(main)
            evecs.record_stream(main)
            for k in range(hi - lo):
                out[idxs[lo + k]] = (evals[k], evecs[k])
    for k in keys:
        stacks[k].record_stream(streams[0])
    return out


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

    Gauss-Jordan without exchanges (the one-workgroup LDS kernel,
    csrc/spdinv.hip, still available with ``KFAC_SPD_SMALL=gj``) was 50x
    less accurate than fp32 LU on rank-deficient factors at the reference
    damping -- the cause of the INVERSE-method divergence on ResNet-32 --
    while Cholesky has LU's backward stability at half the flops.

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
            if os.environ.get('KFAC_SPD_SMALL', 'chol') == 'gj' and n <= int(
                    native().spd_lds_max_n()):
                inv = native().spd_inverse(stack, float(damping))
                bad = ~torch.isfinite(inv).flatten(1).all(dim=1)
            else:
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
