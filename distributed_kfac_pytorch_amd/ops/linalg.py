"""Second-order linear algebra: batched symmetric eigensolver and SPD inverse.

``eigh_many(mats)`` decomposes a list of symmetric fp32 matrices of mixed
sizes (all K-FAC factors a rank owns) with as little latency as possible:

* matrices are bucketed by size; each bucket is ONE batched call;
* n <= 128: the LDS-resident parallel Jacobi kernel (csrc/eigh_jacobi.hip),
  one matrix per workgroup;
* a warm bucket (previous eigenbasis available, 128 < n <= 2048, not a
  chain member) first takes the acceptance test: factors the old basis
  still diagonalises to 1e-6 keep it with fresh eigenvalues;
* n >= ``KFAC_SYTRD_MIN_N`` (2000) in buckets of at most
  ``KFAC_SYTRD_MAX_BATCH`` (8) factors (default tier,
  ``KFAC_EIGH_LARGE=sytrd``): the native batched tridiagonalisation
  (csrc/sytrd.hip).  The factors are
  grouped into chains by size (``KFAC_SYTRD_SPLIT``, default: n >= 4000 and
  the rest), each chain on its own lane advancing every member one column
  per launch pair; a chain is issued in segments ending where each bucket
  ends, so the bucket's tail -- rocSOLVER ``stedc`` on T, then the blocked
  UT back-transform ``apply_q_blocked`` (3 batched fp32 GEMMs per 512
  reflectors; 4-8x faster than rocSOLVER ``ormtr``: 3 x 4608 in 11 vs
  39 ms, profiles/tail_probe_r2.jsonl) -- runs on another lane while the
  chain continues.  The largest chain and its tail run on high-priority
  lanes.  Real step-100 ResNet-50 refresh: 276 ms vs 329-361 ms for syevd
  (profiles/refresh_probe_r2_chains.jsonl, profiles/refresh_trace_r2.txt);
  every result is checked for finiteness once per refresh
  (``_repair_nonfinite``); splitting the largest bucket's tail into one
  factor per high-priority lane measured slower (336 ms: the tails are host-
  and GIL-bound, profiles/tail_split_negative_r2.txt);
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
``KFAC_EIGH_LARGE`` (sytrd | syevd | block), ``KFAC_SYTRD_MIN_N`` (smallest n
for the sytrd tier), ``KFAC_SYTRD_SPLIT`` (chain boundaries),
``KFAC_EIGH_ORMTR`` (blocked | rocsolver), ``KFAC_EIGH_STREAMS`` (lanes, default 8),
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

from distributed_kfac_pytorch_amd.ops import twostage
from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native

JACOBI_SWEEPS = int(os.environ.get('KFAC_JACOBI_SWEEPS', '15'))
JACOBI_TOL = float(os.environ.get('KFAC_JACOBI_TOL', '1e-7'))
_ALGOS = {'syevd': 0, 'syevj': 1, 'syevdj': 2}
# n above which auto picks syevd over syevj (Jacobi sweeps are O(n^3) each)
# largest n sent to the LDS Jacobi kernel (its hard limit is jacobi_max_n())
JACOBI_MAX_N = int(os.environ.get('KFAC_JACOBI_MAX_N', '128'))


def sytrd_min_n() -> int:
    """Smallest factor dimension sent to the native tridiagonalisation
    (every factor above the LDS Jacobi tier by default: no rocSOLVER
    eigensolver runs in a refresh)."""
    return int(os.environ.get('KFAC_SYTRD_MIN_N', str(JACOBI_MAX_N + 1)))


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
# Warm-basis acceptance (reuse the previous eigenbasis when it still
# diagonalises the new factor to KFAC_EIGH_ACCEPT_TOL) for n <= this; off by
# default: its batched Q^T A Q GEMMs and host read-back sit on the lanes'
# critical path, and the ResNet-50 refresh step was faster and steadier
# without it (248 / 253 ms vs 328 / 277 ms with n <= 2048, alternating
# runs: profiles/refresh_accept_r3.txt) -- every factor is then solved
# afresh, as the reference's torch.linalg.eigh does
WARM_ACCEPT_MAX_N = int(os.environ.get('KFAC_EIGH_ACCEPT_MAX_N', '0'))


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


def twostage_min_n() -> int:
    """Smallest factor the auto tier sends to the two-stage solver
    (``KFAC_TWOSTAGE_MIN_N``; default: none).  Measured on the ResNet-50
    step-100 refresh (gpurun_out r3z, one box): chains only 246 ms, two-stage
    for the 3 x 4608 bucket + chains below 307 ms, two-stage for everything
    409 ms -- at these sizes f32 MFMA runs at the f32 VALU rate, so the
    two-stage's 2.5x back-transform flops and its one-workgroup bulge chase
    (69 ms at n = 4608) do not pay for the level-3 stage 1 yet
    (profiles/twostage_r3.md)."""
    return int(os.environ.get('KFAC_TWOSTAGE_MIN_N', str(1 << 30)))


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


# sizes routed to the two-stage solver by bucket population (set per call of
# eigh_many, read by every tier decision of that call)
_TS_BATCH_SIZES: set = set()


def _use_twostage(n: int) -> bool:
    """Native two-stage solver (ops/twostage.py) for this factor size."""
    mode = os.environ.get('KFAC_EIGH', 'auto')
    if mode not in ('auto', 'twostage'):
        return False
    if not JACOBI_MAX_N < n <= twostage.max_n():
        return False
    if mode == 'twostage' or large_algo() == 'twostage':
        return True
    return large_algo() == 'sytrd' and (n >= twostage_min_n() or n in _TS_BATCH_SIZES)


def large_algo() -> str:
    """Solver for factors above the LDS Jacobi tier that the warm-start
    acceptance test did not settle: ``KFAC_EIGH_LARGE`` = sytrd (default:
    one-stage native chains, with factors of ``KFAC_TWOSTAGE_MIN_N`` and more
    on the two-stage solver -- dense -> band -> tridiagonal with a level-3
    stage 1, bulge chasing, native divide and conquer and blocked
    back-transforms, ops/twostage.py) | twostage (every factor) | syevd |
    block.

    Default sytrd: factors with n >= ``KFAC_SYTRD_MIN_N`` (2000) go through
    the native tridiagonalisation chains with the blocked back-transform,
    the rest through batched syevd on the other lanes -- the real ResNet-50
    step-100 refresh takes 276-290 ms against 329-361 ms with syevd alone
    (profiles/refresh_probe_r2_chains.jsonl).  (The non-finite gradients
    seen after a refresh with whole-step HIP graphs occur with syevd too:
    profiles/graph_replay_nonfinite_r2.txt.)

    block: on the real ResNet-50 step-100 refresh the native block
    Jacobi (warm) needs 6-12 sweeps on the large A factors (the step-0
    basis of a rank-deficient early factor is a poor start) and the mix
    takes 1002 ms against 395 ms for syevd at equal accuracy
    (profiles/refresh_probe_r2_resnet50_step100.jsonl)."""
    return os.environ.get('KFAC_EIGH_LARGE', 'sytrd')


def _large_bucket(stack: torch.Tensor, warm: torch.Tensor | None
                  ) -> tuple[torch.Tensor, torch.Tensor]:
    n = stack.shape[-1]
    if _use_twostage(n):
        _tier('twostage', n, stack.shape[0])
        if twostage.graphs_enabled():
            return twostage.eigh_twostage_graphed(stack)
        w, x, _, _ = twostage.eigh_twostage(stack)
        return w, x
    if block_jacobi_enabled() and (
        large_algo() == 'block' and (warm is not None or cold_algo() == 'block')
    ):
        return _block_jacobi(stack, warm)
    algo = _algo_for(n)
    if algo in ('sytrd', 'auto'):
        algo = 'syevd'
    _tier(algo, n, stack.shape[0])
    if algo == 'torch':
        return torch.linalg.eigh(stack)
    evals, evecs = native().rocsolver_eigh(stack.contiguous(), _ALGOS[algo], 100, 1e-7)
    return evals, evecs


def _tier(name: str, n: int, count: int) -> None:
    """Record which solver handled a bucket (``last_stats['tiers']``)."""
    last_stats.setdefault('tiers', []).append((name, int(n), int(count)))


def _gpu_bucket(stack: torch.Tensor, warm: torch.Tensor | None = None
                ) -> tuple[torch.Tensor, torch.Tensor]:
    n = stack.shape[-1]
    lib = native()
    if n <= JACOBI_MAX_N:
        _tier('jacobi', n, stack.shape[0])
        return lib.jacobi_eigh(stack.contiguous(), JACOBI_SWEEPS, JACOBI_TOL)
    # the two-stage tier needs no warm start: the acceptance test's host
    # read-back would cost more than the solves it saves
    if (warm is not None and block_jacobi_enabled() and n <= WARM_ACCEPT_MAX_N
            and not _use_twostage(n)):
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
            counts: dict[int, int] = defaultdict(int)
            for key, idxs in gpu:
                counts[key[0]] += len(idxs)
            _TS_BATCH_SIZES.clear()
            _TS_BATCH_SIZES.update(twostage_sizes(counts))
            stacks = {
                key: torch.stack([mats[i].to(torch.float32) for i in idxs])
                for key, idxs in gpu
            }
            warms = {
                key: torch.stack([warm[i] for i in idxs])  # type: ignore[index]
                for key, idxs in gpu if key[2]
            }
            res = _launch_jobs(gpu, stacks, dev, warms)
            for i, r in res.items():
                out[i] = r
            _repair_nonfinite(mats, out, list(res))
    return [o for o in out if o is not None]


def _repair_nonfinite(mats: list[torch.Tensor], out: list, idxs: list[int]) -> None:
    """A failed solve must never be installed silently: rocSOLVER reports
    divide-and-conquer failures only in a device ``info`` flag, which the
    host never reads.  One fused finiteness check over every result (one
    host read-back per refresh, which is already synchronised by the warm
    acceptance test); a non-finite factor is re-solved by torch's float64
    eigh (the reference's routine, kfac/layers/eigen.py:294-347) and logged.
    ``KFAC_EIGH_CHECK=0`` skips the check."""
    if not idxs or os.environ.get('KFAC_EIGH_CHECK', '1') == '0':
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


def _settle_warm(gpu: list, stacks: dict, warms: dict, out: dict) -> list:
    """Warm-start acceptance (``_accept_warm``'s test) for every warm bucket
    the sytrd tier would otherwise reduce, with ONE host read-back for all
    of them: accepted factors keep their previous basis (eigenvalues are
    the fresh Rayleigh quotients) and leave the bucket."""
    # chain members are not candidates: a fixed chain membership keeps its
    # captured graphs (one per signature) valid from refresh to refresh
    cand = [(k, v) for k, v in gpu if k[2] and k in warms and JACOBI_MAX_N < k[0]
            <= WARM_ACCEPT_MAX_N and not (_use_sytrd(k[0], len(v)) and _chain_graphs_enabled())
            and block_jacobi_enabled_for_sytrd()]
    if not cand:
        return gpu
    flags, stats = [], []
    for key, _ in cand:
        st, w = stacks[key], warms[key]
        aq = torch.bmm(st, w)
        r = (w * aq).sum(1)
        res = (aq - w * r.unsqueeze(1)).flatten(1).norm(dim=1)
        flags.append(res <= WARM_ACCEPT_TOL * st.flatten(1).norm(dim=1))
        stats.append(r)
    ok_all = torch.cat(flags).tolist()
    new_gpu, pos = [], 0
    cand_keys = {k for k, _ in cand}
    for key, idxs in gpu:
        if key not in cand_keys:
            new_gpu.append((key, idxs))
            continue
        j = [k for k, _ in cand].index(key)
        ok = ok_all[pos:pos + len(idxs)]
        pos += len(idxs)
        acc = [i for i, v in enumerate(ok) if v]
        last_stats.setdefault('accepted', []).extend([key[0]] * len(acc))
        if acc:
            _tier('accepted', key[0], len(acc))
        if acc:
            sel = torch.tensor(acc, device=stacks[key].device)
            rs, order = stats[j].index_select(0, sel).sort(dim=1)
            q = warms[key].index_select(0, sel)
            q = q.gather(2, order.unsqueeze(1).expand(-1, q.shape[1], -1))
            for t, i in enumerate(acc):
                out[idxs[i]] = (rs[t], q[t])
        keep = [i for i, v in enumerate(ok) if not v]
        if not keep:
            continue
        if acc:
            sel = torch.tensor(keep, device=stacks[key].device)
            stacks[key] = stacks[key].index_select(0, sel).contiguous()
            warms[key] = warms[key].index_select(0, sel).contiguous()
            idxs = [idxs[i] for i in keep]
        new_gpu.append((key, idxs))
    return new_gpu


def block_jacobi_enabled_for_sytrd() -> bool:
    """Warm acceptance in front of the sytrd tier (``KFAC_EIGH_BLOCK=0``
    turns it off, as for the block-Jacobi tier)."""
    return os.environ.get('KFAC_EIGH_BLOCK', '1') != '0'


def _use_sytrd(n: int, count: int = 1) -> bool:
    """Native tier for a bucket of ``count`` factors of size n.

    Buckets of more than ``KFAC_SYTRD_MAX_BATCH`` (8) factors stay on syevd:
    the chain's symv streams the FULL square of every member per column
    (rocSOLVER's reads one triangle), so it wins where the refresh is
    latency-bound -- a few large factors, ResNet-50: 3 x 4608, 6 x 2304,
    7 x 2048 -- and loses where it is bandwidth-bound: GPT-NeoX-125M's
    12 x 3073 + 12 x 3072 + 12 x 2304 refresh took 947 ms in one chain vs
    737 ms on syevd (profiles/neox_sytrd_vs_syevd_r2.txt)."""
    mode = os.environ.get('KFAC_EIGH', 'auto')
    on = mode == 'sytrd' or (mode == 'auto' and large_algo() == 'sytrd')
    if not on or n < sytrd_min_n():
        return False
    if mode == 'auto' and count > int(os.environ.get('KFAC_SYTRD_MAX_BATCH', '1000000')):
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
    with _lane_lock(stream), torch.cuda.stream(stream):
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
    out: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
    # chain membership is decided on the full buckets (before acceptance);
    # two-stage buckets run as ordinary lane jobs beside the chains
    chain_keys = {k for k, v in gpu if _use_sytrd(k[0], len(v)) and not _use_twostage(k[0])}
    if warms and chain_keys:
        gpu = _settle_warm(gpu, stacks, warms, out)
    ready = torch.cuda.Event()
    ready.record(main)
    streams = _side_streams(dev)
    big = [(k, v) for k, v in gpu if k in chain_keys]
    rest = [(k, v) for k, v in gpu if k not in chain_keys]
    if big:
        out.update(_launch_sytrd(big, rest, stacks, main, ready, streams))
        return out
    jobs = sorted(_jobs(gpu), key=lambda j: -_bucket_cost(j[0][0], j[3] - j[2]))
    # one lane per hardware queue: streams beyond GPU_MAX_HW_QUEUES share a
    # queue, and a lane queued behind another lane's long kernel (a two-stage
    # bulge chase runs for tens of ms on one CU) waits for all of it
    hwq = int(os.environ.get('GPU_MAX_HW_QUEUES', '4'))
    streams = streams[:max(1, min(len(streams), hwq))]
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


def _q_back_transform() -> str:
    """Back-transform of the sytrd tier: ``KFAC_EIGH_ORMTR`` = blocked
    (apply_q_blocked, default) | rocsolver (ormtr)."""
    return os.environ.get('KFAC_EIGH_ORMTR', 'blocked')


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
    eigenpairs of T (rocSOLVER stedc), then X = Q Z."""
    with _lane_lock(stream), torch.cuda.stream(stream):
        stream.wait_event(ev)
        for t in (red, d, e, tau):  # produced on the chain lane
            t.record_stream(stream)
        if _q_back_transform() == 'rocsolver':
            w, x = native().tridiag_eigvecs(red, d, e, tau)
            return w.clone(), x
        _tier('sytrd+' + tridiag_solver(), red.shape[-1], red.shape[0])
        if tridiag_solver() == 'dc':
            n = d.shape[-1]
            w, z = native().tridiag_eigh_dc(d, e[:, :max(n - 1, 0)])
            return w, apply_q_blocked(red, tau, z)
        w, z = native().tridiag_stedc(d, e)
        # d is the chain's persistent buffer when replayed from graphs
        return w.clone(), apply_q_blocked(red, tau, z)


def tridiag_solver() -> str:
    """Eigensolver of the reduced tridiagonal: ``KFAC_EIGH_TRIDIAG`` = dc
    (native divide and conquer, csrc/tridiag.hip; default) | stedc
    (rocSOLVER)."""
    return os.environ.get('KFAC_EIGH_TRIDIAG', 'dc')


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


_chain_cache: dict[tuple, dict] = {}
_hi: list[torch.cuda.Stream] = []


def _hi_streams(device: torch.device) -> list[torch.cuda.Stream]:
    """High-priority lanes for the largest chain and its tail
    (``KFAC_SYTRD_PRIORITY=0``: none)."""
    global _hi
    if os.environ.get('KFAC_SYTRD_PRIORITY', '1') == '0':
        return []
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


def _chain_entry(sig: tuple, keys: list, stacks: dict) -> dict:
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
            lib.sytrd_advance(state[0], sizes, k0, k1)
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
    with torch.cuda.stream(stream):
        if _chain_graphs_enabled(group):
            sig = (str(stream.device), tuple((k[0], stacks[k].shape[0]) for k in keys))
            ent = _chain_entry(sig, keys, stacks)
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
                    lib.sytrd_advance(descs, sizes, k0, k1)
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
) -> dict[int, tuple[torch.Tensor, torch.Tensor]]:
    """Large buckets: native tridiagonalisation chains (``_chain_groups``),
    one lane each, issued in segments that end where each bucket's size
    ends.  As soon as a segment is enqueued, an event marks it and that
    bucket's tail (stedc + back-transform, ``_tail_job``) is issued on
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
    small_jobs = sorted(_jobs(rest), key=lambda j: -_bucket_cost(j[0][0], j[3] - j[2]))
    lanes: list[list] = [[] for _ in others]
    loads = [0.0] * len(others)
    for job in small_jobs:
        k = loads.index(min(loads))
        loads[k] += _bucket_cost(job[0][0], job[3] - job[2])
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
    futs = [pool.submit(_run_lane, s, ln, stacks) for s, ln in active] if pool else []
    cf = [pool.submit(_run_chain, c, g, stacks, tail_lane, pool, gi) if pool else
          _run_chain(c, g, stacks, tail_lane, None, gi)
          for gi, (c, g) in enumerate(zip(chains, groups))]
    results = [f.result() for f in futs] if pool else [
        _run_lane(s, ln, stacks) for s, ln in active]
    tails = [(key, f.result() if pool else f)
             for key, f in sum((c.result() if pool else c for c in cf), [])]
    out: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
    for s in streams + hi:  # every lane's work is enqueued by now
        main.wait_stream(s)
    for (s, ln), res in zip(active, results):
        for (key, idxs, lo, hi), (evals, evecs) in zip(ln, res):
            evals.record_stream(main)
            evecs.record_stream(main)
            for k in range(hi - lo):
                out[idxs[lo + k]] = (evals[k], evecs[k])
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
    eye = torch.eye(nb, device=red.device, dtype=red.dtype)
    for p in reversed(range(0, n - 1, nb)):
        q = min(p + nb, n - 1)
        b = q - p
        v = vt[:, p:q, p + 1:]  # [c, b, m]: V_b^T restricted to rows >= p+1
        g = torch.bmm(v, v.transpose(1, 2))
        t_ = tau[:, p:q]
        dinv = torch.where(t_ == 0, torch.ones_like(t_), 1.0 / torch.where(
            t_ == 0, torch.ones_like(t_), t_))
        u = torch.triu(g, diagonal=1) + torch.diag_embed(dinv)
        tm = torch.linalg.solve_triangular(u, eye[:b, :b].expand(c, b, b), upper=True)
        xs = x[:, p + 1:, :]
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
