"""Two-stage symmetric eigensolver (K-HIP-3 for every factor above the LDS
Jacobi tier): float64 CPU oracle of every stage and the GPU entry point.

The reference decomposes each K-FAC factor with ``torch.linalg.eigh``
(``kfac/layers/eigen.py:294-347``).  On MI355X a one-stage Householder
tridiagonalisation streams the whole trailing matrix once per column (a
matrix-vector product per column: HBM-bound, and one kernel boundary per
column); this solver does the O(n^3) part with level-3 operations:

1. **dense -> band** (width ``B = 16``, csrc/sy2sb.hip): panel QR of 16
   columns at a time, two-sided trailing updates with batched GEMMs.
2. **band -> tridiagonal** (csrc/sb2st.hip): bulge chasing.  Sweep ``j``
   annihilates column ``j`` (task 0) and chases the bulge down the band
   (tasks ``k >= 1``, each on a 32 x 32 window starting at column
   ``j + 1 + 16 (k - 1)``).  Task ``(j, k)`` depends only on ``(j, k-1)`` and
   ``(j-1, k+2)``: sweeps run as a pipeline, one wave each.
3. **tridiagonal eigenpairs**: divide and conquer (``ops.tridiag``).
4. **back-transforms**: ``X = Q1 Q2 Z``.  ``Q2``'s reflectors are grouped
   into compact-WY blocks of 16 sweeps; blocks with the same step
   ``2 (G - 1 - g) + k`` touch disjoint rows, so each step is one launch
   (csrc/bt2.hip).  ``Q1`` is applied in UT blocks of 512 reflectors.

The functions below are the float64 references of those exact algorithms
(and data layouts where they matter); ``tests/test_twostage.py`` checks
them against LAPACK on the CPU and ``tests/test_twostage_gpu.py`` the
kernels against them / float64 ``eigh`` on the GPU.
"""
from __future__ import annotations

import logging

import torch

from distributed_kfac_pytorch_amd.ops._native import native

logger = logging.getLogger(__name__)
BAND = 16


def _house(x: torch.Tensor) -> tuple[torch.Tensor, float, float]:
    """``v`` (``v[0] = 1``), ``tau``, ``beta`` with ``(I - tau v v^T) x = beta e1``
    (LAPACK larfg without the scaling loop)."""
    alpha = float(x[0])
    xn2 = float((x[1:] * x[1:]).sum())
    v = torch.zeros_like(x)
    v[0] = 1.0
    if xn2 == 0.0:
        return v, 0.0, alpha
    beta = -((alpha * alpha + xn2) ** 0.5) * (1.0 if alpha >= 0 else -1.0)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def larft(v: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
    """Forward / columnwise compact-WY factor: ``H_0 H_1 ... = I - V T V^T``."""
    k = v.shape[1]
    t = torch.zeros(k, k, dtype=v.dtype)
    for i in range(k):
        t[i, i] = tau[i]
        if i:
            t[:i, i] = -tau[i] * (t[:i, :i] @ (v[:, :i].T @ v[:, i]))
    return t


def sy2sb_reference(a: torch.Tensor, b: int = BAND) -> tuple[torch.Tensor, list]:
    """Stage 1 (float64): returns the band matrix (dense storage) and the
    panels ``[(p, V, T)]`` with ``A = Q1 B Q1^T``, ``Q1 = prod_p (I - V T V^T)``
    acting on rows ``p + b ..``."""
    a = a.to(torch.float64).clone()
    n = a.shape[0]
    panels = []
    p = 0
    while n - p - b >= 2:
        m = n - p - b
        pan = a[p + b:, p:p + b].clone()
        bb = min(b, m)
        v = torch.zeros(m, b, dtype=a.dtype)
        taus = torch.zeros(b, dtype=a.dtype)
        for t in range(bb):
            vt, tau, _ = _house(pan[t:, t].clone())
            pan[t:, t:] -= tau * torch.outer(vt, vt @ pan[t:, t:])
            v[t:, t] = vt
            taus[t] = tau
        tm = larft(v, taus)
        a[p + b:, p:p + b] = torch.triu(pan)
        a[p:p + b, p + b:] = a[p + b:, p:p + b].T
        a22 = a[p + b:, p + b:]
        y = a22 @ v @ tm
        s = tm.T @ (v.T @ y)
        w = y - 0.5 * v @ (0.5 * (s + s.T))
        a[p + b:, p + b:] = a22 - v @ w.T - w @ v.T
        panels.append((p, v, tm))
        p += b
    return a, panels


def ntasks(j: int, n: int, b: int = BAND) -> int:
    """Tasks of sweep ``j`` of the bulge chase."""
    return 1 + (n - 2 - j) // b


def sb2st_reference(band: torch.Tensor, b: int = BAND, order: str = 'sequential',
                    seed: int = 0) -> tuple[torch.Tensor, torch.Tensor, dict]:
    """Stage 2 (float64) on a dense symmetric band matrix, each task
    restricted to its window.  ``order='pipeline'`` runs the tasks in a
    random order that only respects the kernel's dependencies ((j, k) after
    (j, k-1) and (j-1, min(k+2, last))); the result must be identical.
    Returns ``(d, e, reflectors {(j, k): (start_row, v, tau)})``."""
    a = band.to(torch.float64).clone()
    n = a.shape[0]
    refl: dict = {}
    state: dict = {}
    done = {j: 0 for j in range(n - 2)}
    nk = {j: ntasks(j, n, b) for j in range(n - 2)}

    def task(j: int, k: int) -> None:
        if k == 0:
            st, ed = j + 1, min(j + b, n - 1)
            v, tau, beta = _house(a[st:ed + 1, j].clone())
            a[st:ed + 1, j] = 0.0
            a[st, j] = beta
            a[j, st:ed + 1] = a[st:ed + 1, j]
            h = torch.eye(len(v), dtype=a.dtype) - tau * torch.outer(v, v)
            a[st:ed + 1, st:ed + 1] = h @ a[st:ed + 1, st:ed + 1] @ h
            state[j] = (st, ed, h)
            refl[(j, 0)] = (st, v, tau)
            return
        st, ed, h = state[j]
        j1, j2 = ed + 1, min(ed + b, n - 1)
        blk = a[j1:j2 + 1, st:ed + 1] @ h
        v2, tau2, beta2 = _house(blk[:, 0].clone())
        h2 = torch.eye(len(v2), dtype=a.dtype) - tau2 * torch.outer(v2, v2)
        blk[:, 1:] = h2 @ blk[:, 1:]
        blk[:, 0] = 0.0
        blk[0, 0] = beta2
        a[j1:j2 + 1, st:ed + 1] = blk
        a[st:ed + 1, j1:j2 + 1] = blk.T
        a[j1:j2 + 1, j1:j2 + 1] = h2 @ a[j1:j2 + 1, j1:j2 + 1] @ h2
        state[j] = (j1, j2, h2)
        refl[(j, k)] = (j1, v2, tau2)

    if order == 'sequential':
        for j in range(n - 2):
            for k in range(nk[j]):
                task(j, k)
    else:
        gen = torch.Generator().manual_seed(seed)
        active = list(range(n - 2))
        while active:
            ready = [j for j in active
                     if j == 0 or done[j - 1] >= min(done[j] + 3, nk[j - 1])]
            j = ready[int(torch.randint(len(ready), (1,), generator=gen))]
            task(j, done[j])
            done[j] += 1
            if done[j] == nk[j]:
                active.remove(j)
    return a.diagonal().clone(), a.diagonal(-1).clone(), refl


def bt2_reference(refl: dict, z: torch.Tensor, n: int, b: int = BAND) -> torch.Tensor:
    """``Q2 Z`` by csrc/bt2.hip's schedule: blocks of ``b`` sweeps, applied in
    step order ``2 (G - 1 - g) + k``; all blocks of one step at once."""
    x = z.to(torch.float64).clone()
    groups = -(-(n - 2) // b)
    kmax = ntasks(0, n, b)
    steps = 2 * (groups - 1) + kmax
    for st in range(steps):
        pending = []
        for g in range(groups):
            k = st - 2 * (groups - 1 - g)
            j0 = b * g
            if k < 0 or k >= ntasks(j0, n, b):
                continue
            s = b * (g + k) + 1
            vb = torch.zeros(2 * b, b, dtype=x.dtype)
            tv = torch.zeros(b, dtype=x.dtype)
            for t in range(b):
                j = j0 + t
                if j < n - 2 and (j, k) in refl:
                    st_row, v, tau = refl[(j, k)]
                    assert st_row == s + t
                    vb[t:t + len(v), t] = v
                    tv[t] = tau
            rows = min(2 * b, n - s)
            vb = vb[:rows]
            pending.append((s, rows, vb, larft(vb, tv)))
        # disjoint rows within a step: order-independent
        for s, rows, vb, tm in pending:
            xs = x[s:s + rows]
            xs -= vb @ (tm @ (vb.T @ xs))
    return x


def q1_apply_reference(panels: list, x: torch.Tensor, b: int = BAND) -> torch.Tensor:
    """``Q1 X`` (panels last to first)."""
    x = x.to(torch.float64).clone()
    for p, v, tm in reversed(panels):
        xs = x[p + b:]
        xs -= v @ (tm @ (v.T @ xs))
    return x


def eigh_reference(a: torch.Tensor, b: int = BAND, order: str = 'sequential'
                   ) -> tuple[torch.Tensor, torch.Tensor]:
    """The whole two-stage pipeline in float64 (tridiagonal eigenpairs by
    LAPACK): ascending eigenvalues, eigenvectors in columns."""
    n = a.shape[0]
    band, panels = sy2sb_reference(a, b)
    idx = torch.arange(n)
    mask = (idx[:, None] - idx[None, :]).abs() <= b
    d, e, refl = sb2st_reference(torch.where(mask, band, torch.zeros_like(band)), b, order)
    t = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    w, z = torch.linalg.eigh(t)
    x = bt2_reference(refl, z, n, b)
    return w, q1_apply_reference(panels, x, b)


def max_n() -> int:
    """Largest factor the GPU two-stage path supports (panel rows per
    thread of the 1024-thread panel QR)."""
    lib = native()
    return int(lib.eigh_twostage_max_n()) if lib is not None else 0


def eigh_twostage(stack: torch.Tensor, timed: bool = False
                  ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """GPU two-stage eigensolver of a ``[batch, n, n]`` fp32 stack (one
    bucket of same-size factors) on the current stream.  Returns ``(w, X,
    err, stage_ms)``: ascending eigenvalues, eigenvectors in columns, the
    bulge-chasing timeout flag (``w`` is NaN when set) and -- with
    ``timed`` (synchronises) -- milliseconds of stage 1, stage 2, the
    tridiagonal solve, the stage-2 and the stage-1 back-transforms."""
    w, x, err, ms = native().eigh_twostage(stack.contiguous(), timed)
    return w, x, err, ms


_graphs: dict = {}


def graphs_enabled() -> bool:
    """``KFAC_TWOSTAGE_GRAPHS=1`` (default off): replay each (size, batch)
    signature's whole solve from one captured HIP graph."""
    import os

    return os.environ.get('KFAC_TWOSTAGE_GRAPHS', '0') == '1'


def eigh_twostage_graphed(stack: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """``eigh_twostage`` replayed from a HIP graph per ``(device, n, batch)``.

    A 4608 factor's stage 1 alone is ~290 panels of ~10 launches; issued
    from the host one by one they are launch-bound.  The first call of a
    signature runs eagerly (its result is returned) and then captures the
    same solve on static buffers (thread-local capture: other eigensolver
    lanes keep running); later calls copy the input in and replay.  The
    returned tensors are the graph's static outputs: valid until the next
    call with the same signature (the eigen layers copy them into their own
    buffers when they install a refresh)."""
    key = (stack.device, tuple(stack.shape), torch.cuda.current_stream(stack.device).cuda_stream)
    if key not in _graphs:
        static_in = stack.contiguous().clone()
        w, x, err, _ = eigh_twostage(static_in)
        g = torch.cuda.CUDAGraph()
        ent = None
        try:
            g.capture_begin(capture_error_mode='thread_local')
            try:
                outs = eigh_twostage(static_in)
            finally:
                g.capture_end()
            ent = (g, static_in, outs)
        except RuntimeError as e:  # not capturable here: stay eager for this signature
            logger.warning('two-stage eigensolver graph capture failed (%s); eager', e)
        _graphs[key] = ent
        return w, x
    ent = _graphs[key]
    if ent is None:
        w, x, _, _ = eigh_twostage(stack)
        return w, x
    g, static_in, outs = ent
    static_in.copy_(stack)
    g.replay()
    return outs[0], outs[1]
