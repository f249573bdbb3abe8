"""Batched symmetric tridiagonal eigensolver: Cuppen divide and conquer.

This is the last stage of the native eigensolver (K-HIP-3): after the
Householder reduction ``A = Q T Q^T`` (csrc/sytrd.hip) every factor's
tridiagonal ``T`` (diagonal ``d``, off-diagonal ``e``) is diagonalised here,
``T = Z diag(w) Z^T``, and ``X = Q Z`` gives the eigenvectors of ``A``
(``ops.linalg.apply_q_blocked``).  It replaces rocSOLVER's ``stedc``; the
whole refresh then contains no library eigensolver (reference:
``torch.linalg.eigh`` in ``kfac/layers/eigen.py:294-347``).

Plan (shared by this reference implementation and csrc/tridiag.hip):

* **Padding to a uniform tree.**  ``n`` is padded to ``n_pad = L * 2^k`` with
  ``L <= 64`` chosen to minimise the padding (< 3 %): extra diagonal entries
  hold a value above every eigenvalue (Gershgorin bound) and couple to
  nothing, so every merge level has subproblems of ONE size ``m = L 2^l``
  and runs as one batched launch over (matrix, subproblem).  The padding's
  eigenpairs are the last ``n_pad - n`` of the result and are dropped.
* **Splits.**  ``T = diag(T1', T2') + rho u u^T`` at every split with
  ``rho = |beta|``, ``u = e_last + sign(beta) e_first``; the adjacent diagonal
  entries lose ``rho`` (so ``rho >= 0`` always).
* **Leaves** (``L x L``): dense symmetric eigensolves (the LDS Jacobi kernel,
  csrc/eigh_jacobi.hip, on the GPU).
* **Merge** of two children ``(D1, Q1)``, ``(D2, Q2)``:
  ``z = [Q1[last, :], sign(beta) Q2[0, :]] / sqrt(2)``, ``rho~ = 2 rho``;
  sort ``D`` (two sorted lists: one binary search per element);
  deflation (LAPACK ``slaed2``'s two tests, fp32 tolerance
  ``8 eps32 max(|d|, rho~ |z|)``): ``rho~ |z_i| <= tol`` keeps ``(d_i, e_i)``;
  two entries closer than the tolerance are combined by a Givens rotation;
  the ``K`` survivors are at least ``2 tol`` apart;
  secular equation ``1 + rho~ sum z_i^2 / (d_i - lam) = 0`` per root in
  float64, each root kept as ``origin pole + tau`` so every ``d_i - lam`` is
  formed without cancellation; Gu-Eisenstat ``z^`` recomputed from the roots
  (orthogonal eigenvectors without extra precision); ``u_j = z^ / (d - lam_j)``.
  Everything (permutation, rotations, ``u_j``, deflated unit columns, the
  final ascending order) is folded into one ``m x m`` matrix ``W`` with
  ``Q = diag(Q1, Q2) W``, i.e. two half-height GEMMs per subproblem: one
  batched GEMM per level.

The functions here are the float64 CPU reference of every step (and the CPU
implementation used by ``ops.linalg`` when no GPU is present).
"""
from __future__ import annotations

import math

import torch

EPS32 = 2.0 ** -24
LEAF_MAX = 64


def dc_plan(n: int) -> tuple[int, int, int]:
    """``(leaf, levels, n_pad)`` with ``n_pad = leaf * 2**levels >= n``,
    ``leaf <= LEAF_MAX`` and the smallest padding."""
    if n <= LEAF_MAX:
        return n, 0, n
    k = math.ceil(math.log2(n / LEAF_MAX))
    leaf = -(-n // (1 << k))
    return leaf, k, leaf << k


def pad_value(d: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    """Per matrix: a value strictly above every eigenvalue (Gershgorin)."""
    ae = e.abs()
    rad = torch.zeros_like(d)
    rad[..., :-1] += ae
    rad[..., 1:] += ae
    g = (d + rad).amax(-1)
    return g + torch.clamp(g.abs(), min=1.0)


def split_rhos(e_pad: torch.Tensor, leaf: int, levels: int) -> list[torch.Tensor]:
    """beta of every split, per level (level l merges pairs of size leaf*2^l):
    ``[batch, n_pad / (2 m_child)]`` each."""
    out = []
    n_pad = leaf << levels
    for lv in range(levels):
        h = leaf << lv
        pos = torch.arange(h - 1, n_pad - 1, 2 * h)
        out.append(e_pad[:, pos])
    return out


def leaf_matrices(d_pad: torch.Tensor, e_pad: torch.Tensor, leaf: int) -> torch.Tensor:
    """Dense leaf blocks ``[batch * n_pad / leaf, leaf, leaf]`` with the
    split corrections applied to their first / last diagonal entries."""
    b, n_pad = d_pad.shape
    dm = d_pad.clone()
    ae = e_pad.abs()
    cut = torch.arange(leaf - 1, n_pad - 1, leaf)  # every leaf boundary is a split
    dm[:, cut] -= ae[:, cut]
    dm[:, cut + 1] -= ae[:, cut]
    nl = n_pad // leaf
    blocks = torch.zeros(b, nl, leaf, leaf, dtype=d_pad.dtype)
    idx = torch.arange(leaf)
    blocks[:, :, idx, idx] = dm.view(b, nl, leaf)
    off = e_pad.clone()
    off[:, cut] = 0.0
    off = torch.cat([off, off.new_zeros(b, 1)], 1).view(b, nl, leaf)[:, :, :-1]
    blocks[:, :, idx[:-1], idx[1:]] = off
    blocks[:, :, idx[1:], idx[:-1]] = off
    return blocks.view(b * nl, leaf, leaf)


def secular_roots(d: torch.Tensor, z: torch.Tensor, rho: float
                  ) -> tuple[torch.Tensor, torch.Tensor]:
    """Roots of ``1 + rho sum z_i^2/(d_i - lam)`` for ascending distinct
    ``d`` (float64); returns (origin index, tau) per root: lam_j = d[o_j] +
    tau_j.  Safeguarded two-pole rational iteration with bisection."""
    k = d.numel()
    org = torch.empty(k, dtype=torch.long)
    tau = torch.empty(k, dtype=torch.float64)
    z2 = z * z
    for j in range(k):
        if j < k - 1:
            gap = float(d[j + 1] - d[j])
            mid = 0.5 * gap
            f = 1.0 + rho * float((z2 / (d - d[j] - mid)).sum())
            if f > 0:
                o, lo, hi = j, 0.0, mid
            else:
                o, lo, hi = j + 1, -mid, 0.0
        else:
            o, lo, hi = j, 0.0, rho * float(z2.sum())
        dl = (d - d[o]).tolist()
        zl = z2.tolist()
        t = 0.5 * (lo + hi)
        for _ in range(200):
            psi = dpsi = phi = dphi = 0.0
            for i in range(k):
                r = 1.0 / (dl[i] - t)
                if i <= j:
                    psi += zl[i] * r
                    dpsi += zl[i] * r * r
                else:
                    phi += zl[i] * r
                    dphi += zl[i] * r * r
            f = 1.0 + rho * (psi + phi)
            if f == 0.0:
                break
            if f > 0:
                hi = t
            else:
                lo = t
            if hi - lo <= 4 * 2.2e-16 * max(abs(lo), abs(hi), abs(dl[j]) + abs(t)):
                break
            if abs(f) <= 8 * k * 2.2e-16 * (1.0 + rho * (abs(psi) + abs(phi))):
                break
            # Newton on the two-pole model (poles at dl[j], dl[j+1])
            tn = _two_pole_step(t, f, rho, psi, dpsi, phi, dphi, dl, j, k)
            if not (lo < tn < hi):
                tn = 0.5 * (lo + hi)
            t = tn
        org[j] = o
        tau[j] = t
    return org, tau


def _two_pole_step(t: float, f: float, rho: float, psi: float, dpsi: float,
                   phi: float, dphi: float, dl: list, j: int, k: int) -> float:
    """Zero of c + s1/(p1 - x) + s2/(p2 - x) matching f and its two pole
    parts' derivatives at t (Gragg's scheme); Newton if degenerate."""
    p1 = dl[j]
    a1 = p1 - t
    s1 = rho * dpsi * a1 * a1
    if j < k - 1:
        p2 = dl[j + 1]
        a2 = p2 - t
        s2 = rho * dphi * a2 * a2
    else:
        p2, a2, s2 = 0.0, 0.0, 0.0
    c = f - s1 / a1 - (s2 / a2 if j < k - 1 else rho * phi)
    if j == k - 1:
        # c + s1/(p1 - x) = 0  ->  x = p1 + s1/c
        return p1 + s1 / c if c != 0 else t
    # c (p1-x)(p2-x) + s1 (p2-x) + s2 (p1-x) = 0 in y = x - t:
    # c (a1-y)(a2-y) + s1 (a2-y) + s2 (a1-y) = 0
    qa = c
    qb = -(c * (a1 + a2) + s1 + s2)
    qc = c * a1 * a2 + s1 * a2 + s2 * a1
    if qa == 0:
        return t - qc / qb if qb != 0 else t
    disc = qb * qb - 4 * qa * qc
    if disc < 0:
        disc = 0.0
    sq = math.sqrt(disc)
    # stable quadratic roots
    qq = -0.5 * (qb + math.copysign(sq, qb))
    cands = []
    if qq != 0:
        cands.append(qc / qq)
    if qa != 0:
        cands.append(qq / qa)
    lo, hi = min(a1, a2), max(a1, a2)
    for y in cands:
        if lo < y < hi:
            return t + y
    deriv = rho * (dpsi + dphi)
    return t - f / deriv if deriv > 0 else t


def merge(D1: torch.Tensor, Q1: torch.Tensor, D2: torch.Tensor, Q2: torch.Tensor,
          beta: float) -> tuple[torch.Tensor, torch.Tensor]:
    """One merge (float64 reference): children eigenpairs -> parent's."""
    h1, h2 = D1.numel(), D2.numel()
    m = h1 + h2
    sgn = 1.0 if beta >= 0 else -1.0
    rho = 2.0 * abs(beta)
    D = torch.cat([D1, D2])
    z = torch.cat([Q1[-1, :], sgn * Q2[0, :]]) / math.sqrt(2.0)
    perm = torch.argsort(D, stable=True)
    d = D[perm].clone()
    zs = z[perm].clone()
    tol = 8.0 * EPS32 * max(float(d.abs().max()), rho * float(zs.abs().max()))
    # deflation walk; W0 = identity on sorted coordinates, rotations recorded
    rot = []
    nd: list[int] = []
    dfl: list[int] = []
    for i in range(m):
        if rho * abs(float(zs[i])) <= tol:
            dfl.append(i)
            continue
        if nd:
            p = nd[-1]
            s, c = float(zs[p]), float(zs[i])
            tau = math.hypot(c, s)
            c, s = c / tau, -s / tau
            if abs((float(d[i]) - float(d[p])) * c * s) <= tol:
                zs[i] = tau
                zs[p] = 0.0
                dp, di = float(d[p]), float(d[i])
                d[p] = dp * c * c + di * s * s
                d[i] = dp * s * s + di * c * c
                rot.append((p, i, c, s))
                nd[-1] = i
                dfl.append(p)
                continue
        nd.append(i)
    K = len(nd)
    lam = torch.empty(m, dtype=torch.float64)
    W = torch.zeros(m, m, dtype=torch.float64)
    if K:
        dn, zn = d[nd], zs[nd]
        org, tau = secular_roots(dn, zn, rho)
        lamn = dn[org] + tau
        # Gu-Eisenstat z^
        zh = torch.empty(K, dtype=torch.float64)
        for i in range(K):
            dif = (dn[org] - dn[i]) + tau  # lam_j - d_i
            den = dn - dn[i]
            num = dif[i] / rho
            for j in range(K):
                if j != i:
                    num *= float(dif[j]) / float(den[j])
            zh[i] = math.copysign(math.sqrt(max(num, 0.0)), float(zn[i]))
        U = torch.empty(K, K, dtype=torch.float64)
        for j in range(K):
            col = zh / ((dn - dn[org[j]]) - tau[j])
            U[:, j] = col / col.norm()
    # final ascending order over roots and deflated values
    vals = torch.cat([lamn if K else torch.empty(0, dtype=torch.float64), d[dfl]])
    order = torch.argsort(vals, stable=True)
    pos = torch.empty(m, dtype=torch.long)
    pos[order] = torch.arange(m)
    lam = vals[order]
    for jj, j in enumerate(range(K)):
        W[torch.tensor(nd), pos[jj]] = U[:, j]
    for t_, i in enumerate(dfl):
        W[i, pos[K + t_]] = 1.0
    # rotations: Q_sorted_rot = Q_sorted G_1^T ... G_r^T  ->  fold into W rows
    for (p, i, c, s) in reversed(rot):
        wp, wi = W[p].clone(), W[i].clone()
        W[p] = c * wp - s * wi
        W[i] = s * wp + c * wi
    # sorted coordinates -> children's column order
    Wc = torch.zeros_like(W)
    Wc[perm] = W
    Q = torch.zeros(m, m, dtype=torch.float64)
    Q[:h1] = Q1 @ Wc[:h1]
    Q[h1:] = Q2 @ Wc[h1:]
    return lam, Q


def tridiag_eigh_reference(d: torch.Tensor, e: torch.Tensor
                           ) -> tuple[torch.Tensor, torch.Tensor]:
    """Divide and conquer for ONE tridiagonal (float64, CPU): ascending
    eigenvalues and eigenvectors (columns).  Follows the batched plan of the
    module docstring step for step (padding, leaves, level merges)."""
    d = d.to(torch.float64).reshape(1, -1)
    e = e.to(torch.float64).reshape(1, -1)
    n = d.shape[1]
    leaf, levels, n_pad = dc_plan(n)
    pv = pad_value(d, e)
    dp = torch.cat([d, pv.reshape(1, 1).expand(1, n_pad - n)], 1)
    ep = torch.cat([e, e.new_zeros(1, n_pad - 1 - e.shape[1])], 1)
    blocks = leaf_matrices(dp, ep, leaf)
    w, v = torch.linalg.eigh(blocks)
    subs = [(w[i], v[i]) for i in range(w.shape[0])]
    rhos = split_rhos(ep, leaf, levels)
    for lv in range(levels):
        nxt = []
        for s in range(len(subs) // 2):
            (D1, Q1), (D2, Q2) = subs[2 * s], subs[2 * s + 1]
            nxt.append(merge(D1, Q1, D2, Q2, float(rhos[lv][0, s])))
        subs = nxt
    lam, Q = subs[0]
    return lam[:n], Q[:n, :n]
