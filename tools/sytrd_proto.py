"""CPU prototype of the batched blocked tridiagonalisation in csrc/sytrd.hip.

Mirrors the kernel decomposition exactly (row-major storage, reflector k in
row k, panel width NB): per column k a ``col`` step (finalise column k-1,
update row k with the panel's V/W, larfg partial sums) and a ``symv`` step
(w = tau (A22 v - V Wᵀv - W Vᵀv)), and per panel a ``fin`` step plus the
rank-2NB trailing update.  Checks A = Q T Qᵀ and the eigenvalues against
numpy.  Run: python tools/sytrd_proto.py (also checks the triangle-tile symv algebra
of BASELINE.md round 4: slot-summed y and w.v = tau (v^T A22 v - 2 t1.t2))
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

NB = 8


def sytrd(A: np.ndarray, nb: int = NB, tri: bool = False, tt: int = 4):
    A = A.copy()
    n = A.shape[0]
    Wt = np.zeros((nb, n))
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    tau = np.zeros(max(n - 1, 0))
    sc = {}  # per column: (tau, scale, dot-partial)

    def finalize(k, i):
        # normalise reflector row k-1 and apply alpha2 to Wt[i-1]
        t, s, dw = sc[k - 1]
        alpha2 = -0.5 * t * dw
        r = np.arange(k, n)
        v = np.where(r == k, 1.0, A[k - 1, k:] * s)
        A[k - 1, k + 1:] = v[1:]
        Wt[i - 1, k:] = Wt[i - 1, k:] + alpha2 * v

    def vrow(p, j, k):  # V_j over r >= k (j panel-local)
        r = np.arange(k, n)
        return np.where(r == p + j + 1, 1.0, np.where(r > p + j + 1, A[p + j, k:], 0.0))

    for p in range(0, n, nb):
        q = min(p + nb, n)
        for k in range(p, q):
            i = k - p
            if i > 0:
                finalize(k, i)
            # col step: update row k over r >= k
            a = A[k, k:].copy()
            for j in range(i):
                vk = 1.0 if k == p + j + 1 else A[p + j, k]
                a -= vrow(p, j, k) * Wt[j, k] + Wt[j, k:] * vk
            A[k, k:] = a
            d[k] = a[0]
            if k == n - 1:
                break
            alpha = a[1]
            x = a[2:]
            xn2 = float(x @ x)
            dW = np.array([Wt[j, k + 2:] @ x for j in range(i)])
            dV = np.array([vrow(p, j, k + 2) @ x for j in range(i)])
            # symv step
            if xn2 == 0.0:
                t, beta, s = 0.0, alpha, 0.0
            else:
                beta = -np.copysign(np.sqrt(alpha * alpha + xn2), alpha)
                t = (beta - alpha) / beta
                s = 1.0 / (alpha - beta)
            e[k] = beta
            tau[k] = t
            v = np.concatenate([[1.0], s * x])
            t1 = np.array([Wt[j, k + 1] + s * dW[j] for j in range(i)])
            t2 = np.array([A[p + j, k + 1] + s * dV[j] for j in range(i)])
            if tri:
                # triangle-tile symv: lower
                # tiles (I >= J) of the stale trailing matrix add A_IJ v_J to
                # the row slots of I and A_IJ^T v_I to those of J; a row's
                # y is the sum of its slots; w.v from the tiles' quadratic
                # partials, w.v = tau (v^T A22 v - 2 t1.t2)
                m = n - k - 1
                nt = -(-m // tt)
                slots = np.zeros((nt, m))
                quad = 0.0
                A22 = A[k + 1:, k + 1:]
                for I in range(nt):
                    for J in range(I + 1):
                        ri = slice(I * tt, min(m, (I + 1) * tt))
                        cj = slice(J * tt, min(m, (J + 1) * tt))
                        blk = A22[ri, cj]
                        slots[J, ri] += blk @ v[cj]
                        qt = float(v[ri] @ (blk @ v[cj]))
                        if I != J:
                            slots[I, cj] += blk.T @ v[ri]
                            qt *= 2.0
                        quad += qt
                y = slots.sum(axis=0)
            else:
                y = A[k + 1:, k + 1:] @ v
            for j in range(i):
                y -= vrow(p, j, k + 1) * t1[j] + Wt[j, k + 1:] * t2[j]
            w = t * y
            Wt[i, k + 1:] = w
            wv = float(w @ v)
            if tri:
                wv_tiles = t * (quad - 2.0 * float(t1 @ t2))
                assert abs(wv_tiles - wv) <= 1e-9 * max(1.0, abs(wv)), (k, wv_tiles, wv)
                wv = wv_tiles
            sc[k] = (t, s, wv)
        # panel end: finalise the last column, trailing rank-2nb update
        klast = q - 1
        if klast < n - 1:
            finalize(klast + 1, klast - p + 1)
            V = np.stack([vrow(p, j, q) for j in range(q - p)])
            W = Wt[: q - p, q:]
            A[q:, q:] -= V.T @ W + W.T @ V
    return A, d, e, tau


def form_q(A, tau):
    n = A.shape[0]
    Q = np.eye(n)
    for k in range(n - 2, -1, -1):
        v = np.zeros(n)
        v[k + 1] = 1.0
        v[k + 2:] = A[k, k + 2:]
        Q = Q - tau[k] * np.outer(v, v @ Q)
    return Q


def main() -> None:
    rng = np.random.default_rng(0)
    for n, tri in ((1, False), (2, False), (3, False), (5, False), (8, False), (9, False),
                   (17, False), (40, False), (9, True), (17, True), (40, True)):
        x = rng.standard_normal((n, 2 * n))
        M = x @ x.T / (2 * n)
        R, d, e, tau = sytrd(M, tri=tri)
        Q = form_q(R, tau)
        T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
        err = np.abs(Q @ T @ Q.T - M).max()
        orth = np.abs(Q.T @ Q - np.eye(n)).max()
        w = scipy.linalg.eigh_tridiagonal(d, e, eigvals_only=True) if n > 1 else d
        ew = np.abs(np.sort(w) - np.linalg.eigvalsh(M)).max()
        print(f'n={n:3d} tri={int(tri)} recon={err:.2e} orth={orth:.2e} eig={ew:.2e}')
        assert err < 1e-10 and orth < 1e-10 and ew < 1e-10


if __name__ == '__main__':
    main()
