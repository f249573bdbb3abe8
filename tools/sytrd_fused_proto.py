"""CPU prototype of the one-launch-per-column tridiagonalisation (fused
symv + next col step).

Per column k (panel column i = k - p) ONE kernel F(k) runs over row blocks:

1. every block reduces the previous column's totals: alpha2_{k-1} = -tau/2
   (w.v), X = w_raw_{k-1}[k] + 2 alpha2_{k-1}; row k is a_k = B - v_{k-1} X
   where B was written by F(k-1); the larfg sums of row k are polynomials in
   X of the totals F(k-1) left (so no block needs another block's rows);
2. reflector v_k, t1 = W^T v, t2 = V^T v, y = A22 v, w_raw = tau (y - V t1 -
   W t2) for the block's rows (W final = w_raw + alpha2 v, applied on the
   fly: no write-back race);
3. pre-col of row k+1 for the block's rows: B[r] = A[r][k+1] - sum_{j<i}
   (V_j[r] W_j[k+1] + W_j[r] V_j[k+1]) - w_raw[r], plus the partial sums of
   B^2, B.v_k, v_k^2, w_raw.B, w_raw.v_k and W_j.B, W_j.v_k, V_j.B, V_j.v_k.

Checks A = Q T Q^T against numpy like tools/sytrd_proto.py.
Run: python tools/sytrd_fused_proto.py
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

NB = 8


def sytrd_fused(A: np.ndarray, nb: int = NB):
    A = A.copy()
    n = A.shape[0]
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    tau = np.zeros(max(n - 1, 0))

    def vcol(j_row, r0):  # reflector stored in row j_row, entries r >= r0
        r = np.arange(r0, n)
        return np.where(r == j_row + 1, 1.0, np.where(r > j_row + 1, A[j_row, r0:], 0.0))

    for p in range(0, n, nb):
        q = min(p + nb, n)
        Wraw = np.zeros((nb, n))
        alpha2 = np.zeros(nb)
        tau_l = np.zeros(nb)

        def wfin(j, r0):  # final W_j over r >= r0
            return Wraw[j, r0:] + alpha2[j] * vcol(p + j, r0)

        # head: row p is fully updated (previous panels applied)
        B = A[p, :].copy()
        tot = None
        for k in range(p, q):
            i = k - p
            # ---- 1. row k and its larfg sums
            if i == 0:
                a = B.copy()
                xn2 = float(a[k + 2:] @ a[k + 2:]) if k + 2 < n else 0.0
                dW = np.zeros(0)
                dV = np.zeros(0)
            else:
                vk1 = vcol(k - 1, 0)  # v_{k-1} over all rows (0 below k)
                dot = float(Wraw[i - 1, k:] @ vk1[k:])
                alpha2[i - 1] = -0.5 * tau_l[i - 1] * dot
                X = Wraw[i - 1, k] + 2.0 * alpha2[i - 1]
                a = B - vk1 * X
                S = tot
                xn2 = S['BB'] - 2 * X * S['Bv'] + X * X * S['vv']
                dW = np.array([S['WB'][j] - X * S['Wv'][j] for j in range(i - 1)]
                              + [S['wB'] - X * S['wv'] + alpha2[i - 1] * (S['Bv'] - X * S['vv'])])
                dV = np.array([S['VB'][j] - X * S['Vv'][j] for j in range(i - 1)]
                              + [S['Bv'] - X * S['vv']])
            d[k] = a[k]
            if k == n - 1:
                break
            alpha = a[k + 1]
            if xn2 <= 0.0:
                t, beta, s = 0.0, alpha, 0.0
            else:
                beta = -np.copysign(np.sqrt(alpha * alpha + xn2), alpha)
                t = (beta - alpha) / beta
                s = 1.0 / (alpha - beta)
            e[k] = beta
            tau[k] = t
            tau_l[i] = t
            vk = np.zeros(n)
            vk[k + 1] = 1.0
            vk[k + 2:] = s * a[k + 2:]
            A[k, k + 2:] = vk[k + 2:]  # final reflector k (rows r >= k+2 write theirs)
            # ---- 2. symv for rows r >= k+1
            t1 = np.array([wfin(j, k + 1)[0] + s * dW[j] for j in range(i)])
            t2 = np.array([vcol(p + j, k + 1)[0] + s * dV[j] for j in range(i)])
            y = A[k + 1:, k + 1:] @ vk[k + 1:]
            for j in range(i):
                y -= vcol(p + j, k + 1) * t1[j] + wfin(j, k + 1) * t2[j]
            Wraw[i, k + 1:] = t * y
            # ---- 3. pre-col of row k+1 (inside the panel only)
            if k + 1 < q and k + 1 < n:
                r0 = k + 1
                Bn = np.zeros(n)
                acc = A[r0:, k + 1].copy()  # = A[k+1][r] by symmetry (panel-start)
                for j in range(i):
                    acc -= vcol(p + j, r0) * wfin(j, r0)[0] + wfin(j, r0) * vcol(p + j, r0)[0]
                acc -= Wraw[i, r0:]
                Bn[r0:] = acc
                x0 = k + 3
                Bx, vx, wx = Bn[x0:], vk[x0:], Wraw[i, x0:]
                tot = {'BB': float(Bx @ Bx), 'Bv': float(Bx @ vx), 'vv': float(vx @ vx),
                       'wB': float(wx @ Bx), 'wv': float(wx @ vx),
                       'WB': [float(wfin(j, x0) @ Bx) for j in range(i)],
                       'Wv': [float(wfin(j, x0) @ vx) for j in range(i)],
                       'VB': [float(vcol(p + j, x0) @ Bx) for j in range(i)],
                       'Vv': [float(vcol(p + j, x0) @ vx) for j in range(i)]}
                B = Bn
        # ---- panel end: finalise the last column, trailing update
        klast = q - 1
        if klast < n - 1:
            il = klast - p
            dot = float(Wraw[il, q:] @ vcol(klast, q)) + Wraw[il, q - 1] * 0.0
            # w.v over r >= klast+1 (v[klast+1] = 1)
            dot = float(Wraw[il, klast + 1:] @ vcol(klast, klast + 1))
            alpha2[il] = -0.5 * tau_l[il] * dot
            V = np.stack([vcol(p + j, q) for j in range(q - p)])
            W = np.stack([wfin(j, q) for j in range(q - p)])
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
    for n in (1, 2, 3, 5, 8, 9, 16, 17, 23, 40, 65):
        x = rng.standard_normal((n, 2 * n))
        M = x @ x.T / (2 * n)
        R, d, e, tau = sytrd_fused(M)
        Q = form_q(R, tau)
        T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
        err = np.abs(Q @ T @ Q.T - M).max()
        orth = np.abs(Q.T @ Q - np.eye(n)).max()
        w = scipy.linalg.eigh_tridiagonal(d, e, eigvals_only=True) if n > 1 else d
        ew = np.abs(np.sort(w) - np.linalg.eigvalsh(M)).max()
        print(f'n={n:3d} recon={err:.2e} orth={orth:.2e} eig={ew:.2e}')
        assert err < 1e-10 and orth < 1e-10 and ew < 1e-10


if __name__ == '__main__':
    main()
