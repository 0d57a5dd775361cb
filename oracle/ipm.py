"""ORACLE (test infrastructure only) -- dense primal-dual conic QP interior-point method.

This is the CPU checker for the agent-QP hot path. It is NOT part of the product and
must only be imported from ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``.

What it restates
----------------
The reference hands every per-step QP to cvxpy + Clarabel
(``control/rqp_centralized.py:132,440``, ``control/rqp_cadmm.py:140,492``,
``control/rqp_dd.py:145,485``).  Clarabel is a primal-dual interior-point method
for conic programs (Nesterov-Todd scaling on second-order cones).  Neither cvxpy
nor Clarabel is installed here, so Clarabel's *answer* is restated: every QP on the
path is strictly convex ("Hard parts"), its minimiser is unique,
and a solution that carries a tight KKT certificate IS the answer Clarabel returns up
to Clarabel's own tolerance (~1e-8).  This module solves

    min 1/2 x'Px + q'x   s.t.  A x = b,  G x + s = h,  s in K
    K = R_+^l  x  Q^{q_1} x ... x Q^{q_k}

with a Mehrotra predictor-corrector on the NT-scaled Newton system, dense KKT
solves (numpy.linalg), tolerance 1e-11 -- three orders tighter than Clarabel's
default -- and returns the KKT certificate (primal/dual residual, gap) with x.

Parity status: the solver answer is pinned by optimality certificates and by an
independent scipy cross-check in ``tests/test_oracle_ipm.py``; Clarabel itself is
absent, so bit-level parity with Clarabel is *unpinned* ("Oracle").
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

OPTIMAL = 0
MAX_ITER = 1
NUMERICAL = 2
INFEASIBLE = 3  # a linear row 0'x <= h_j with h_j < 0: primal infeasible (Clarabel reports "infeasible")


@dataclass
class ConeDims:
    l: int = 0
    q: list = field(default_factory=list)

    @property
    def m(self) -> int:
        return self.l + int(sum(self.q))

    @property
    def degree(self) -> int:
        return self.l + len(self.q)

    def blocks(self):
        off = self.l
        for d in self.q:
            yield off, d
            off += d


def _e(dims: ConeDims) -> np.ndarray:
    e = np.zeros(dims.m)
    e[: dims.l] = 1.0
    for off, _ in dims.blocks():
        e[off] = 1.0
    return e


def _jprod(u, v, dims):
    w = np.empty_like(u)
    w[: dims.l] = u[: dims.l] * v[: dims.l]
    for off, d in dims.blocks():
        a, b = u[off : off + d], v[off : off + d]
        w[off] = a @ b
        w[off + 1 : off + d] = a[0] * b[1:] + b[0] * a[1:]
    return w


def _jdiv(lam, y, dims):
    """Solve lam o x = y for x (inverse Jordan product)."""
    x = np.empty_like(y)
    x[: dims.l] = y[: dims.l] / lam[: dims.l]
    for off, d in dims.blocks():
        l0, l1 = lam[off], lam[off + 1 : off + d]
        y0, y1 = y[off], y[off + 1 : off + d]
        det = l0 * l0 - l1 @ l1
        x0 = (l0 * y0 - l1 @ y1) / det
        x[off] = x0
        x[off + 1 : off + d] = (y1 - x0 * l1) / l0
    return x


def _soc_jnorm(v):
    return np.sqrt(max((v[0] - np.linalg.norm(v[1:])) * (v[0] + np.linalg.norm(v[1:])), 0.0))


def _nt_scaling(s, z, dims):
    """Return dense W (symmetric) with W z = W^{-1} s = lambda, and W^{-1}."""
    m = dims.m
    W = np.zeros((m, m))
    Wi = np.zeros((m, m))
    d = np.sqrt(s[: dims.l] / z[: dims.l])
    W[np.arange(dims.l), np.arange(dims.l)] = d
    Wi[np.arange(dims.l), np.arange(dims.l)] = 1.0 / d
    for off, k in dims.blocks():
        sb, zb = s[off : off + k], z[off : off + k]
        sn, zn = _soc_jnorm(sb), _soc_jnorm(zb)
        ss, zz = sb / sn, zb / zn
        gam = np.sqrt(0.5 * (1.0 + ss @ zz))
        w = ss.copy()
        w[0] += zz[0]
        w[1:] -= zz[1:]
        w /= 2.0 * gam
        eta = np.sqrt(sn / zn)
        Hw = np.empty((k, k))
        Hw[0, 0] = w[0]
        Hw[0, 1:] = w[1:]
        Hw[1:, 0] = w[1:]
        Hw[1:, 1:] = np.eye(k - 1) + np.outer(w[1:], w[1:]) / (1.0 + w[0])
        Hwi = Hw.copy()
        Hwi[0, 1:] *= -1.0
        Hwi[1:, 0] *= -1.0
        W[off : off + k, off : off + k] = eta * Hw
        Wi[off : off + k, off : off + k] = Hwi / eta
    return W, Wi


def _max_step(x, dx, dims):
    """Largest a >= 0 with x + a dx in K (x interior); inf if unbounded."""
    amax = np.inf
    if dims.l:
        neg = dx[: dims.l] < 0
        if np.any(neg):
            amax = min(amax, np.min(-x[: dims.l][neg] / dx[: dims.l][neg]))
    for off, k in dims.blocks():
        x0, x1 = x[off], x[off + 1 : off + k]
        d0, d1 = dx[off], dx[off + 1 : off + k]
        a = d0 * d0 - d1 @ d1
        b = x0 * d0 - x1 @ d1
        c = (x0 - np.linalg.norm(x1)) * (x0 + np.linalg.norm(x1))
        disc = b * b - a * c
        if a < 0 or (b < 0 and disc >= 0):
            den = -b + np.sqrt(max(disc, 0.0))
            if den > 0:
                amax = min(amax, c / den)
            else:
                amax = 0.0
    return amax


def _min_eig(v, dims):
    mins = []
    if dims.l:
        mins.append(np.min(v[: dims.l]))
    for off, k in dims.blocks():
        mins.append(v[off] - np.linalg.norm(v[off + 1 : off + k]))
    return min(mins)


@dataclass
class IPMResult:
    x: np.ndarray
    s: np.ndarray
    z: np.ndarray
    y: np.ndarray
    status: int
    iters: int
    pres: float
    dres: float
    gap: float
    obj: float


def solve_qp(P, q, G, h, dims: ConeDims, A=None, b=None, tol=1e-11, max_iter=80) -> IPMResult:
    """Dense conic QP solve (see module docstring)."""
    n = P.shape[0]
    m = dims.m
    if A is None:
        A = np.zeros((0, n))
        b = np.zeros(0)
    p = A.shape[0]
    e = _e(dims)
    z0 = np.zeros(n)
    if not all(np.all(np.isfinite(v)) for v in (P, q, G, h, A, b)):
        # non-finite problem data: the solver errors out (the reference's exception branch)
        return IPMResult(z0, np.zeros(m), np.zeros(m), np.zeros(p), NUMERICAL, 0, np.nan, np.nan, np.nan, np.nan)
    zero_rows = ~np.any(G[: dims.l] != 0.0, axis=1)
    if np.any(zero_rows & (h[: dims.l] < 0.0)):
        # 0 <= h_j < 0 cannot hold: certificate of primal infeasibility without iterating
        return IPMResult(z0, np.zeros(m), np.zeros(m), np.zeros(p), INFEASIBLE, 0, np.inf, np.nan, np.nan, np.nan)

    # Initial point: least-squares KKT with W = I, then shift into the cone interior.
    K0 = np.zeros((n + p + m, n + p + m))
    K0[:n, :n] = P
    K0[:n, n : n + p] = A.T
    K0[:n, n + p :] = G.T
    K0[n : n + p, :n] = A
    K0[n + p :, :n] = G
    K0[n + p :, n + p :] = -np.eye(m)
    sol = np.linalg.lstsq(K0, np.concatenate([-q, b, h]), rcond=None)[0]
    x = sol[:n]
    y = sol[n : n + p]
    z = sol[n + p :].copy()
    s = -z.copy()
    ap = _min_eig(s, dims)
    if ap <= 0:
        s = s + (1.0 - ap) * e
    ad = _min_eig(z, dims)
    if ad <= 0:
        z = z + (1.0 - ad) * e

    nq = max(1.0, np.linalg.norm(q))
    nh = max(1.0, np.linalg.norm(np.concatenate([h, b])))
    status = MAX_ITER
    it = 0
    for it in range(max_iter + 1):
        rx = P @ x + q + A.T @ y + G.T @ z
        ry = A @ x - b
        rz = G @ x + s - h
        gap = s @ z
        mu = gap / dims.degree
        pobj = 0.5 * x @ P @ x + q @ x
        pres = max(np.linalg.norm(rz), np.linalg.norm(ry)) / nh
        dres = np.linalg.norm(rx) / nq
        if not np.all(np.isfinite([pres, dres, gap])):
            status = NUMERICAL
            break
        if pres < tol and dres < tol and gap < tol * max(1.0, abs(pobj)):
            status = OPTIMAL
            break
        if it == max_iter:
            break
        W, Wi = _nt_scaling(s, z, dims)
        lam = W @ z
        Gs = Wi @ G  # scaled constraint matrix W^{-1} G
        # Scaled augmented (quasi-definite) KKT system, as conic IPMs (ECOS/Clarabel) use:
        #   [P  A'  Gs'] [dx ]   [-rx        ]
        #   [A  0   0  ] [dy ] = [-ry        ]
        #   [Gs 0   -I ] [dzs]   [-W^{-1} t  ]      dzs = W dz,  t = rz - W (lam \ rs)
        KKT = np.zeros((n + p + m, n + p + m))
        KKT[:n, :n] = P
        KKT[:n, n : n + p] = A.T
        KKT[:n, n + p :] = Gs.T
        KKT[n : n + p, :n] = A
        KKT[n + p :, :n] = Gs
        KKT[n + p :, n + p :] = -np.eye(m)
        try:
            lu = np.linalg.inv(KKT)
        except np.linalg.LinAlgError:
            status = NUMERICAL
            break

        def newton(rs):
            t = rz - W @ _jdiv(lam, rs, dims)
            rhs = np.concatenate([-rx, -ry, -(Wi @ t)])
            d = lu @ rhs
            for _ in range(2):  # iterative refinement
                d = d + lu @ (rhs - KKT @ d)
            dx, dy = d[:n], d[n : n + p]
            dz = Wi @ d[n + p :]
            ds = -rz - G @ dx
            return dx, dy, dz, ds

        ls = _jprod(lam, lam, dims)
        dx, dy, dz, ds = newton(ls)
        dsl = Wi @ ds
        dzl = W @ dz
        a_aff = min(1.0, _max_step(lam, dsl, dims), _max_step(lam, dzl, dims))
        sig = ((s + a_aff * ds) @ (z + a_aff * dz) / gap) ** 3
        rs = ls + _jprod(dsl, dzl, dims) - sig * mu * e
        dx, dy, dz, ds = newton(rs)
        dsl = Wi @ ds
        dzl = W @ dz
        amax = min(_max_step(lam, dsl, dims), _max_step(lam, dzl, dims))
        alpha = min(1.0, 0.99 * amax)
        # Safeguard: on a (nearly) feasible iterate Mehrotra's corrector can increase the gap and
        # cycle; backtrack until the complementarity gap decreases.
        if pres < 1e-8 and dres < 1e-8:
            for _ in range(8):
                if (lam + alpha * dsl) @ (lam + alpha * dzl) <= gap * (1.0 - 0.01 * alpha):
                    break
                alpha *= 0.5
        x = x + alpha * dx
        y = y + alpha * dy
        z = z + alpha * dz
        s = s + alpha * ds
    rx = P @ x + q + A.T @ y + G.T @ z
    rz = G @ x + s - h
    return IPMResult(
        x=x,
        s=s,
        z=z,
        y=y,
        status=status,
        iters=it,
        pres=float(max(np.linalg.norm(rz), np.linalg.norm(A @ x - b)) if m or p else 0.0),
        dres=float(np.linalg.norm(rx)),
        gap=float(s @ z),
        obj=float(0.5 * x @ P @ x + q @ x),
    )


def cone_violation(s, dims: ConeDims) -> float:
    """Largest violation of s in K (0 when feasible)."""
    v = 0.0
    if dims.l:
        v = max(v, float(np.max(-s[: dims.l], initial=0.0)))
    for off, k in dims.blocks():
        v = max(v, float(np.linalg.norm(s[off + 1 : off + k]) - s[off]))
    return v
