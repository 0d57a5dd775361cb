"""ORACLE (test infrastructure only) -- the three high-level controllers' outer loops.

Restates, step for step:
  * RQPCentralizedController.control      control/rqp_centralized.py:436-448
  * RQPCADMMController.control            control/rqp_cadmm.py:569-675 (+ RQPPrimalSolver.solve :482-501)
  * RQPDDController.control               control/rqp_dd.py:618-752  (+ RQPPrimalSolver.solve :475-505,
                                          strong_convexity_matrix :513-555)
with every per-step QP answered by ``oracle.ipm.solve_qp`` on the uncondensed problem
``oracle.model.build_qp`` -- the problem cvxpy would hand to Clarabel.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
from scipy.linalg import cho_factor, cho_solve

from . import forest as _forest
from .ipm import NUMERICAL, OPTIMAL, solve_qp
from .model import Consts, EnvRows, Params, State, build_qp, equilibrium_forces, exp3, skew


@dataclass
class SolverStatistics:
    """control/rqp_centralized.py:18-24."""

    iter: int
    solve_time: float
    collision: bool
    min_env_dist: float
    err_seq: list = field(default_factory=list)


def _env(forest, c, s, col_r, r_i):
    if forest is None:
        return EnvRows.empty(c)
    return _forest.env_rows(forest, c, s, col_r, r_i)


class Centralized:
    def __init__(self, p: Params, col_r: float, forest=None):
        self.p, self.col_r, self.forest = p, col_r, forest
        self.c = Consts.make(p, col_r, distributed=False)
        self.f_eq = equilibrium_forces(p)
        self.prev_f = self.f_eq.copy()
        self.last = None

    def control(self, s: State, acc_des):
        env = _env(self.forest, self.c, s, self.col_r, None)
        P, q, G, h, dims, A, b = build_qp("centralized", self.p, self.c, s, acc_des, env, f_eq=self.f_eq)
        r = solve_qp(P, q, G, h, dims, A, b)
        self.last = r
        if r.status == OPTIMAL:
            self.prev_f = r.x[9:].reshape((3, self.p.n), order="F")
        return self.prev_f.copy(), SolverStatistics(-1, 0.0, env.collision, env.min_env_dist)


class CADMM:
    """Consensus ADMM (control/rqp_cadmm.py:510-688)."""

    def __init__(self, p: Params, col_r: float, forest=None):
        self.p, self.col_r, self.forest = p, col_r, forest
        n = p.n
        self.n = n
        self.c = Consts.make(p, col_r, distributed=True)
        self.f_eq = equilibrium_forces(p)
        self.res_tol, self.use_total_res, self.max_iter = 1e-2, True, 100
        self.rho0, self.tau_incr, self.rho_max = 1.0, 1.0, 2.0
        self.f = np.stack([self.f_eq] * n, axis=2)          # (3, n, n): f[:, :, i] agent i's copy
        self.f_mean = self.f_eq.copy()
        self.lam = np.zeros((3, n, n))
        self.prev_f = [self.f_eq.copy() for _ in range(n)]   # RQPPrimalSolver.prev_f
        self.qp_iters = []

    def set_force_err_tolerance(self, tol, use_total_res=True):
        self.res_tol, self.use_total_res = tol, use_total_res

    def set_max_iter(self, k):
        self.max_iter = k

    def solve_agent(self, i, s, acc_des, env, rho):
        P, q, G, h, dims, A, b = build_qp("cadmm", self.p, self.c, s, acc_des, env, i=i, f_eq=self.f_eq,
                                          lam=self.lam[:, :, i], rho=rho, f_mean=self.f_mean)
        r = solve_qp(P, q, G, h, dims, A, b)
        self.qp_iters.append(r.iters)
        if r.status == NUMERICAL:
            self.prev_f[i] = self.f_eq.copy()
        elif r.status == OPTIMAL:
            self.prev_f[i] = r.x[9:].reshape((3, self.n), order="F")
        return self.prev_f[i], r

    def mean_and_residual(self, s: State):
        n = self.n
        f_mean = np.zeros((3, n))
        for i in range(n):
            f_mean += self.f[:, :, i]
        f_mean = f_mean / n
        total_res = 0.0
        for i in range(n):
            total_res = max(total_res, np.linalg.norm(self.f[:, :, i] - f_mean, np.inf))
        if self.use_total_res:
            return f_mean, total_res
        # aggregate residual (control/rqp_cadmm.py:602-621)
        f_app = np.stack([self.f[:, i, i] for i in range(n)], axis=1)
        F = np.empty((3, n))
        M = np.empty((3, n))
        for i in range(n):
            F[:, i] = np.sum(self.f[:, :, i], axis=1) - self.f[:, i, i]
            mom = np.cross(self.p.r_com, s.Rl.T @ self.f[:, :, i], axisa=0, axisb=0, axisc=0)
            M[:, i] = np.sum(mom, axis=1) - mom[:, i]
        mom_app = np.cross(self.p.r_com, s.Rl.T @ f_app, axisa=0, axisb=0, axisc=0)
        eF = np.empty((3, n))
        eM = np.empty((3, n))
        for i in range(n):
            eF[:, i] = F[:, i] - (np.sum(f_app, axis=1) - f_app[:, i])
            eM[:, i] = M[:, i] - (np.sum(mom_app, axis=1) - mom_app[:, i])
        return f_mean, max(np.linalg.norm(eF, np.inf), np.linalg.norm(eM, np.inf))

    def control(self, s: State, acc_des):
        n = self.n
        envs = [_env(self.forest, self.c, s, self.col_r, self.p.r[:, i]) for i in range(n)]
        it = 0
        rho = self.rho0
        err_seq = []
        collision = False
        min_env_dist = self.c.vision_radius
        while True:
            for i in range(n):
                fi, _ = self.solve_agent(i, s, acc_des, envs[i], rho)
                self.f[:, :, i] = fi
                collision = collision or envs[i].collision
                min_env_dist = min(min_env_dist, envs[i].min_env_dist)
            it += 1
            rho = min(rho * self.tau_incr, self.rho_max)
            self.f_mean, res = self.mean_and_residual(s)
            if res < self.res_tol or it > self.max_iter:
                break
            err_seq.append(res)
            for i in range(n):
                self.lam[:, :, i] += rho * (self.f[:, :, i] - self.f_mean)
        f_app = np.stack([self.f[:, i, i] for i in range(n)], axis=1)
        return f_app, SolverStatistics(it, 0.0, collision, min_env_dist, err_seq)


class DD:
    """Dual decomposition (control/rqp_dd.py:558-764)."""

    def __init__(self, p: Params, col_r: float, forest=None, dt: float = 1e-3):
        self.p, self.col_r, self.forest, self.dt = p, col_r, forest, dt
        n = p.n
        self.n = n
        self.c = Consts.make(p, col_r, distributed=True)
        self.f_eq = equilibrium_forces(p)
        self.prim_inf_tol, self.max_iter, self.beta = 1e-2, 100, 0.0
        self.lam_F = np.zeros((3, n))
        self.lam_M = np.zeros((3, n))
        # warm start (control/rqp_dd.py:628-632): f aliases solver-0's f_eq (quirk a15)
        self.f = self.f_eq.copy()
        fi0 = self.f_eq[:, 0]
        F0 = np.sum(self.f_eq, axis=1) - fi0
        M0 = -p.JT_inv @ skew(p.r_com[:, 0]) @ fi0
        self.F = np.stack([F0] * n, axis=1)
        self.M = np.stack([M0] * n, axis=1)
        self.prev = []
        for i in range(n):
            fi = self.f_eq[:, i].copy()
            self.prev.append((fi, np.sum(self.f_eq, axis=1) - fi, -p.JT_inv @ skew(p.r_com[:, i]) @ fi))
        self.qp_iters = []

    def set_force_err_tolerance(self, tol):
        self.prim_inf_tol = tol

    def set_max_iter(self, k):
        self.max_iter = k

    def strong_convexity_matrix(self, i, s: State):
        """control/rqp_dd.py:513-555 (k_smooth = 0 term omitted: it is identically zero)."""
        p, c = self.p, self.c
        mat = 1e-6 * np.eye(9)
        t = np.zeros((3, 9))
        t[:, :3] = np.eye(3)
        mat += 2 * c.k_feq * (t.T @ t)
        t[:, 3:6] = np.eye(3)
        mat += 2 * c.k_f * (t.T @ t)
        t[:, :3] = skew(p.r_com[:, i]) @ s.Rl.T
        t[:, 3:6] = 0.0
        t[:, 6:] = np.eye(3)
        mat += 2 * c.k_m * (t.T @ t)
        leader = 1.0 if i == 0 else 0.0
        cdwl_f = p.JT_inv @ skew(p.r_com[:, i]) @ s.Rl.T
        t[:, :3] = cdwl_f
        t[:, 3:6] = 0.0
        t[:, 6:] = p.JT_inv
        mat += 2 * leader * (t.T @ t)
        t[:, :3] = np.eye(3) / p.mT + s.Rl @ skew(p.x_com) @ cdwl_f
        t[:, 3:6] = np.eye(3) / p.mT
        t[:, 6:] = s.Rl @ skew(p.x_com) @ p.JT_inv
        mat += 2 * leader * (t.T @ t)
        return mat

    def qn_matrix(self, s: State):
        """H = A Q^-1 A' (control/rqp_dd.py:634-657)."""
        n, p = self.n, self.p
        Qinv = np.zeros((9 * n, 9 * n))
        for i in range(n):
            Qi = np.linalg.inv(self.strong_convexity_matrix(i, s))
            Qinv[9 * i : 9 * i + 9, 9 * i : 9 * i + 9] = 0.5 * (Qi + Qi.T)
        A = np.zeros((6 * n, 9 * n))
        for i in range(n):
            A[6 * i : 6 * i + 3, 9 * i + 3 : 9 * i + 6] = np.eye(3)
            A[6 * i + 3 : 6 * i + 6, 9 * i + 6 : 9 * i + 9] = np.eye(3)
            for j in range(n):
                if j == i:
                    continue
                A[6 * i : 6 * i + 3, 9 * j : 9 * j + 3] = -np.eye(3)
                A[6 * i + 3 : 6 * i + 6, 9 * j : 9 * j + 3] = -skew(p.r_com[:, j]) @ s.Rl.T
        return A, A @ Qinv @ A.T + self.beta * np.eye(6 * n)

    def primal_inf_err(self, s: State):
        n = self.n
        mom = np.cross(self.p.r_com, s.Rl.T @ self.f, axisa=0, axisb=0, axisc=0)
        eF = np.empty((3, n))
        eM = np.empty((3, n))
        for i in range(n):
            eF[:, i] = self.F[:, i] - (np.sum(self.f, axis=1) - self.f[:, i])
            eM[:, i] = self.M[:, i] - (np.sum(mom, axis=1) - mom[:, i])
        return max(np.linalg.norm(eF, np.inf), np.linalg.norm(eM, np.inf))

    def solve_agent(self, i, s, acc_des, env, cf, cF, cM):
        P, q, G, h, dims, A, b = build_qp("dd", self.p, self.c, s, acc_des, env, i=i, f_eq=self.f_eq,
                                          c_fi=cf, c_Fi=cF, c_Mi=cM)
        r = solve_qp(P, q, G, h, dims, A, b)
        self.qp_iters.append(r.iters)
        if r.status == NUMERICAL:
            # exception -> equilibrium forces (control/rqp_dd.py:484-489).  Quirk a15: the
            # controller's f IS solver 0's f_eq (control/rqp_dd.py:629, written in place at :725), so
            # agent 0's fallback F_0 = sum of the controller's current f - fi_eq (fi_eq itself is a
            # separate array, :173,181); the other agents read their own, unaliased f_eq.
            fi = self.f_eq[:, i].copy()
            fsum = np.sum(self.f, axis=1) if i == 0 else np.sum(self.f_eq, axis=1)
            self.prev[i] = (fi, fsum - fi, -self.p.JT_inv @ skew(self.p.r_com[:, i]) @ fi)
        elif r.status == OPTIMAL:
            self.prev[i] = (r.x[9:12].copy(), r.x[12:15].copy(), r.x[15:18].copy())
        return self.prev[i], r

    def control(self, s: State, acc_des):
        n = self.n
        A, H = self.qn_matrix(s)
        chol = cho_factor(H)
        envs = [_env(self.forest, self.c, s, self.col_r, self.p.r[:, i]) for i in range(n)]
        it = 0
        err_seq = []
        collision = False
        min_env_dist = self.c.vision_radius
        while True:
            for i in range(n):
                cF = self.lam_F[:, i]
                cM = self.lam_M[:, i]
                cf = -(np.sum(self.lam_F, axis=1) - cF) + s.Rl @ skew(self.p.r_com[:, i]) @ (
                    np.sum(self.lam_M, axis=1) - cM)
                (fi, Fi, Mi), _ = self.solve_agent(i, s, acc_des, envs[i], cf, cF, cM)
                self.f[:, i], self.F[:, i], self.M[:, i] = fi, Fi, Mi
                collision = collision or envs[i].collision
                min_env_dist = min(min_env_dist, envs[i].min_env_dist)
            it += 1
            err = self.primal_inf_err(s)
            if err < self.prim_inf_tol or it > self.max_iter:
                break
            err_seq.append(err)
            x = np.empty((9, n))
            x[:3], x[3:6], x[6:] = self.f, self.F, self.M
            step = cho_solve(chol, A @ x.reshape(9 * n, order="F")).reshape((6, n), order="F")
            self.lam_F += step[:3]
            self.lam_M += step[3:]
        return self.f.copy(), SolverStatistics(it, 0.0, collision, min_env_dist, err_seq)


def desired_acceleration_forest(s: State, forest, x_offset=1.5):
    """_desired_acceleration_forest (example/rqp_example.py:33-59)."""
    x_ref = np.zeros(3)
    x_ref[0] = s.xl[0] + x_offset
    norm = np.linalg.norm(s.xl[:2] - forest.mountain_center)
    if norm >= forest.mountain_radius:
        x_ref[2] = 1.5
    else:
        x_ref[2] = np.sqrt(forest.mountain_sphere_radius**2 - norm**2) - forest.mountain_center_depth + 1.5
    v_ref = np.array([0.5, 0.0, 0.0])
    dvl = -(s.vl - v_ref) - (s.xl - x_ref)
    nrm = np.linalg.norm(dvl)
    if nrm > 0:
        dvl = dvl / nrm * min(nrm, 1.0)
    return (dvl, np.zeros(3)), x_ref, v_ref


__all__ = ["Centralized", "CADMM", "DD", "SolverStatistics", "desired_acceleration_forest", "exp3"]
