"""ORACLE (test infrastructure only) -- CPU restatement of the reference's hot-path math.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package.  Every function cites the reference lines it restates
(paths relative to the reference repository root).

Contents
  * Lie-group helpers (the four pinocchio ops the path uses: skew, skewSquare, exp3,
    unSkew -- closed forms, ``control/rqp_*.py`` and ``system/rigid_quadrotor_payload.py``)
  * ``Params``      -- RQPParameters derived constants   (system/rigid_quadrotor_payload.py:48-84)
  * ``State``       -- RQPState + integrate/project_R    (system/rigid_quadrotor_payload.py:87-148)
  * ``forward_dynamics`` / ``inverse_dynamics_error``     (system/rigid_quadrotor_payload.py:173-269)
  * ``low_level_control`` (SO(3) PD)  (control/rqp_centralized.py:503-535, utils/so3_tracking_controllers.py:18-43)
  * ``equilibrium_forces``            (control/rqp_cadmm.py:165-174)
  * ``Consts``      -- controller constants               (control/rqp_cadmm.py:192-236 etc.)
  * ``build_qp``    -- the exact (uncondensed) conic QP each controller hands to cvxpy
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
from scipy.linalg import polar

from .ipm import ConeDims

G = 9.80665  # scipy.constants.g
E3 = np.array([0.0, 0.0, 1.0])


# ----------------------------------------------------------------------------- Lie helpers
def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def skew_sq(u, v):
    """pinocchio.skewSquare(u, v) = skew(u) @ skew(v)."""
    return skew(u) @ skew(v)


def unskew(M):
    return np.array([M[2, 1], M[0, 2], M[1, 0]])


def exp3(v):
    """Rodrigues formula with the small-angle series (pinocchio.exp3)."""
    t2 = v @ v
    t = np.sqrt(t2)
    if t < 1e-4:
        a = 1.0 - t2 / 6.0 + t2 * t2 / 120.0
        b = 0.5 - t2 / 24.0 + t2 * t2 / 720.0
    else:
        a = np.sin(t) / t
        b = (1.0 - np.cos(t)) / t2
    K = skew(v)
    return np.eye(3) + a * K + b * (K @ K)


# ----------------------------------------------------------------------------- parameters
class Params:
    """RQPParameters (system/rigid_quadrotor_payload.py:48-84)."""

    def __init__(self, m, J, ml, Jl, r):
        self.n = r.shape[1]
        self.m = np.asarray(m, float)
        self.J = np.asarray(J, float)
        self.ml = float(ml)
        self.Jl = np.asarray(Jl, float)
        self.r = np.asarray(r, float)
        self.mT = np.sum(self.m) + self.ml
        self.x_com = np.sum(self.r * self.m, axis=1) / self.mT
        self.r_com = (self.r.T - self.x_com).T
        JT = self.Jl - self.ml * skew_sq(self.x_com, self.x_com)
        for i in range(self.n):
            JT = JT - self.m[i] * skew_sq(self.r_com[:, i], self.r_com[:, i])
        self.JT = JT
        self.JT_inv = np.linalg.inv(JT)
        self.J_inv = np.stack([np.linalg.inv(self.J[:, :, i]) for i in range(self.n)], axis=2)


def collision_radius(payload_mesh_vertices, quad_radius=0.3):
    """RQPCollision.collision_radius (system/rigid_quadrotor_payload.py:302-306)."""
    return float(np.max(np.linalg.norm(payload_mesh_vertices, axis=1)) + quad_radius + 0.1)


MAX_DECELERATION = G / 5.0  # system/rigid_quadrotor_payload.py:310


def equilibrium_forces(p: Params) -> np.ndarray:
    """f_eq (control/rqp_cadmm.py:165-174): min-norm lstsq of [1'; skew(r_com_i)[:2,2]] f_z = [mT g,0,0]."""
    W = np.empty((3, p.n))
    W[0, :] = 1.0
    for i in range(p.n):
        W[1:, i] = skew(p.r_com[:, i])[:2, 2]
    f_eq = np.zeros((3, p.n))
    f_eq[2, :] = np.linalg.lstsq(W, np.array([p.mT * G, 0.0, 0.0]), rcond=None)[0]
    return f_eq


# ----------------------------------------------------------------------------- state & dynamics
class State:
    """RQPState (system/rigid_quadrotor_payload.py:87-148)."""

    STEPS_PER_PROJECTION = 20

    def __init__(self, R, w, xl, vl, Rl, wl, project=True):
        self.n = w.shape[1]
        self.R = np.array(R, float)
        self.w = np.array(w, float)
        self.xl = np.array(xl, float)
        self.vl = np.array(vl, float)
        self.Rl = np.array(Rl, float)
        self.wl = np.array(wl, float)
        if project:
            self.project_R()
        self.counter = 0

    def copy(self):
        s = State(self.R, self.w, self.xl, self.vl, self.Rl, self.wl, project=False)
        s.counter = self.counter
        return s

    def project_R(self):
        self.Rl, _ = polar(self.Rl)
        for i in range(self.n):
            self.R[:, :, i], _ = polar(self.R[:, :, i])

    def integrate(self, dw, dvl, dwl, dt):
        for i in range(self.n):
            self.R[:, :, i] = self.R[:, :, i] @ exp3((self.w[:, i] + dw[:, i] * dt / 2) * dt)
            self.w[:, i] = self.w[:, i] + dw[:, i] * dt
        self.xl = self.xl + self.vl * dt + dvl * dt**2 / 2
        self.vl = self.vl + dvl * dt
        self.Rl = self.Rl @ exp3((self.wl + dwl * dt / 2) * dt)
        self.wl = self.wl + dwl * dt
        self.counter += 1
        if self.counter >= self.STEPS_PER_PROJECTION:
            self.project_R()
            self.counter = 0


def forward_dynamics(p: Params, s: State, f, M):
    """RQPDynamics.forward_dynamics (system/rigid_quadrotor_payload.py:173-222)."""
    n = p.n
    dw = np.empty((3, n))
    for i in range(n):
        dw[:, i] = p.J_inv[:, :, i] @ (M[:, i] - skew(s.w[:, i]) @ p.J[:, :, i] @ s.w[:, i])
    quad_force = s.R[:, 2, :] * f
    dv_com = np.sum(quad_force, axis=1) / p.mT - G * E3
    net_moment = np.sum(np.cross(p.r_com, s.Rl.T @ quad_force, axisa=0, axisb=0, axisc=0), axis=1)
    dwl = p.JT_inv @ (net_moment - skew(s.wl) @ p.JT @ s.wl)
    dvl = dv_com - s.Rl @ (skew_sq(s.wl, s.wl) + skew(dwl)) @ p.x_com
    return dw, dvl, dwl


def inverse_dynamics_error(s: State, p: Params, f, M, dw, dvl, dwl):
    """RQPDynamics.inverse_dynamics_error (system/rigid_quadrotor_payload.py:224-269)."""
    gvec = -G * E3
    dv_quad = dvl[:, None] + s.Rl @ (skew_sq(s.wl, s.wl) + skew(dwl)) @ p.r
    internal = s.R[:, 2, :] * f + gvec[:, None] * p.m - p.m * dv_quad
    e1 = np.linalg.norm(p.ml * dvl - p.ml * gvec - np.sum(internal, axis=1))
    lm = np.sum(np.cross(p.r, s.Rl.T @ internal, axisa=0, axisb=0, axisc=0), axis=1)
    e2 = np.linalg.norm(p.Jl @ dwl + skew(s.wl) @ p.Jl @ s.wl - lm)
    e3 = 0.0
    for i in range(p.n):
        e3 += np.linalg.norm(p.J[:, :, i] @ dw[:, i] + skew(s.w[:, i]) @ p.J[:, :, i] @ s.w[:, i] - M[:, i]) ** 2
    return float(np.sqrt(e1**2 + e2**2 + e3))


def rotation_from_unit_vector(q):
    """RQPLowLevelController._rotation_from_unit_vector (control/rqp_centralized.py:503-516)."""
    R = np.empty((3, 3))
    sin_x = -q[1]
    cos_x = np.sqrt(q[0] ** 2 + q[2] ** 2)
    sin_y = q[0] / cos_x
    cos_y = q[2] / cos_x
    R[0, 0], R[1, 0], R[2, 0] = cos_y, 0.0, -sin_y
    R[0, 1], R[1, 1], R[2, 1] = sin_x * sin_y, cos_x, cos_y * sin_x
    R[:, 2] = q
    return R


K_R_PD, K_OMEGA_PD = 0.25, 0.075  # control/rqp_centralized.py:488-489


SM_R, SM_K_R, SM_L_R, SM_K_S, SM_L_S = 0.5, 1.415, 0.707, 0.113, 0.057  # control/rqp_centralized.py:491-496


def so3_sm(R, Rd, w, J):
    """so3_sm_tracking_control with wd = dwd = 0 (utils/so3_tracking_controllers.py:52-95), including
    the reference's call T(e_R, r) (:92) against the definition T = lambda r, y (:87-88): the diagonal
    is (|r| + 1e-6)^(e_R - 1), i.e. the arguments are swapped relative to the paper."""
    e_R = 0.5 * unskew(Rd.T @ R - R.T @ Rd)
    e_W = w
    E = 0.5 * (np.trace(R.T @ Rd) * np.eye(3) - R.T @ Rd)
    S = lambda r, y: np.power(np.abs(y), r) * np.sign(y)  # noqa: E731
    s = e_W + SM_K_R * e_R + SM_L_R * S(SM_R, e_R)
    T = lambda r, y: np.diag(np.power(np.abs(y) + 1e-6, r - 1))  # noqa: E731
    return (-SM_K_S * s - SM_L_S * S(SM_R, s) + np.cross(w, J @ w)
            - (SM_K_R * J + SM_L_S * SM_R * (J @ T(e_R, SM_R))) @ E @ e_W)


def low_level_control(p: Params, s: State, f_des, kind: str = "pd"):
    """RQPLowLevelController.control with the 'pd' (utils/so3_tracking_controllers.py:18-43) or 'sm'
    (:52-95) SO(3) law, wd = dwd = 0 (control/rqp_centralized.py:518-535)."""
    n = p.n
    f = np.zeros(n)
    M = np.zeros((3, n))
    for i in range(n):
        f[i] = f_des[:, i] @ s.R[:, 2, i]
        qd = f_des[:, i] / np.linalg.norm(f_des[:, i])
        Rd = rotation_from_unit_vector(qd)
        R = s.R[:, :, i]
        w = s.w[:, i]
        if kind == "sm":
            M[:, i] = so3_sm(R, Rd, w, p.J[:, :, i])
            continue
        e_R = 0.5 * unskew(Rd.T @ R - R.T @ Rd)
        M[:, i] = -K_R_PD * e_R - K_OMEGA_PD * w + np.cross(w, p.J[:, :, i] @ w)
    return f, M


# ----------------------------------------------------------------------------- controller constants
@dataclass
class Consts:
    """Controller constants (control/rqp_centralized.py:182-225; control/rqp_cadmm.py:192-236;
    control/rqp_dd.py:197-241)."""

    n: int
    mT: float
    min_fz: float
    max_f_ang: float
    sec_max_f_ang: float
    max_f: float
    cos_max_p_ang: float
    max_wl_sq: float
    max_vl_sq: float
    dist_eps: float
    vision_radius: float
    vision_cone_ang: float
    nenv_cbfs: int
    max_deceleration: float
    alpha_env: float
    k_f: float
    k_m: float
    k_feq: float

    @staticmethod
    def make(p: Params, col_radius: float, distributed: bool) -> "Consts":
        n = p.n
        return Consts(
            n=n,
            mT=p.mT,
            min_fz=p.mT * G / (n * 10.0),
            max_f_ang=np.pi / 6.0,
            sec_max_f_ang=1.0 / np.cos(np.pi / 6.0),
            max_f=(2.0 / n) * p.mT * G,
            cos_max_p_ang=np.cos(np.pi / 12.0),
            max_wl_sq=(np.pi / 6.0) ** 2,
            max_vl_sq=1.0,
            dist_eps=0.1,
            vision_radius=col_radius + 5.0,
            vision_cone_ang=100.0 * np.pi / 180.0,
            nenv_cbfs=10,
            max_deceleration=MAX_DECELERATION,
            alpha_env=1.5 if distributed else 2.0,
            k_f=0.1 / n if distributed else 0.1,
            k_m=0.1 / n if distributed else 0.1,
            k_feq=0.1,
        )


# ----------------------------------------------------------------------------- QP assembly
class _QPBuilder:
    """Accumulates cost/constraints of a cvxpy-shaped problem over a flat variable vector."""

    def __init__(self, nx):
        self.nx = nx
        self.P = np.zeros((nx, nx))
        self.q = np.zeros(nx)
        self.A, self.b = [], []
        self.Gl, self.hl = [], []
        self.Gq, self.hq = [], []

    def sum_squares(self, k, Amat, c):
        """k * ||Amat x + c||^2  ->  1/2 x'(2k A'A)x + (2k A'c)'x."""
        self.P += 2.0 * k * Amat.T @ Amat
        self.q += 2.0 * k * Amat.T @ c

    def linear(self, c):
        self.q += c

    def eq(self, Amat, rhs):
        self.A.append(Amat)
        self.b.append(rhs)

    def ge(self, a, beta):
        """a'x + beta >= 0  ->  -a'x + s = beta, s >= 0."""
        self.Gl.append(-a)
        self.hl.append(beta)

    def soc(self, Gq, hq):
        """(hq - Gq x) in Q^k  (caller passes the cone rows in s = h - Gx form)."""
        self.Gq.append(Gq)
        self.hq.append(hq)

    def finish(self):
        G_ = np.vstack([np.array(self.Gl).reshape(-1, self.nx)] + self.Gq)
        h_ = np.concatenate([np.array(self.hl, float)] + self.hq)
        dims = ConeDims(l=len(self.Gl), q=[g.shape[0] for g in self.Gq])
        return self.P, self.q, G_, h_, dims, np.vstack(self.A), np.concatenate(self.b)


@dataclass
class EnvRows:
    """Environment CBF rows: lhs (10,3) @ dvl >= rhs (10,)  (control/rqp_cadmm.py:432-433)."""

    lhs: np.ndarray
    rhs: np.ndarray
    collision: bool
    min_env_dist: float

    @staticmethod
    def empty(c: Consts) -> "EnvRows":
        # control/rqp_cadmm.py:308-317: no env -> zero lhs, rhs = -alpha (vision_r - eps)
        return EnvRows(
            np.zeros((c.nenv_cbfs, 3)),
            -c.alpha_env * (c.vision_radius - c.dist_eps) * np.ones(c.nenv_cbfs),
            False,
            c.vision_radius,
        )


def _state_terms(p: Params, s: State):
    R_w_hat = s.Rl @ skew(s.wl)
    R_w_hat_sq = s.Rl @ skew_sq(s.wl, s.wl)
    J_inv_w_cross_Jw = p.JT_inv @ np.cross(s.wl, p.JT @ s.wl)
    return R_w_hat, R_w_hat_sq, J_inv_w_cross_Jw


def build_qp(kind: str, p: Params, c: Consts, s: State, acc_des, env: EnvRows, i: int = 0,
             f_eq=None, lam=None, rho=0.0, f_mean=None, c_fi=None, c_Fi=None, c_Mi=None):
    """The exact (uncondensed) conic QP a controller hands to cvxpy.

    kind = "centralized"  control/rqp_centralized.py:340-425  vars (dv_com, dvl, dwl, f[3,n] col-major)
    kind = "cadmm"        control/rqp_cadmm.py:376-471       vars (dv_com, dvl, dwl, f[3,n] col-major)
    kind = "dd"           control/rqp_dd.py:379-460          vars (dv_com, dvl, dwl, fi, Fi, Mi)
    Returns (P, q, G, h, dims, A, b); variable offsets: dv_com 0:3, dvl 3:6, dwl 6:9, rest 9:.
    """
    n = p.n
    dvl_des, dwl_des = acc_des
    leader = i == 0
    R_w_hat, R_w_hat_sq, c_w = _state_terms(p, s)
    nf = 3 * n if kind != "dd" else 9
    nx = 9 + nf
    B = _QPBuilder(nx)
    I3 = np.eye(3)

    def sel(off):
        S = np.zeros((3, nx))
        S[:, off : off + 3] = I3
        return S

    DVC, DVL, DWL = sel(0), sel(3), sel(6)
    if kind == "dd":
        FI, FF, MM = sel(9), sel(12), sel(15)
        F_sum = FI + FF                                            # fi + Fi
        Mo = skew(p.r_com[:, i]) @ s.Rl.T @ FI + MM                # r_i x Rl'fi + Mi
        Jmo = p.JT_inv @ skew(p.r_com[:, i]) @ s.Rl.T @ FI + p.JT_inv @ MM
        cone_blocks = [FI]
    else:
        Fj = [sel(9 + 3 * j) for j in range(n)]
        F_sum = sum(Fj)
        Mo = sum(skew(p.r_com[:, j]) @ s.Rl.T @ Fj[j] for j in range(n))
        Jmo = sum(p.JT_inv @ skew(p.r_com[:, j]) @ s.Rl.T @ Fj[j] for j in range(n))
        cone_blocks = Fj if kind == "centralized" else [Fj[i]]

    # Dynamics & kinematics equalities (rqp_cadmm.py:376-392).
    B.eq(p.mT * DVC - F_sum, -p.mT * G * E3)
    B.eq(DWL - Jmo, -c_w)
    B.eq(DVL - DVC - s.Rl @ skew(p.x_com) @ DWL, -R_w_hat_sq @ p.x_com)

    # Agent-local force constraints (rqp_cadmm.py:394-404).
    for Fb in cone_blocks:
        B.ge(Fb[2], -c.min_fz)
        B.soc(-np.vstack([c.sec_max_f_ang * Fb[2], Fb]), np.zeros(4))
        B.soc(-np.vstack([np.zeros(nx), Fb]), np.array([c.max_f, 0.0, 0.0, 0.0]))
    # Payload angle / angular-velocity / velocity CBFs (rqp_cadmm.py:406-430).
    e3R = E3 @ s.Rl @ skew(E3)
    B.ge(-(e3R @ DWL), R_w_hat_sq[2, 2] + 2.0 * R_w_hat[2, 2] + (s.Rl[2, 2] - c.cos_max_p_ang))
    B.ge(-2.0 * s.wl @ DWL, c.max_wl_sq - s.wl @ s.wl)
    B.ge(-2.0 * s.vl @ DVL, c.max_vl_sq - s.vl @ s.vl)
    for k in range(c.nenv_cbfs):
        a = env.lhs[k] @ DVL
        if np.any(a != 0.0) or env.rhs[k] != 0.0:
            # a 0 >= 0 row carries no information; it is dropped (it cannot change the optimum)
            B.ge(a, -env.rhs[k])

    # Costs.
    if kind == "dd":
        B.sum_squares(c.k_f, F_sum, -p.mT * G * E3)
        B.sum_squares(c.k_m, Mo, np.zeros(3))
        B.sum_squares(c.k_feq, FI, -f_eq[:, i])
    else:
        B.sum_squares(c.k_f, F_sum, -p.mT * G * E3)
        B.sum_squares(c.k_m, Mo, np.zeros(3))
        if kind == "centralized":
            for j in range(n):
                B.sum_squares(c.k_feq, Fj[j], -f_eq[:, j])
        else:
            B.sum_squares(c.k_feq, Fj[i], -f_eq[:, i])
    k_dvl = 1.0 if (kind == "centralized" or leader) else 0.0
    k_dwl = k_dvl
    if k_dvl:
        B.sum_squares(k_dvl, DVL, np.zeros(3))
        B.linear(-2.0 * k_dvl * DVL.T @ dvl_des)
        B.sum_squares(k_dwl, DWL, np.zeros(3))
        B.linear(-2.0 * k_dwl * DWL.T @ dwl_des)
    if kind == "cadmm":
        # <lambda, f> + (rho/2)||f||^2 - <rho f_mean, f>   (rqp_cadmm.py:465-471)
        q = np.zeros(nx)
        q[9:] = lam.reshape(-1, order="F") - (rho * f_mean).reshape(-1, order="F")
        B.linear(q)
        B.P[9:, 9:] += rho * np.eye(nf)
    if kind == "dd":
        B.linear(c_fi @ FI + c_Fi @ FF + c_Mi @ MM)
    return B.finish()
