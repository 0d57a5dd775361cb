"""Host-side system description: the reference's RQP data types and their packing into the
fixed-shape fp64 blocks the HIP library consumes (``csrc/dat_layout.h``).

Mirrors ``system/rigid_quadrotor_payload.py`` of the reference:
  * ``RQPParameters``  (:48-84)  derived mass/inertia constants
  * ``RQPState``       (:87-148) state container (+ host-side polar projection at construction)
  * ``RQPCollision``   (:279-310) collision radius / max deceleration (display meshes dropped)
Batched variants carry a leading scenario axis.  The dynamics themselves run on the GPU
(``RQPDynamics`` / ``BatchRollout`` in ``control.py``).
"""

from __future__ import annotations

import numpy as np

from . import layout as L

GRAVITY = L.GRAVITY
QUADROTOR_RADIUS = 0.3


def _skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def _polar(X):
    U, _, Vt = np.linalg.svd(X)
    return U @ Vt


class RQPParameters:
    """RQPParameters(m, J, ml, Jl, r) -- same arguments and derived fields as the reference."""

    def __init__(self, m: np.ndarray, J: np.ndarray, ml: float, Jl: np.ndarray, r: np.ndarray) -> None:
        self.n = r.shape[1]
        assert m.shape == (self.n,)
        assert J.shape == (3, 3, self.n)
        assert Jl.shape == (3, 3)
        assert r.shape == (3, self.n)
        self.m, self.J, self.ml, self.Jl, self.r = m, J, float(ml), Jl, r
        self.mT = np.sum(m) + ml
        self.x_com = np.sum(r * m, axis=1) / self.mT
        self.r_com = (r.T - self.x_com).T
        JT = Jl - ml * _skew(self.x_com) @ _skew(self.x_com)
        for i in range(self.n):
            JT = JT - m[i] * _skew(self.r_com[:, i]) @ _skew(self.r_com[:, i])
        self.JT = JT
        self.JT_inv = np.linalg.inv(JT)
        self.J_inv = np.stack([np.linalg.inv(J[:, :, i]) for i in range(self.n)], axis=2)


class RQPState:
    """RQPState(R, w, xl, vl, Rl, wl); rotations are projected onto SO(3) at construction."""

    def __init__(self, R, w, xl, vl, Rl, wl, project: bool = True) -> None:
        self.n = w.shape[1]
        assert R.shape == (3, 3, self.n) and w.shape == (3, self.n)
        self.R = np.array(R, float)
        self.w = np.array(w, float)
        self.xl = np.array(xl, float)
        self.vl = np.array(vl, float)
        self.Rl = np.array(Rl, float)
        self.wl = np.array(wl, float)
        if project:
            self.project_R()
        self._counter = 0

    def project_R(self) -> None:
        self.Rl = _polar(self.Rl)
        for i in range(self.n):
            self.R[:, :, i] = _polar(self.R[:, :, i])

    def pack(self) -> np.ndarray:
        return pack_state(self)

    @staticmethod
    def unpack(x: np.ndarray, n: int) -> "RQPState":
        s = RQPState.__new__(RQPState)
        s.n = n
        s.R = np.transpose(x[L.s_off("R", n) : L.s_off("R", n) + 9 * n].reshape(n, 3, 3), (1, 2, 0)).copy()
        s.w = x[L.s_off("W", n) : L.s_off("W", n) + 3 * n].reshape(n, 3).T.copy()
        s.xl = x[L.s_off("XL", n) : L.s_off("XL", n) + 3].copy()
        s.vl = x[L.s_off("VL", n) : L.s_off("VL", n) + 3].copy()
        s.Rl = x[L.s_off("RL", n) : L.s_off("RL", n) + 9].reshape(3, 3).copy()
        s.wl = x[L.s_off("WL", n) : L.s_off("WL", n) + 3].copy()
        s._counter = 0
        return s


class RQPCollision:
    """Collision data (system/rigid_quadrotor_payload.py:279-310) without the display meshes."""

    def __init__(self, payload_vertices: np.ndarray, payload_mesh_vertices: np.ndarray) -> None:
        assert payload_vertices.shape[1] == 3 and payload_mesh_vertices.shape[1] == 3
        self.payload_vertices = payload_vertices
        self.payload_mesh_vertices = payload_mesh_vertices
        self.quadrotor_radius = QUADROTOR_RADIUS
        self.collision_radius = float(np.max(np.linalg.norm(payload_mesh_vertices, axis=1)) + QUADROTOR_RADIUS + 0.1)
        self.max_deceleration = GRAVITY / 5.0


def equilibrium_forces(p: RQPParameters) -> np.ndarray:
    """f_eq: min-norm least squares of the hover wrench (control/rqp_cadmm.py:165-174)."""
    W = np.empty((3, p.n))
    W[0, :] = 1.0
    for i in range(p.n):
        W[1:, i] = _skew(p.r_com[:, i])[:2, 2]
    f = np.zeros((3, p.n))
    f[2, :] = np.linalg.lstsq(W, np.array([p.mT * GRAVITY, 0.0, 0.0]), rcond=None)[0]
    return f


def pack_params(p: RQPParameters, col: RQPCollision) -> np.ndarray:
    """One scenario's parameter block (dat_layout.h DAT_P_*)."""
    n = p.n
    b = np.zeros(L.param_size(n))
    P = L.P
    b[P["MT"]] = p.mT
    b[P["XCOM"] : P["XCOM"] + 3] = p.x_com
    b[P["JT"] : P["JT"] + 9] = p.JT.reshape(-1)
    b[P["JTI"] : P["JTI"] + 9] = p.JT_inv.reshape(-1)
    b[P["MINFZ"]] = p.mT * GRAVITY / (n * 10.0)              # control/rqp_cadmm.py:195
    b[P["MAXF"]] = (2.0 / n) * p.mT * GRAVITY                 # :200
    b[P["SEC"]] = 1.0 / np.cos(np.pi / 6.0)                   # :197-198
    b[P["COSP"]] = np.cos(np.pi / 12.0)                       # :202-203
    b[P["MAXWL2"]] = (np.pi / 6.0) ** 2                       # :207-208
    b[P["MAXVL2"]] = 1.0                                      # :211-212
    b[P["DISTEPS"]] = 0.1                                     # :215
    b[P["VISR"]] = col.collision_radius + 5.0                 # :216
    b[P["COSCONE"]] = np.cos(100.0 * np.pi / 180.0)           # :217
    b[P["MAXDEC"]] = col.max_deceleration                     # :220
    b[P["COLR"]] = col.collision_radius
    b[P["KFD"]] = 0.1 / n                                     # :225
    b[P["KMD"]] = 0.1 / n                                     # :227
    b[P["KFC"]] = 0.1                                         # control/rqp_centralized.py:214
    b[P["KMC"]] = 0.1                                         # :216
    b[P["KFEQ"]] = 0.1                                        # :218
    b[P["AENVD"]] = 1.5                                       # control/rqp_cadmm.py:221
    b[P["AENVC"]] = 2.0                                       # control/rqp_centralized.py:210
    b[P["ML"]] = p.ml
    b[L.p_off("R", n) : L.p_off("R", n) + 3 * n] = p.r.T.reshape(-1)
    b[L.p_off("RCOM", n) : L.p_off("RCOM", n) + 3 * n] = p.r_com.T.reshape(-1)
    b[L.p_off("FEQ", n) : L.p_off("FEQ", n) + 3 * n] = equilibrium_forces(p).T.reshape(-1)
    b[L.p_off("J", n) : L.p_off("J", n) + 9 * n] = np.transpose(p.J, (2, 0, 1)).reshape(-1)
    b[L.p_off("JINV", n) : L.p_off("JINV", n) + 9 * n] = np.transpose(p.J_inv, (2, 0, 1)).reshape(-1)
    return b


def pack_state(s) -> np.ndarray:
    """One scenario's state block (dat_layout.h DAT_S_*); accepts any object with R, w, xl, vl, Rl, wl."""
    n = s.w.shape[1]
    x = np.empty(L.state_size(n))
    x[L.s_off("R", n) : L.s_off("R", n) + 9 * n] = np.transpose(s.R, (2, 0, 1)).reshape(-1)
    x[L.s_off("W", n) : L.s_off("W", n) + 3 * n] = s.w.T.reshape(-1)
    x[L.s_off("XL", n) : L.s_off("XL", n) + 3] = s.xl
    x[L.s_off("VL", n) : L.s_off("VL", n) + 3] = s.vl
    x[L.s_off("RL", n) : L.s_off("RL", n) + 9] = s.Rl.reshape(-1)
    x[L.s_off("WL", n) : L.s_off("WL", n) + 3] = s.wl
    return x


def pack_mountain(forest) -> np.ndarray:
    m = np.zeros(L.const("DAT_MOUNTAIN_SIZE"))
    m[L.M["CX"]], m[L.M["CY"]] = forest.mountain_center
    m[L.M["RADIUS"]] = forest.mountain_radius
    m[L.M["SPHERE_R"]] = forest.mountain_sphere_radius
    m[L.M["DEPTH"]] = forest.mountain_center_depth
    return m
