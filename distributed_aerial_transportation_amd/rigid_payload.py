"""Rigid payload carried by force actuators: RPCentralizedController on the GPU.

The reference's RPCentralizedController (control/rp_centralized.py:9-302) is the same second-order-
cone QP family as the quadrotor-payload centralized controller: variables (dvl, dwl, f), dynamics
    ml dvl = sum_i f_i - ml g e3,   Jl dwl + wl x Jl wl = sum_i hat(r_i) Rl' f_i       (:226-235)
per-actuator cones f_iz >= min_fz, |f_i| <= sec(pi/6) f_iz, |f_i| <= max_f (:237-245), the three CBF
rows (payload tilt with max_p_ang = pi/6 and alpha1 = alpha2 = 1, |wl| and |vl| with alpha 1,
:247-272), cost k_f |sum f - ml g e3|^2 + k_feq sum |f_i - f_eq,i|^2 + |dvl - dvl_des|^2 +
|dwl - dwl_des|^2 (:275-294), no env rows, no moment cost.  That is exactly the reduced QP the
centralized kernel (k_cent) solves, with the parameter block mapped:
    mT -> ml, x_com -> 0 (so dvl has no moment term), JT -> Jl, r_com -> r, k_m -> 0,
    cos(max_p_ang) -> cos(pi/6), min_fz = ml g / (10 n), max_f = 2 ml g / n,
    f_eq = min-norm lstsq of [1'; hat(r_i)[:2, 2]] f_z = (ml g, 0, 0)      (:126-132)
``pack_rp_params`` builds that block; ``RPCentralizedController`` keeps the reference's constructor and
``control(state, acc_des) -> f (3, n)`` (hold the previous f when not OPTIMAL, :299-306).
``RPDynamics`` integrates system/rigid_payload.py:93-130 (forces applied at r_i) on the device
(k_rp_rollout, dat_rp_rollout).
"""

from __future__ import annotations

from typing import Optional

import numpy as np

from . import layout as L
from .system import GRAVITY, RQPCollision, _polar, _skew

_PROJ = 20  # _INTEGRATION_STEPS_PER_ROTATION_PROJECTION (system/rigid_payload.py:11)


class RPParameters:
    """system/rigid_payload.py:34-49."""

    def __init__(self, ml: float, Jl: np.ndarray, r: np.ndarray) -> None:
        self.n = r.shape[1]
        assert Jl.shape == (3, 3) and r.shape == (3, self.n)
        self.ml = float(ml)
        self.Jl = np.asarray(Jl, float)
        self.r = np.asarray(r, float)
        self.Jl_inv = np.linalg.inv(self.Jl)


class RPState:
    """system/rigid_payload.py:52-90 (Rl is projected onto SO(3) on construction)."""

    def __init__(self, xl, vl, Rl, wl, project: bool = True) -> None:
        self.xl = np.array(xl, float)
        self.vl = np.array(vl, float)
        self.Rl = np.array(Rl, float)
        self.wl = np.array(wl, float)
        if project:
            self.Rl = _polar(self.Rl)
        self.counter = 0


class RPCollision:
    """system/rigid_payload.py:176-200 without the display meshes."""

    def __init__(self, payload_vertices: np.ndarray, payload_mesh_vertices: np.ndarray) -> None:
        self.payload_vertices = np.asarray(payload_vertices, float)
        self.payload_mesh_vertices = np.asarray(payload_mesh_vertices, float)


def rp_setup(n: int = 3):
    """example/setup.py:10-60 (n = 3 only, as in the reference)."""
    if n != 3:
        raise NotImplementedError
    r = np.array([[-0.42, -0.27, 0], [0.48, -0.27, 0], [-0.06, 0.55, 0]], float).T
    verts = np.array([[-0.42, -0.27, 0], [0.48, -0.27, 0], [-0.06, 0.55, 0], [-0.42, -0.27, -0.1],
                      [0.48, -0.27, -0.1], [-0.06, 0.55, -0.1]])
    mesh = np.array([[-0.52, -0.37, 0.1], [0.58, -0.37, 0.1], [-0.06, 0.65, 0.1], [-0.52, -0.37, -0.2],
                     [0.58, -0.37, -0.2], [-0.06, 0.65, -0.2]])
    return (RPParameters(0.225, np.diag([2.1, 1.87, 3.97]) * 1e-2, r), RPCollision(verts, mesh),
            RPState(np.zeros(3), np.zeros(3), np.eye(3), np.zeros(3)))


def rp_equilibrium_forces(p: RPParameters) -> np.ndarray:
    """control/rp_centralized.py:126-132."""
    W = np.empty((3, p.n))
    W[0, :] = 1.0
    for i in range(p.n):
        W[1:, i] = _skew(p.r[:, i])[:2, 2]
    f = np.zeros((3, p.n))
    f[2, :] = np.linalg.lstsq(W, np.array([p.ml * GRAVITY, 0.0, 0.0]), rcond=None)[0]
    return f


def pack_rp_params(p: RPParameters) -> np.ndarray:
    """The k_cent parameter block of the rigid-payload QP (mapping in the module docstring)."""
    n = p.n
    b = np.zeros(L.param_size(n))
    P = L.P
    b[P["MT"]] = p.ml
    b[P["JT"]: P["JT"] + 9] = p.Jl.reshape(-1)
    b[P["JTI"]: P["JTI"] + 9] = p.Jl_inv.reshape(-1)
    b[P["MINFZ"]] = p.ml * GRAVITY / (n * 10.0)               # control/rp_centralized.py:147
    b[P["MAXF"]] = (2.0 / n) * p.ml * GRAVITY                  # :152
    b[P["SEC"]] = 1.0 / np.cos(np.pi / 6.0)                    # :149-150
    b[P["COSP"]] = np.cos(np.pi / 6.0)                         # :154-155
    b[P["MAXWL2"]] = (np.pi / 6.0) ** 2                        # :159-160
    b[P["MAXVL2"]] = 1.0                                       # :163-164
    b[P["VISR"]] = 1e300                                       # no env (:76)
    b[P["KFC"]] = 0.1                                          # :169
    b[P["KMC"]] = 0.0                                          # no moment cost
    b[P["KFEQ"]] = 0.1                                         # :171
    b[P["ML"]] = p.ml
    b[L.p_off("R", n): L.p_off("R", n) + 3 * n] = p.r.T.reshape(-1)
    b[L.p_off("RCOM", n): L.p_off("RCOM", n) + 3 * n] = p.r.T.reshape(-1)
    b[L.p_off("FEQ", n): L.p_off("FEQ", n) + 3 * n] = rp_equilibrium_forces(p).T.reshape(-1)
    eye = np.tile(np.eye(3).reshape(-1), n)                    # actuator inertias: unused by the QP
    b[L.p_off("J", n): L.p_off("J", n) + 9 * n] = eye
    b[L.p_off("JINV", n): L.p_off("JINV", n) + 9 * n] = eye
    return b


def pack_rp_state(s: RPState, n: int) -> np.ndarray:
    """RPState as a dat state block (actuator attitudes unused: identity, zero rates)."""
    x = np.zeros(L.state_size(n))
    x[L.s_off("R", n): L.s_off("R", n) + 9 * n] = np.tile(np.eye(3).reshape(-1), n)
    x[L.s_off("XL", n): L.s_off("XL", n) + 3] = s.xl
    x[L.s_off("VL", n): L.s_off("VL", n) + 3] = s.vl
    x[L.s_off("RL", n): L.s_off("RL", n) + 9] = s.Rl.reshape(-1)
    x[L.s_off("WL", n): L.s_off("WL", n) + 3] = s.wl
    return x


def unpack_rp_state(x: np.ndarray, n: int) -> RPState:
    o = L.s_off("XL", n)
    return RPState(x[o:o + 3], x[o + 3:o + 6], x[o + 6:o + 15].reshape(3, 3), x[o + 15:o + 18], project=False)


class RPCentralizedController:
    """control/rp_centralized.py:9-306 on the GPU (k_cent with the rigid-payload parameter block)."""

    def __init__(self, params: RPParameters, col: Optional[RPCollision], state: RPState, dt: float,
                 verbose: bool = False, device: int = 0) -> None:
        from .control import BatchedController

        assert params.n >= 3
        self.n, self.params, self.col, self.dt, self.verbose = params.n, params, col, dt, verbose
        self.f_eq = rp_equilibrium_forces(params)
        self.min_fz = params.ml * GRAVITY / (self.n * 10.0)
        self.max_f = (2.0 / self.n) * params.ml * GRAVITY
        self._eng = BatchedController("centralized", self.n, 1, pack_rp_params(params), dt=dt, device=device)
        self.prev_f = self.f_eq.copy()

    def control(self, state: RPState, acc_des) -> np.ndarray:
        acc = np.concatenate([np.asarray(acc_des[0], float), np.asarray(acc_des[1], float)])[None]
        r = self._eng.control(pack_rp_state(state, self.n)[None], acc)
        if int(r.qp_status[0, 0]) == 0:
            self.prev_f = r.f_des[0].copy()
        elif self.verbose:
            print(f"Problem not solved to optimality, status: {int(r.qp_status[0, 0])}")
        return self.prev_f


class RPDynamics:
    """system/rigid_payload.py:93-172 on the device: ``integrate(f)`` advances one step of dt with the
    actuator forces f (3, n) (k_rp_rollout); ``state`` reads it back."""

    def __init__(self, params: RPParameters, state: RPState, dt: float, device: int = 0) -> None:
        from .control import BatchedController

        self.params, self.dt, self.n = params, dt, params.n
        self._eng = BatchedController("centralized", self.n, 1, pack_rp_params(params), dt=dt, device=device)
        self._eng.set_state(pack_rp_state(state, self.n)[None], np.array([state.counter], dtype=np.int32))

    def integrate(self, f: np.ndarray, steps: int = 1) -> None:
        self._eng.rp_rollout(steps, np.asarray(f, float)[None])

    @property
    def state(self) -> RPState:
        x, c = self._eng.get_state()
        s = unpack_rp_state(x[0], self.n)
        s.counter = int(c[0])
        return s


__all__ = ["RPParameters", "RPState", "RPCollision", "rp_setup", "rp_equilibrium_forces", "pack_rp_params",
           "pack_rp_state", "unpack_rp_state", "RPCentralizedController", "RPDynamics"]
