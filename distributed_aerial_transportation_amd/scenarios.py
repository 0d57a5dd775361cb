"""Scenario definitions (reference example/setup.py:64-126 for n = 3; build-defined teams otherwise).

The reference only defines the 3-quadrotor team (``example/setup.py:80-81`` raises for other n).
The benchmark configurations need n = 6 and n = 16 teams:
  * n = 6: hexagon attachment r_i = 0.55 (cos 2 pi i/6, sin 2 pi i/6, 0), reference masses/inertias;
  * n = 16: ring of radius 1 m, payload mass and inertia scaled by 16/3;
  * any other n: ring of radius 0.55 m.
Randomised payloads (config C3): ml ~ U(0.15, 0.30), Jl = diag(2.1, 1.87, 3.97)e-2 * U(0.8, 1.2)^3.
"""

from __future__ import annotations

import numpy as np

from .system import RQPCollision, RQPParameters, RQPState, pack_params, pack_state

PAYLOAD_VERTICES = np.array([[-0.42, -0.27, 0.0], [0.48, -0.27, 0.0], [-0.06, 0.55, 0.0],
                             [-0.42, -0.27, -0.1], [0.48, -0.27, -0.1], [-0.06, 0.55, -0.1]])
PAYLOAD_MESH_VERTICES = np.array([[-0.52, -0.37, 0.1], [0.58, -0.37, 0.1], [-0.06, 0.65, 0.1],
                                  [-0.52, -0.37, -0.2], [0.58, -0.37, -0.2], [-0.06, 0.65, -0.2]])
JQ = np.diag([2.32, 2.32, 4.0]) * 1e-3
JL = np.diag([2.1, 1.87, 3.97]) * 1e-2


def geometry(n: int):
    if n == 3:
        r = np.array([[-0.42, -0.27, 0.0], [0.48, -0.27, 0.0], [-0.06, 0.55, 0.0]]).T
        ml, Jl = 0.225, JL.copy()
    elif n == 16:
        a = 2 * np.pi * np.arange(16) / 16
        r = np.stack([np.cos(a), np.sin(a), np.zeros(16)])
        ml, Jl = 0.225 * 16 / 3, JL * 16 / 3
    else:
        a = 2 * np.pi * np.arange(n) / n
        r = np.stack([0.55 * np.cos(a), 0.55 * np.sin(a), np.zeros(n)])
        ml, Jl = 0.225, JL.copy()
    return np.full(n, 0.5), np.stack([JQ] * n, axis=2), ml, Jl, r


def collision(n: int) -> RQPCollision:
    if n == 3:
        return RQPCollision(PAYLOAD_VERTICES, PAYLOAD_MESH_VERTICES)
    # build-defined teams: mesh = attachment ring inflated by 0.1 m (collision radius = R + 0.5)
    _, _, _, _, r = geometry(n)
    R = np.linalg.norm(r, axis=0).max()
    return RQPCollision(np.vstack([r.T, r.T - [0, 0, 0.1]]), r.T * (R + 0.1) / R)


def rest_state(n: int) -> RQPState:
    return RQPState(np.stack([np.eye(3)] * n, axis=2), np.zeros((3, n)), np.zeros(3), np.zeros(3), np.eye(3),
                    np.zeros(3))


def rqp_setup(n: int):
    """(RQPParameters, RQPCollision, RQPState) -- reference example/setup.py:121-126."""
    return RQPParameters(*geometry(n)), collision(n), rest_state(n)


def randomized_params(n: int, batch: int, rng: np.random.Generator) -> np.ndarray:
    """Per-scenario parameter blocks with randomised payload mass / inertia (config C3)."""
    m, J, _, _, r = geometry(n)
    col = collision(n)
    blocks = []
    for _ in range(batch):
        ml = rng.uniform(0.15, 0.30)
        Jl = JL * np.diag(rng.uniform(0.8, 1.2, 3))
        blocks.append(pack_params(RQPParameters(m, J, ml, Jl, r), col))
    return np.stack(blocks)


def _exp3(v):
    t = np.linalg.norm(v)
    K = np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])
    if t < 1e-8:
        return np.eye(3) + K + 0.5 * K @ K
    return np.eye(3) + np.sin(t) / t * K + (1 - np.cos(t)) / t**2 * K @ K


def perturbed_states(n: int, batch: int, rng: np.random.Generator) -> np.ndarray:
    """Rest state + per-scenario perturbations: xl ~ U(-1,1)^3,
    vl ~ U(-0.5,0.5)^3, Rl = exp3(U(-0.1,0.1)^3), wl ~ U(-0.2,0.2)^3."""
    out = []
    for _ in range(batch):
        s = RQPState(np.stack([np.eye(3)] * n, axis=2), np.zeros((3, n)), rng.uniform(-1, 1, 3),
                     rng.uniform(-0.5, 0.5, 3), _exp3(rng.uniform(-0.1, 0.1, 3)), rng.uniform(-0.2, 0.2, 3))
        out.append(pack_state(s))
    return np.stack(out)


def forest_start_states(n: int, batch: int, rng: np.random.Generator) -> np.ndarray:
    """Config C4 start: xl = (U(-2,0), U(-10,10), 1.5), vl = (0.5, 0, 0), rest attitude."""
    out = []
    for _ in range(batch):
        s = RQPState(np.stack([np.eye(3)] * n, axis=2), np.zeros((3, n)),
                     np.array([rng.uniform(-2, 0), rng.uniform(-10, 10), 1.5]), np.array([0.5, 0.0, 0.0]), np.eye(3),
                     np.zeros(3))
        out.append(pack_state(s))
    return np.stack(out)


def forest_path_states(n: int, batch: int, rng: np.random.Generator, forests: list, scenario_forest: np.ndarray,
                       x_range=(-2.0, 50.0), y_half=5.0, speed=(0.5, 1.0), clearance: float = 2.0) -> np.ndarray:
    """Config C4 spread along the forest crossing of the reference run (example/rqp_example.py: the
    payload starts at the origin, the forest spans x in [5, 55] and |vl| <= 1 m/s, so a 100 s run
    is inside the forest for most of its steps): xl = (U(x_range), U(-y_half, y_half), terrain +
    1.5), vl = (U(speed), 0, 0), rest attitude.  Positions whose xy distance to a tree axis is below
    `clearance` are redrawn (no scenario starts inside a tree)."""
    xl = np.empty((batch, 3))
    sf = np.asarray(scenario_forest)
    todo = np.arange(batch)
    while todo.size:
        xl[todo, 0] = rng.uniform(*x_range, todo.size)
        xl[todo, 1] = rng.uniform(-y_half, y_half, todo.size)
        bad = []
        for f in np.unique(sf[todo]):
            idx = todo[sf[todo] == f]
            d = np.linalg.norm(xl[idx, None, :2] - forests[f].tree_pos[None, :, :2], axis=2).min(axis=1)
            bad.append(idx[d < clearance])
        todo = np.concatenate(bad) if bad else np.zeros(0, dtype=int)
    for f in np.unique(sf):
        idx = np.nonzero(sf == f)[0]
        xl[idx, 2] = [forests[f].terrain_height(p) + 1.5 for p in xl[idx, :2]]
    vx = rng.uniform(*speed, batch)
    # rest attitude, zero rates: one packed template, then the per-scenario position and velocity
    # (layout: csrc/dat_layout.h, DAT_S_XL = 12 n, DAT_S_VL = 12 n + 3)
    tmpl = pack_state(rest_state(n))
    out = np.tile(tmpl, (batch, 1))
    out[:, 12 * n:12 * n + 3] = xl
    out[:, 12 * n + 3] = vx
    return out


def params_block(n: int) -> np.ndarray:
    p, col, _ = rqp_setup(n)
    return pack_params(p, col)
