"""ORACLE (test infrastructure only) -- scenario definitions.

n = 3 restates ``example/setup.py:64-126`` (_rqp_nquadrotors_parameters, _rqp_collision,
_rqp_nquadrotors_init_state).  The reference defines no n != 3 geometry
(``example/setup.py:80-81`` raises NotImplementedError); n = 6 (hexagon) and n = 16 (ring)
follow SURVEY.md section 8(d) (configs C3-C5) and are build-defined.
"""

import numpy as np

from .model import Params, State, collision_radius

PAYLOAD_MESH_VERTICES = np.array(
    [[-0.52, -0.37, 0.1], [0.58, -0.37, 0.1], [-0.06, 0.65, 0.1],
     [-0.52, -0.37, -0.2], [0.58, -0.37, -0.2], [-0.06, 0.65, -0.2]])
JQ = np.diag([2.32, 2.32, 4.0]) * 1e-3
JL = np.diag([2.1, 1.87, 3.97]) * 1e-2


def geometry(n: int):
    """(m, J, ml, Jl, r) for the build's scenario families."""
    if n == 3:
        r = np.array([[-0.42, -0.27, 0.0], [0.48, -0.27, 0.0], [-0.06, 0.55, 0.0]]).T
        ml, Jl = 0.225, JL.copy()
    elif n == 6:
        a = 2 * np.pi * np.arange(6) / 6
        r = np.stack([0.55 * np.cos(a), 0.55 * np.sin(a), np.zeros(6)])
        ml, Jl = 0.225, JL.copy()
    elif n == 16:
        a = 2 * np.pi * np.arange(16) / 16
        r = np.stack([np.cos(a), np.sin(a), np.zeros(16)])
        ml, Jl = 0.225 * 16 / 3, JL * 16 / 3
    else:
        a = 2 * np.pi * np.arange(n) / n
        r = np.stack([0.55 * np.cos(a), 0.55 * np.sin(a), np.zeros(n)])
        ml, Jl = 0.225, JL.copy()
    m = np.full(n, 0.5)
    J = np.stack([JQ] * n, axis=2)
    return m, J, ml, Jl, r


def params(n: int) -> Params:
    return Params(*geometry(n))


def col_radius(n: int = 3) -> float:
    """n = 3 uses the reference payload mesh; other n scale the mesh to the attachment ring."""
    if n == 3:
        return collision_radius(PAYLOAD_MESH_VERTICES)
    _, _, _, _, r = geometry(n)
    return float(np.max(np.linalg.norm(r, axis=0)) + 0.1 + 0.3 + 0.1)


def rest_state(n: int) -> State:
    return State(np.stack([np.eye(3)] * n, axis=2), np.zeros((3, n)), np.zeros(3), np.zeros(3),
                 np.eye(3), np.zeros(3))
