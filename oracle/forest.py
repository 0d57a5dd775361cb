"""ORACLE (test infrastructure only) -- forest environment, capsule/tree distances, env CBF rows.

Restates
  * ``Forest._generate_trees``                 example/env_forest.py:47-85
  * ``Forest.centralized_distance``            example/env_forest.py:139-167
  * ``Forest.distributed_distance``            example/env_forest.py:169-212
  * ``_set_collision_avoidance_cbf_parameters`` control/rqp_cadmm.py:307-373 (same in
    control/rqp_dd.py:310-376 and, without the vision cone, control/rqp_centralized.py:280-337)

The reference measures capsule-vs-cylinder distance with hppfcl (GJK/EPA, C++), which
is absent here.  The oracle computes the same quantity -- distance between the capsule
(segment xl -> xl + h v/|v|, radius col_r; ``hppfcl.Capsule(radius, lz)`` is centred with
its axis on z, posed by ``rotation_matrix_a_to_b(e3, v/|v|)``, example/env_forest.py and
utils/math_utils.py:45-60) and each tree (solid cylinder, radius 0.3, length 4, axis z) --
by brute force: a dense sweep of the segment parameter followed by a bounded scalar
refinement of the (convex) point-to-cylinder distance.  Parity with hppfcl's GJK output is
*unpinned* (hppfcl absent); its ~1e-6 GJK tolerance is inside the 1e-5 control tolerance.
"""

from __future__ import annotations

import numpy as np
from scipy.optimize import minimize_scalar

from .model import Consts, EnvRows, State

MOUNTAIN_CENTER = np.array([30.0, 0.0])
MOUNTAIN_RADIUS = 25.0
MOUNTAIN_HEIGHT = 7.5
BARK_HEIGHT = 4.0
BARK_RADIUS = 0.3
MIN_DIST_BETWEEN_TREES = 3.2
MAX_TREES = 200


class Forest:
    """Forest geometry with the reference's (global, legacy) np.random draw order.
    Seed with ``np.random.seed(s)`` before constructing for a reproducible layout."""

    def __init__(self):
        self.mountain_center = MOUNTAIN_CENTER
        self.mountain_radius = MOUNTAIN_RADIUS
        self.bark_radius = BARK_RADIUS
        np.random.rand(1)
        max_tries = MAX_TREES * 50
        tree_xy = (MOUNTAIN_CENTER + np.array([0.5, 0.5])).reshape((1, 2))
        self.num_trees = 1
        for _ in range(max_tries):
            pos = np.random.random((2,)) - 0.5
            norm = np.linalg.norm(pos)
            if norm == 0:
                continue
            radius = np.random.random()
            pos = pos / norm * radius * MOUNTAIN_RADIUS + MOUNTAIN_CENTER
            if np.min(np.linalg.norm(tree_xy - pos, axis=1)) < MIN_DIST_BETWEEN_TREES:
                continue
            tree_xy = np.vstack((tree_xy, pos))
            self.num_trees += 1
            if self.num_trees >= MAX_TREES:
                break
        self.tree_pos = np.empty((self.num_trees, 3))
        self.tree_pos[:, :2] = tree_xy
        ang = np.pi / 2.0 - np.arctan2(MOUNTAIN_RADIUS, MOUNTAIN_HEIGHT)
        self.mountain_sphere_radius = MOUNTAIN_RADIUS / np.sin(ang)
        self.mountain_center_depth = self.mountain_sphere_radius * np.cos(ang)
        for i in range(self.num_trees):
            d = self.tree_pos[i, :2] - MOUNTAIN_CENTER
            hgt = np.sqrt(self.mountain_sphere_radius**2 - d @ d) - self.mountain_center_depth
            self.tree_pos[i, 2] = (hgt + BARK_HEIGHT) / 2.0


def _point_cyl(p, c):
    """Distance from point p to the solid tree cylinder centred at c, and nearest point."""
    dxy = p[:2] - c[:2]
    rho = np.linalg.norm(dxy)
    hz = p[2] - c[2]
    q = p.copy()
    if rho > BARK_RADIUS:
        q[:2] = c[:2] + dxy / rho * BARK_RADIUS
    q[2] = c[2] + np.clip(hz, -BARK_HEIGHT / 2, BARK_HEIGHT / 2)
    return np.linalg.norm(p - q), q


def capsule_tree_distance(x0, x1, radius, c):
    """Signed distance capsule(seg x0->x1, radius) vs tree c; nearest points (world frame)."""
    seg = x1 - x0
    f = lambda t: _point_cyl(x0 + t * seg, c)[0]
    ts = np.linspace(0.0, 1.0, 2001)
    # the dense sample (vectorised _point_cyl) only brackets the minimiser; the refinement below and
    # the returned points use the scalar path
    P = x0[None, :] + ts[:, None] * seg[None, :]
    dxy = P[:, :2] - c[:2]
    rho = np.sqrt(dxy[:, 0] ** 2 + dxy[:, 1] ** 2)
    Q = P.copy()
    out = rho > BARK_RADIUS
    Q[out, :2] = c[:2] + dxy[out] / rho[out, None] * BARK_RADIUS
    Q[:, 2] = c[2] + np.clip(P[:, 2] - c[2], -BARK_HEIGHT / 2, BARK_HEIGHT / 2)
    vals = np.sqrt(np.sum((P - Q) ** 2, axis=1))
    k = int(np.argmin(vals))
    lo, hi = ts[max(k - 1, 0)], ts[min(k + 1, len(ts) - 1)]
    if hi > lo:
        r = minimize_scalar(f, bounds=(lo, hi), method="bounded", options={"xatol": 1e-15})
        t = r.x if r.fun <= vals[k] else ts[k]
    else:
        t = ts[k]
    p = x0 + t * seg
    dseg, q = _point_cyl(p, c)
    if dseg > 0:
        p1 = p + (q - p) / dseg * radius
    else:
        p1 = p
    return dseg - radius, p1, q


def _query(forest: Forest, x0, x1, radius, center, vision_radius, cone=None):
    min_d, p1s, p2s = [], [], []
    collision = False
    for i in range(forest.num_trees):
        pos = forest.tree_pos[i]
        if np.linalg.norm(center - pos) > vision_radius + BARK_RADIUS:
            continue
        if cone is not None:
            direction, camera_pos, cos_ang = cone
            dt = pos[:2] - camera_pos
            nrm = np.linalg.norm(dt)
            if nrm > 0 and (dt / nrm) @ direction < cos_ang:
                continue
        d, p1, p2 = capsule_tree_distance(x0, x1, radius, pos)
        if d < 1e-4:
            collision = True
        min_d.append(d)
        p1s.append(p1)
        p2s.append(p2)
    return collision, np.array(min_d), np.array(p1s).reshape(-1, 3), np.array(p2s).reshape(-1, 3)


def env_rows(forest, c: Consts, s: State, col_radius: float, r_i=None) -> EnvRows:
    """Env CBF rows for one solve (control/rqp_cadmm.py:307-373; centralized when r_i is None)."""
    rows = EnvRows.empty(c)
    if forest is None:
        return rows
    h = 0.5 * (s.vl @ s.vl) / c.max_deceleration
    speed = np.linalg.norm(s.vl)
    if speed == 0:
        v_dir = None
        x0 = x1 = s.xl.copy()
        center = s.xl.copy()
    else:
        v_dir = s.vl / speed
        x0 = s.xl.copy()
        x1 = s.xl + h * v_dir
        center = s.xl + h / 2.0 * v_dir
    cone = None
    if r_i is not None:
        camera_pos = (s.xl + s.Rl @ r_i)[:2]
        d = camera_pos - s.xl[:2]
        nrm = np.linalg.norm(d)
        if nrm == 0:
            rows.collision = True
            return rows
        cone = (d / nrm, camera_pos, np.cos(c.vision_cone_ang))
    collision, dists, p1, p2 = _query(forest, x0, x1, col_radius, center, c.vision_radius, cone)
    rows.collision = collision
    k = min(dists.shape[0], c.nenv_cbfs)
    if k > 0 and speed > 0:
        rows.min_env_dist = float(np.min(dists))
        idx = np.argsort(dists, kind="stable")[:k] if k < dists.shape[0] else np.arange(k)
        lhs = np.zeros((c.nenv_cbfs, 3))
        rhs = np.zeros(c.nenv_cbfs)
        for j in range(k):
            t = idx[j]
            di = dists[t]
            if di <= 1e-4:
                continue
            proj = np.dot(p1[t] - s.xl, v_dir)
            proj = max(0.0, min(h, proj))
            mt = np.sqrt(2.0 * (h - proj) / c.max_deceleration)
            mt = max(0.0, speed / c.max_deceleration - mt)
            nrm = p1[t] - p2[t]
            nrm = nrm / np.linalg.norm(nrm)
            lhs[j] = nrm * mt
            rhs[j] = -c.alpha_env * (di - c.dist_eps) - nrm @ s.vl
        rows.lhs, rows.rhs = lhs, rhs
    return rows
