"""Forest environment data (reference example/env_forest.py:22-85).

Tree layouts are generated on the host exactly as the reference does (global legacy
``np.random`` stream, rejection sampling), so ``np.random.seed(s); Forest()`` reproduces the
reference's layout for seed s.  Distance queries and CBF rows run on the GPU (K5 in
``csrc/dat_core.hpp::env_rows``); there is no hppfcl here.
"""

from __future__ import annotations

import numpy as np

MOUNTAIN_CENTER = np.array([30.0, 0.0])  # example/env_forest.py:22-31
MOUNTAIN_RADIUS = 25.0
MOUNTAIN_HEIGHT = 7.5
BARK_HEIGHT = 4.0
BARK_RADIUS = 0.3
MIN_DIST_BETWEEN_TREES = 3.2
MAX_TREES = 200


class Forest:
    def __init__(self) -> None:
        self.mountain_center = MOUNTAIN_CENTER
        self.mountain_radius = MOUNTAIN_RADIUS
        self.bark_radius = BARK_RADIUS
        self._generate_trees()

    def _generate_trees(self) -> None:
        np.random.rand(1)  # the reference burns one draw first (example/env_forest.py:48)
        tree_xy = (MOUNTAIN_CENTER + np.array([0.5, 0.5])).reshape((1, 2))
        self.num_trees = 1
        for _ in range(MAX_TREES * 50):
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
            height = np.sqrt(self.mountain_sphere_radius**2 - np.dot(d, d)) - self.mountain_center_depth
            self.tree_pos[i, 2] = (height + BARK_HEIGHT) / 2.0

    @staticmethod
    def seeded(seed: int) -> "Forest":
        np.random.seed(seed)
        return Forest()

    def terrain_height(self, xy: np.ndarray) -> float:
        d = np.linalg.norm(np.asarray(xy)[:2] - self.mountain_center)
        if d >= self.mountain_radius:
            return 0.0
        return float(np.sqrt(self.mountain_sphere_radius**2 - d**2) - self.mountain_center_depth)
