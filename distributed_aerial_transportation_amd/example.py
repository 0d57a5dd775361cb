"""The reference's forest example on the GPU, with its log format and statistics printout.

``simulate`` reproduces example/rqp_example.py:main (:83-165) -- HL control every ``hl_rel_freq``
steps from the forest desired-acceleration law (:33-59), the LL SO(3) law and the dynamics at every
step -- with every piece on the device (k_desired, the controller kernels, k_low_level, k_rollout),
and returns the ``logs`` dict of :141-165 with the same keys, element types and logging instants:

    n, dt, T, hl_rel_freq, log_freq, num_trees, tree_pos, controller_type,
    state_seq (RQPStateData after step i), x_err_seq, v_err_seq (|x_ref - xl|, |v_ref - vl| after step i),
    f_des_seq (3, n), iter_seq (not for centralized), solve_time_seq [s], min_env_dist_seq,
    w_seq ((f (n,), M (3, n)) applied at step i),      logged at i % log_freq == 0

so example/rqp_plots.py (:494-521) can read a GPU run (``save_logs`` writes the pickle it loads).
``simulate_batch`` runs B scenarios at once (different forests / start states) and returns one such
dict per scenario.  ``print_stats`` is ``_print_stats`` (:62-80) with the same format.
"""

from __future__ import annotations

import pickle
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import scenarios
from .env_forest import Forest
from .system import RQPState, pack_state

CONTROLLER_TYPES = ("centralized", "dual-decomposition", "consensus-admm")


@dataclass
class RQPStateData:
    """example/rqp_example.py:23-30."""

    R: np.ndarray
    w: np.ndarray
    xl: np.ndarray
    vl: np.ndarray
    Rl: np.ndarray
    wl: np.ndarray


def compute_aggregate_statistics(a: np.ndarray):
    """utils/math_utils.py:63-73: min, max, avg, std along axis 0."""
    return np.min(a, axis=0), np.max(a, axis=0), np.mean(a, axis=0), np.std(a, axis=0)


def print_stats(iter: List[int], solve_time: List[float]) -> None:  # noqa: A002 -- the reference's name
    """example/rqp_example.py:62-80."""
    if len(iter) > 0:
        s = compute_aggregate_statistics(np.array(iter))
        print(f"Solver iterations: min: {s[0]:5.2f}, max: {s[1]:5.2f}, avg: {s[2]:5.2f}, std: {s[3]:5.2f}")
    if len(solve_time) > 0:
        s = compute_aggregate_statistics(np.array(solve_time))
        print(f"Solver solve time (ms): min: {s[0] * 1e3:7.3f}, max: {s[1] * 1e3:7.3f}, avg: {s[2] * 1e3:7.3f}, "
              f"std: {s[3] * 1e3:7.3f}")


def save_logs(logs: dict, file_name: str) -> None:
    """The pickle example/rqp_example.py:167-170 writes (logs/rqp_forest_<controller_type>.pkl)."""
    with open(file_name, "wb") as f:
        pickle.dump(logs, f)


def references(xl: np.ndarray, forest) -> tuple:
    """x_ref, v_ref of _desired_acceleration_forest (example/rqp_example.py:36-48) for positions xl (B, 3)."""
    xl = np.atleast_2d(xl)
    x_ref = np.zeros_like(xl)
    x_ref[:, 0] = xl[:, 0] + 1.5
    nrm = np.linalg.norm(xl[:, :2] - np.asarray(forest.mountain_center), axis=1)
    inside = nrm < forest.mountain_radius
    x_ref[:, 2] = 1.5
    x_ref[inside, 2] = (np.sqrt(forest.mountain_sphere_radius ** 2 - nrm[inside] ** 2) - forest.mountain_center_depth
                        + 1.5)
    v_ref = np.tile([0.5, 0.0, 0.0], (xl.shape[0], 1))
    return x_ref, v_ref


def simulate_batch(controller_type: str, states: np.ndarray, forests: list, scenario_forest=None, n: int = 3,
                   T: float = 100.0, dt: float = 1e-3, hl_rel_freq: int = 10, log_freq: Optional[int] = None,
                   so3_controller_type: str = "pd", params: Optional[np.ndarray] = None, device: int = 0,
                   progress: bool = False) -> List[dict]:
    """B closed loops of example/rqp_example.py:main on one GPU; states (B, 12n + 18) (packed
    RQPState), forests[scenario_forest[b]] the forest of scenario b.  Returns one logs dict per scenario."""
    from .control import BatchedController

    if controller_type not in CONTROLLER_TYPES:
        raise NotImplementedError(controller_type)
    log_freq = hl_rel_freq if log_freq is None else log_freq
    states = np.atleast_2d(np.asarray(states, float))
    B = states.shape[0]
    sf = np.zeros(B, dtype=np.int32) if scenario_forest is None else np.asarray(scenario_forest, dtype=np.int32)
    prm = scenarios.params_block(n) if params is None else params
    eng = BatchedController(controller_type, n, B, prm, dt=dt, hl_every=hl_rel_freq, device=device)
    eng.set_forests(forests, sf)
    eng.set_low_level(so3_controller_type)
    eng.set_state(states, np.zeros(B, dtype=np.int32))
    steps = len(np.arange(0, T, dt))  # t_seq = np.arange(0, T, dt) (:107)
    logs = [dict(n=n, dt=dt, T=T, hl_rel_freq=hl_rel_freq, log_freq=log_freq,
                 num_trees=forests[sf[b]].num_trees, tree_pos=forests[sf[b]].tree_pos, controller_type=controller_type,
                 state_seq=[], x_err_seq=[], v_err_seq=[], f_des_seq=[], iter_seq=[], solve_time_seq=[],
                 min_env_dist_seq=[], w_seq=[]) for b in range(B)]
    x_ref = v_ref = None
    i = 0
    while i < steps:
        if i % hl_rel_freq == 0:
            x, _ = eng.get_state()
            x_ref = np.empty((B, 3))
            v_ref = np.empty((B, 3))
            for f in np.unique(sf):
                idx = np.nonzero(sf == f)[0]
                x_ref[idx], v_ref[idx] = references(x[idx, 12 * n:12 * n + 3], forests[f])
            r = eng.control(None, None)  # desired acceleration on device (:102-103), then control (:104)
            for b in range(B):
                lg = logs[b]
                lg["f_des_seq"].append(r.f_des[b].copy())
                if r.iters[b] != -1:
                    lg["iter_seq"].append(int(r.iters[b]))
                lg["solve_time_seq"].append(r.gpu_ms * 1e-3)
                lg["min_env_dist_seq"].append(float(r.min_env_dist[b]))
        if i % log_freq == 0:
            fw, Mw = eng.low_level(None)  # the wrench integrated at step i (:111-112)
            eng.rollout(1)
            x, _ = eng.get_state()
            for b in range(B):
                s = RQPState.unpack(x[b], n)
                lg = logs[b]
                lg["w_seq"].append((fw[b].copy(), Mw[b].copy()))
                lg["x_err_seq"].append(float(np.linalg.norm(x_ref[b] - s.xl)))
                lg["v_err_seq"].append(float(np.linalg.norm(v_ref[b] - s.vl)))
                lg["state_seq"].append(RQPStateData(s.R, s.w, s.xl, s.vl, s.Rl, s.wl))
            i += 1
            continue
        # advance to the next control or log instant
        nxt = min(steps, (i // hl_rel_freq + 1) * hl_rel_freq, (i // log_freq + 1) * log_freq)
        eng.rollout(nxt - i)
        i = nxt
        if progress and i % 5000 == 0:
            print(f"t = {i * dt:.0f} s", flush=True)
    eng.close()
    return logs


def simulate(controller_type: str = "dual-decomposition", n: int = 3, T: float = 100.0, dt: float = 1e-3,
             hl_rel_freq: int = 10, log_freq: Optional[int] = None, env=None, state: Optional[RQPState] = None,
             so3_controller_type: str = "pd", device: int = 0, verbose: bool = True) -> dict:
    """example/rqp_example.py:main on the GPU for one scenario (rqp_setup(n) start state, Forest()
    environment -- pass env = Forest.seeded(s) for a reproducible layout); prints the statistics of
    :140 and returns the logs dict of :141-165."""
    env = Forest() if env is None else env
    if state is None:
        _, _, state = scenarios.rqp_setup(n)
    logs = simulate_batch(controller_type, pack_state(state)[None], [env], None, n=n, T=T, dt=dt,
                          hl_rel_freq=hl_rel_freq, log_freq=log_freq, so3_controller_type=so3_controller_type,
                          device=device)[0]
    if verbose:
        print_stats(logs["iter_seq"], logs["solve_time_seq"])
    return logs


__all__ = ["RQPStateData", "simulate", "simulate_batch", "print_stats", "save_logs", "compute_aggregate_statistics",
           "references"]
