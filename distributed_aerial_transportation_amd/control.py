"""Controllers on top of libdat.so -- the reference's controller API, batched and drop-in.

Batched engine
  ``BatchedController(mode, n, batch, params, col, ...)``: one HIP handle driving B independent
  scenarios; ``control(states, acc_des)`` runs one high-level step for all of them on the GPU.

Drop-in single-scenario classes (same constructor and per-step interface as the reference):
  ``RQPCentralizedController``  control/rqp_centralized.py:27-455
  ``RQPCADMMController``        control/rqp_cadmm.py:510-688
  ``RQPDDController``           control/rqp_dd.py:558-764
  each: ``__init__(params, col, state, dt, env=None, verbose=False)``,
        ``control(state, acc_des) -> (f_des (3, n), SolverStatistics)``,
        ``get_force_cone_angle_bound()``, ``get_dist_eps()``,
        ``set_force_err_tolerance(tol[, use_total_res])``, ``set_max_iter(k)`` (C-ADMM / DD).
  ``RQPLowLevelController(so3_controller_type, params, max_f_ang)``: control/rqp_centralized.py:457-535
        ("pd" or "sm" SO(3) law) on the GPU; ``BatchedController.set_low_level`` selects the law of the
        device rollout (SO(3) law + rigid-body dynamics + Lie integration).
The QPs are solved by the HIP kernels; the reference's Clarabel per-call solve time becomes the
GPU kernel time of the step (``SolverStatistics.solve_time``).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Any, List, Optional

import numpy as np

from . import _lib as L
from . import layout
from .system import (RQPCollision, RQPParameters, RQPState, _skew, equilibrium_forces, pack_mountain, pack_params,
                     pack_state)

MODES = {"centralized": L.MODE_CENTRALIZED, "consensus-admm": L.MODE_CADMM, "cadmm": L.MODE_CADMM,
         "dual-decomposition": L.MODE_DD, "dd": L.MODE_DD}


@dataclass
class SolverStatistics:
    """control/rqp_centralized.py:18-24."""

    iter: int
    solve_time: float
    collision: bool
    min_env_dist: float
    err_seq: Optional[List[float]] = None


@dataclass
class StepResult:
    """Batched outputs of one high-level step (leading axis: scenario)."""

    f_des: np.ndarray           # (B, 3, n)
    iters: np.ndarray           # (B,)
    qp_status: np.ndarray       # (B, n)
    min_env_dist: np.ndarray    # (B,)
    collision: Optional[np.ndarray]  # (B,) bool (None: not computed, control_steps)
    err_seq: Optional[np.ndarray] = None  # (B, max_iter + 1), NaN padded
    gpu_ms: float = 0.0


class BatchedController:
    """B independent scenarios of one controller type on one GPU."""

    def __init__(self, mode, n: int, batch: int, params: np.ndarray, *, per_scenario_params: bool = False,
                 dt: float = 1e-3, hl_every: int = 10, device: int = 0, max_iter: int = 100, res_tol: float = 1e-2,
                 use_total_res: bool = True, record_err: bool = False, rho0: float = 1.0, tau_incr: float = 1.0,
                 rho_max: float = 2.0) -> None:
        self.mode = MODES[mode] if isinstance(mode, str) else int(mode)
        self.n, self.batch = n, batch
        lib = L.lib()
        cfg = L.Config()
        lib.dat_default_config(cfg)
        cfg.device, cfg.mode, cfg.n, cfg.batch = device, self.mode, n, batch
        cfg.dt, cfg.hl_every, cfg.max_iter, cfg.res_tol = dt, hl_every, max_iter, res_tol
        cfg.use_total_res, cfg.record_err = int(use_total_res), int(record_err)
        cfg.rho0, cfg.tau_incr, cfg.rho_max = rho0, tau_incr, rho_max
        self.cfg = cfg
        h = L.H()
        L.check(lib.dat_create(cfg, h))
        self._h = h
        self._lib = lib
        params = L.f64(params)
        if per_scenario_params:
            assert params.shape == (batch, layout.param_size(n)), params.shape
        else:
            assert params.shape == (layout.param_size(n),), params.shape
        self.params = params
        L.check(lib.dat_set_params(h, L.ptr(params), int(per_scenario_params)))

    # -- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.dat_destroy(self._h)
            self._h = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    # -- configuration
    def set_forests(self, forests: list, scenario_forest: Optional[np.ndarray] = None) -> None:
        """forests: list of objects with tree_pos (T, 3) and mountain constants; [] removes the env."""
        if not forests:
            L.check(self._lib.dat_set_forests(self._h, 0, None, None, None, None))
            return
        offs = np.zeros(len(forests) + 1, dtype=np.int32)
        for k, f in enumerate(forests):
            offs[k + 1] = offs[k] + f.tree_pos.shape[0]
        trees = L.f64(np.concatenate([f.tree_pos for f in forests]))
        mountains = L.f64(np.stack([pack_mountain(f) for f in forests]))
        sf = None if scenario_forest is None else L.i32(scenario_forest)
        if sf is not None:
            assert sf.shape == (self.batch,)
        L.check(self._lib.dat_set_forests(self._h, len(forests), L.ptr(offs, L.I), L.ptr(trees),
                                          None if sf is None else L.ptr(sf, L.I), L.ptr(mountains)))

    def set_force_err_tolerance(self, tol: float, use_total_res: bool = True) -> None:
        L.check(self._lib.dat_set_tolerance(self._h, float(tol), int(use_total_res)))
        self.cfg.res_tol, self.cfg.use_total_res = tol, int(use_total_res)

    def set_max_iter(self, max_iter: int) -> None:
        L.check(self._lib.dat_set_max_iter(self._h, int(max_iter)))
        self.cfg.max_iter = max_iter

    def set_qp_tolerance(self, tol: float) -> None:
        """IPM stopping tolerance of every QP (default 1e-10; 1e-8 is Clarabel's default, which the
        reference runs with: control/rqp_cadmm.py:492). Must lie in [1e-12, 1e-7]."""
        L.check(self._lib.dat_set_qp_tolerance(self._h, float(tol)))

    def set_persistent_blocks(self, blocks: int) -> None:
        """C-ADMM / DD: resident k_cadmm / k_dd workgroups draining the scenario queues (0: default)."""
        L.check(self._lib.dat_set_persistent_blocks(self._h, int(blocks)))

    def reset_warm_start(self) -> None:
        L.check(self._lib.dat_reset_warm_start(self._h))

    # -- state
    def set_state(self, states: np.ndarray, counters: Optional[np.ndarray] = None) -> None:
        states = L.f64(states)
        assert states.shape == (self.batch, layout.state_size(self.n))
        c = None if counters is None else L.i32(counters)
        L.check(self._lib.dat_set_state(self._h, L.ptr(states), None if c is None else L.ptr(c, L.I)))

    def get_state(self):
        st = np.empty((self.batch, layout.state_size(self.n)))
        c = np.empty(self.batch, dtype=np.int32)
        L.check(self._lib.dat_get_state(self._h, L.ptr(st), L.ptr(c, L.I)))
        return st, c

    # -- steps
    def control(self, states: Optional[np.ndarray] = None, acc_des: Optional[np.ndarray] = None) -> StepResult:
        B, n = self.batch, self.n
        st = None if states is None else L.f64(states)
        acc = None if acc_des is None else L.f64(acc_des)
        if st is not None:
            assert st.shape == (B, layout.state_size(n))
        if acc is not None:
            assert acc.shape == (B, 6)
        f = np.empty((B, 3 * n))
        it = np.empty(B, dtype=np.int32)
        qs = np.empty((B, n), dtype=np.int32)
        md = np.empty(B)
        col = np.empty(B, dtype=np.uint8)
        err = np.empty((B, self.cfg.max_iter + 1)) if self.cfg.record_err else None
        _, _, _, ms0 = self.counters()
        L.check(self._lib.dat_control_step(self._h, L.ptr(st), L.ptr(acc), L.ptr(f), L.ptr(it, L.I), L.ptr(qs, L.I),
                                           L.ptr(md), L.ptr(col, L.U8), L.ptr(err)))
        _, _, _, ms1 = self.counters()
        return StepResult(f.reshape(B, n, 3).transpose(0, 2, 1), it, qs, md, col.astype(bool), err, ms1 - ms0)

    def set_low_level(self, so3_controller_type: str) -> None:
        """Low-level law of rollout / closed_loop: "pd" (default) or "sm" (control/rqp_centralized.py:468-482)."""
        if so3_controller_type not in L.LL_KINDS:
            raise NotImplementedError(so3_controller_type)
        L.check(self._lib.dat_set_low_level(self._h, L.LL_KINDS[so3_controller_type]))

    def low_level(self, f_des: Optional[np.ndarray] = None):
        """RQPLowLevelController.control at the current states: (thrust (B, n), moment (B, 3, n))."""
        B, n = self.batch, self.n
        fd = None
        if f_des is not None:
            fd = L.f64(np.asarray(f_des, float).reshape(B, 3, n).transpose(0, 2, 1).reshape(B, 3 * n))
        f = np.empty((B, n))
        M = np.empty((B, n, 3))
        L.check(self._lib.dat_low_level_control(self._h, L.ptr(fd), L.ptr(f), L.ptr(M)))
        return f, M.transpose(0, 2, 1)

    def rollout(self, steps: int, f_des: Optional[np.ndarray] = None) -> None:
        fd = None
        if f_des is not None:
            fd = L.f64(np.asarray(f_des).transpose(0, 2, 1).reshape(self.batch, 3 * self.n))
        L.check(self._lib.dat_rollout(self._h, int(steps), L.ptr(fd)))

    def rp_rollout(self, steps: int, f: Optional[np.ndarray] = None) -> None:
        """Rigid-payload dynamics (dat_rp_rollout) with forces f (B, 3, n) held for `steps` steps."""
        fd = None
        if f is not None:
            fd = L.f64(np.asarray(f).transpose(0, 2, 1).reshape(self.batch, 3 * self.n))
        L.check(self._lib.dat_rp_rollout(self._h, int(steps), L.ptr(fd)))

    def set_sub_batches(self, count: int) -> None:
        """dat_set_sub_batches: closed_loop on `count` sub-batches with one stream each (C-ADMM)."""
        L.check(self._lib.dat_set_sub_batches(self._h, int(count)))

    def closed_loop(self, hl_steps: int) -> None:
        L.check(self._lib.dat_closed_loop(self._h, int(hl_steps)))

    def control_steps(self, acc_seq: np.ndarray) -> StepResult:
        """dat_control_steps: acc_seq (K, B, 6) -> K fused control steps of every scenario from the resident
        states (C-ADMM / DD without a forest); the result holds the last step's outputs.  The fused path
        evaluates no environment rows: min_env_dist is NaN and collision None (not computed)."""
        acc_seq = L.f64(acc_seq)
        K = acc_seq.shape[0]
        assert acc_seq.shape[1:] == (self.batch, 6), acc_seq.shape
        f = np.zeros((self.batch, 3 * self.n))
        it = np.zeros(self.batch, dtype=np.int32)
        qs = np.zeros((self.batch, self.n), dtype=np.int32)
        L.check(self._lib.dat_control_steps(self._h, int(K), L.ptr(acc_seq), L.ptr(f), L.ptr(it, L.I),
                                            L.ptr(qs, L.I)))
        return StepResult(f.reshape(self.batch, self.n, 3).transpose(0, 2, 1).copy(), it, qs,
                          np.full(self.batch, np.nan), None)

    def step_marks(self) -> np.ndarray:
        """Host clock marks [ms] of the last closed_loop call (dat_get_step_marks): its start, then each
        HL step's control-kernel completion.  With sub-batch streams (set_sub_batches > 1) only the run's
        start and end: np.diff gives one whole-run time, not per-step times."""
        m = self._lib.dat_get_step_marks(self._h, None, 0)
        if m < 0:
            L.check(m)
        out = np.zeros(m)
        self._lib.dat_get_step_marks(self._h, L.ptr(out), m)
        return out

    def env_rows(self):
        B, n = self.batch, self.n
        lhs = np.empty((B, n, layout.NENV, 3))
        rhs = np.empty((B, n, layout.NENV))
        nr = np.empty((B, n), dtype=np.int32)
        col = np.empty((B, n), dtype=np.uint8)
        md = np.empty((B, n))
        L.check(self._lib.dat_env_rows(self._h, L.ptr(lhs), L.ptr(rhs), L.ptr(nr, L.I), L.ptr(col, L.U8), L.ptr(md)))
        return lhs, rhs, nr, col.astype(bool), md

    def solve_agent_qps(self, scenario, agent, acc_des, lam=None, rho=None, f_mean=None, c=None) -> dict:
        """Raw batched agent QPs (dat_solve_agent_qp_batch): RQPPrimalSolver.solve of C-ADMM
        (control/rqp_cadmm.py:482-501; lam, f_mean (K, 3, n), rho (K,)) or DD (control/rqp_dd.py:475-505;
        c (K, 9) = (c_fi, c_Fi, c_Mi)) at the handle's current states.  Returns x ((K, 3, n) C-ADMM copies
        f, or (K, 9) DD (f_i, F_i, M_i)), status, ipm_iters, collision, min_env_dist."""
        n = self.n
        sc, ag = L.i32(np.atleast_1d(scenario)), L.i32(np.atleast_1d(agent))
        K = sc.shape[0]
        acc = L.f64(acc_des).reshape(K, 6)
        dd = self.mode == L.MODE_DD
        if dd:
            cc = L.f64(c).reshape(K, 9)
            la = rh = fm = None
            x = np.empty((K, 9))
        else:
            cc = None
            la = L.f64(np.asarray(lam, float).reshape(K, 3, n).transpose(0, 2, 1).reshape(K, 3 * n))
            fm = L.f64(np.asarray(f_mean, float).reshape(K, 3, n).transpose(0, 2, 1).reshape(K, 3 * n))
            rh = L.f64(np.broadcast_to(np.asarray(rho, float), (K,)))
            x = np.empty((K, 3 * n))
        st = np.empty(K, dtype=np.int32)
        it = np.empty(K, dtype=np.int32)
        col = np.empty(K, dtype=np.uint8)
        md = np.empty(K)
        L.check(self._lib.dat_solve_agent_qp_batch(self._h, K, L.ptr(sc, L.I), L.ptr(ag, L.I), L.ptr(acc), L.ptr(la),
                                                   L.ptr(rh), L.ptr(fm), L.ptr(cc), L.ptr(x), L.ptr(st, L.I),
                                                   L.ptr(it, L.I), L.ptr(col, L.U8), L.ptr(md)))
        if not dd:
            x = x.reshape(K, n, 3).transpose(0, 2, 1)
        return {"x": x, "status": st, "ipm_iters": it, "collision": col.astype(bool), "min_env_dist": md}

    def counters(self):
        """(agent-QP solves, IPM iterations, HL steps, summed HL kernel ms) since the last reset."""
        w = self.work()
        return w["qp_solves"], w["ipm_iters"], w["hl_steps"], w["hl_kernel_ms"]

    def work(self) -> dict:
        """Device work counters since the last reset (dat_get_counters)."""
        q, it, rw, hs, ms = (ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong(),
                             ctypes.c_double())
        L.check(self._lib.dat_get_counters(self._h, ctypes.byref(q), ctypes.byref(it), ctypes.byref(rw),
                                           ctypes.byref(hs), ctypes.byref(ms)))
        ib, lo = ctypes.c_longlong(), ctypes.c_longlong()
        L.check(self._lib.dat_get_inband_exits(self._h, ctypes.byref(ib), ctypes.byref(lo)))
        rp, rc = ctypes.c_longlong(), ctypes.c_longlong()
        L.check(self._lib.dat_get_refinement_counters(self._h, ctypes.byref(rp), ctypes.byref(rc)))
        rr = ctypes.c_longlong()
        if hasattr(self._lib, "dat_get_robust_redos"):  # absent only from an older A/B build (DAT_LIB_PATH)
            L.check(self._lib.dat_get_robust_redos(self._h, ctypes.byref(rr)))
        out = {"qp_solves": q.value, "ipm_iters": it.value, "ipm_row_iters": rw.value, "hl_steps": hs.value,
               "hl_kernel_ms": ms.value, "inband_exits": ib.value, "inband_beyond_clarabel_tol": lo.value,
               "refine_passes": rp.value, "refine_corrections": rc.value, "robust_redos": rr.value}
        if hasattr(self._lib, "dat_get_tail_counters"):  # absent only from an older A/B build (DAT_LIB_PATH)
            tc = (ctypes.c_longlong * 6)()
            L.check(self._lib.dat_get_tail_counters(self._h, tc))
            out.update(tail_passes=tc[0], tail_critical_ipm_iters=tc[1], tail_routed=tc[2], certified_infeasible=tc[3],
                       stall_exits=tc[4], warm_starts=tc[5])
            col, md = ctypes.c_longlong(), ctypes.c_double()
            L.check(self._lib.dat_get_collision_stats(self._h, ctypes.byref(col), ctypes.byref(md)))
            out.update(collisions=col.value, min_env_dist=md.value)
        return out

    def agent_qp_ms(self) -> float:
        """Device time of the last solve_agent_qps launch (dat_get_agent_qp_ms)."""
        ms = ctypes.c_double()
        L.check(self._lib.dat_get_agent_qp_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def class_work(self, env_class: int) -> dict:
        """C-ADMM only: work counters, summed kernel time and SIMD occupancy of one env class (0:
        scenarios whose agent QPs carry no env CBF row in the step; 1, 2, 3: at most 2, 5, 10 env rows
        per agent QP) -- dat_get_class_counters, dat_get_class_occupancy."""
        q, it, rw, ms = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_double()
        L.check(self._lib.dat_get_class_counters(self._h, int(env_class), ctypes.byref(q), ctypes.byref(it),
                                                 ctypes.byref(rw), ctypes.byref(ms)))
        sl, wp = ctypes.c_longlong(), ctypes.c_longlong()
        L.check(self._lib.dat_get_class_occupancy(self._h, int(env_class), ctypes.byref(sl), ctypes.byref(wp)))
        return {"qp_solves": q.value, "ipm_iters": it.value, "ipm_row_iters": rw.value, "kernel_ms": ms.value,
                "slot_ipm_iters": sl.value, "wave_admm_iters": wp.value}

    def kernel_ms(self) -> float:
        """Summed device time of k_cadmm / k_dd since the last counter reset (dat_get_kernel_ms)."""
        ms = ctypes.c_double()
        L.check(self._lib.dat_get_kernel_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def reset_counters(self) -> None:
        L.check(self._lib.dat_reset_counters(self._h))

    def synchronize(self) -> None:
        L.check(self._lib.dat_synchronize(self._h))


# ================================================================================================
# drop-in single-scenario controllers
# ================================================================================================
class _DropIn:
    _mode = None

    def __init__(self, params: RQPParameters, col: RQPCollision, state: RQPState, dt: float, env: Any = None,
                 verbose: bool = False, device: int = 0) -> None:
        assert params.n >= 3
        self.n = params.n
        self.params, self.col, self.dt, self.env, self.verbose = params, col, dt, env, verbose
        self.max_f_ang = np.pi / 6.0
        self.dist_eps = 0.1
        self.vision_radius = col.collision_radius + 5.0
        self._eng = BatchedController(self._mode, self.n, 1, pack_params(params, col), dt=dt, device=device,
                                      record_err=self._mode != L.MODE_CENTRALIZED)
        if env is not None:
            self._eng.set_forests([env])

    def control(self, state, acc_des):
        acc = np.concatenate([np.asarray(acc_des[0], float), np.asarray(acc_des[1], float)])[None]
        r = self._eng.control(pack_state(state)[None], acc)
        f = r.f_des[0]
        if self._mode == L.MODE_CENTRALIZED:
            return f, SolverStatistics(-1, r.gpu_ms * 1e-3, bool(r.collision[0]), float(r.min_env_dist[0]))
        it = int(r.iters[0])
        err = r.err_seq[0][: max(it - 1, 0)].tolist() if r.err_seq is not None else []
        err = [e for e in err if e == e]
        return f, SolverStatistics(it, r.gpu_ms * 1e-3, bool(r.collision[0]), float(r.min_env_dist[0]), err)

    def set_qp_tolerance(self, tol: float) -> None:
        """Extension (no reference counterpart): IPM stopping tolerance, 1e-8 = Clarabel's default."""
        self._eng.set_qp_tolerance(tol)

    def get_force_cone_angle_bound(self) -> float:
        return self.max_f_ang

    def get_dist_eps(self) -> float:
        return self.dist_eps


class RQPCentralizedController(_DropIn):
    _mode = L.MODE_CENTRALIZED


class RQPCADMMController(_DropIn):
    _mode = L.MODE_CADMM

    def set_force_err_tolerance(self, tol: float, use_total_res: bool = True) -> None:
        self._eng.set_force_err_tolerance(tol, use_total_res)

    def set_max_iter(self, max_iter: int) -> None:
        self._eng.set_max_iter(max_iter)


class RQPDDController(_DropIn):
    _mode = L.MODE_DD

    def set_force_err_tolerance(self, tol: float) -> None:
        self._eng.set_force_err_tolerance(tol, True)

    def set_max_iter(self, max_iter: int) -> None:
        self._eng.set_max_iter(max_iter)


class _PrimalSolver:
    """One agent's QP solver with the reference's per-call interface and status handling, solved by
    k_agent_qp through dat_solve_agent_qp_batch.  ``idx`` is the reference's Index(i, is_leader) or a
    plain agent number; agent 0 is the leader (control/rqp_cadmm.py:553-555; set_leader after
    construction does not change the cost weights)."""

    _mode = None

    def __init__(self, params: RQPParameters, col: RQPCollision, idx: Any, state: RQPState, dt: float,
                 env: Any = None, verbose: bool = False, device: int = 0) -> None:
        assert params.n >= 3
        self.n = params.n
        self.i = int(getattr(idx, "i", idx))
        self.verbose = verbose
        self.params = params
        self._eng = BatchedController(self._mode, self.n, 1, pack_params(params, col), dt=dt, device=device)
        if env is not None:
            self._eng.set_forests([env])
        self.f_eq = equilibrium_forces(params)
        self.collision, self.min_env_dist = False, col.collision_radius + 5.0
        self._set_warm_start()

    def _run(self, state, acc_des, **kw):
        self._eng.set_state(pack_state(state)[None])
        acc = np.concatenate([np.asarray(acc_des[0], float), np.asarray(acc_des[1], float)])[None]
        r = self._eng.solve_agent_qps([0], [self.i], acc, **kw)
        self.collision, self.min_env_dist = bool(r["collision"][0]), float(r["min_env_dist"][0])
        if self.verbose and r["status"][0] != L.QP_OPTIMAL:
            print(f"Problem not solved to optimality, status: {int(r['status'][0])}")
        # solve_time [s]: the device time of the QP kernel, as Clarabel's solver_stats.solve_time is the
        # solver's own time (control/rqp_cadmm.py:500)
        return r, self._eng.agent_qp_ms() * 1e-3


class RQPCADMMPrimalSolver(_PrimalSolver):
    """control/rqp_cadmm.py:26-507: solve(state, acc_des, lambda_f, cadmm_rho, f_mean) ->
    (f (3, n), solve_time, collision, min_env_dist).  Exception -> f_eq (:491-494); non-OPTIMAL ->
    previous solution (:496-499).  The reference's default cadmm_rho = 0 (:487) is used only by its
    constructor's warm-up solve (:131-140), where the copies f_j, j != i, are not unique (that solve only seeds
    Clarabel's warm start); here cadmm_rho defaults to the controller's initial penalty rho0 = 1
    (control/rqp_cadmm.py:564), and an explicit rho <= 0 raises ValueError instead of silently solving another
    QP."""

    _mode = L.MODE_CADMM

    def _set_warm_start(self) -> None:
        self.prev_f = self.f_eq.copy()

    RHO0 = 1.0  # RQPCADMMController.rho0 (control/rqp_cadmm.py:564)

    def solve(self, state, acc_des, lambda_f=None, cadmm_rho: Optional[float] = None, f_mean=None):
        n = self.n
        if cadmm_rho is None:
            cadmm_rho = self.RHO0
        if not float(cadmm_rho) > 0.0:
            raise ValueError(f"cadmm_rho must be > 0 (got {cadmm_rho}): at rho = 0 the agent QP's copies f_j, "
                             "j != i, are not unique (the reference uses rho = 0 only for its constructor's "
                             "warm-up solve, control/rqp_cadmm.py:131-140)")
        lam = np.zeros((3, n)) if lambda_f is None else np.asarray(lambda_f, float)
        fm = np.zeros((3, n)) if f_mean is None else np.asarray(f_mean, float)
        r, t = self._run(state, acc_des, lam=lam[None], rho=[cadmm_rho], f_mean=fm[None])
        st = int(r["status"][0])
        if st == L.QP_FAILED:
            self.prev_f = self.f_eq.copy()
        elif st == L.QP_OPTIMAL:
            self.prev_f = r["x"][0].copy()
        return self.prev_f, t, self.collision, self.min_env_dist


class RQPDDPrimalSolver(_PrimalSolver):
    """control/rqp_dd.py:27-511: solve(state, acc_des, c_fi, c_Fi, c_Mi) -> (f_i, F_i, M_i, solve_time,
    collision, min_env_dist).  Exception -> (f_eq,i, sum f_eq - f_eq,i, -JT^-1 hat(r_com,i) f_eq,i)
    (:484-489); non-OPTIMAL -> previous solution."""

    _mode = L.MODE_DD

    def _set_warm_start(self) -> None:
        p, i = self.params, self.i
        self.prev_fi = self.f_eq[:, i].copy()
        self.prev_Fi = np.sum(self.f_eq, axis=1) - self.prev_fi
        self.prev_Mi = -p.JT_inv @ _skew(p.r_com[:, i]) @ self.prev_fi

    def solve(self, state, acc_des, c_fi=np.zeros(3), c_Fi=np.zeros(3), c_Mi=np.zeros(3)):
        c = np.concatenate([np.asarray(c_fi, float), np.asarray(c_Fi, float), np.asarray(c_Mi, float)])
        r, t = self._run(state, acc_des, c=c[None])
        st = int(r["status"][0])
        if st == L.QP_FAILED:
            self._set_warm_start()
        elif st == L.QP_OPTIMAL:
            x = r["x"][0]
            self.prev_fi, self.prev_Fi, self.prev_Mi = x[:3].copy(), x[3:6].copy(), x[6:].copy()
        return self.prev_fi, self.prev_Fi, self.prev_Mi, t, self.collision, self.min_env_dist


class RQPLowLevelController:
    """control/rqp_centralized.py:457-535: RQPLowLevelController(so3_controller_type, params, max_f_ang)
    .control(state, f_des) -> (f (n,), M (3, n)); "pd" or "sm" SO(3) law, evaluated on the GPU
    (k_low_level).  Unknown types raise NotImplementedError like the reference (:483-484)."""

    def __init__(self, so3_controller_type: str, params: RQPParameters, max_f_ang: float, device: int = 0) -> None:
        if so3_controller_type not in L.LL_KINDS:
            raise NotImplementedError(so3_controller_type)
        self.n = params.n
        self.cos_max_f_ang = np.cos(max_f_ang)
        col = RQPCollision(np.zeros((1, 3)), np.zeros((1, 3)))  # the LL law reads only J
        self._eng = BatchedController(L.MODE_CADMM, self.n, 1, pack_params(params, col), device=device)
        self._eng.set_low_level(so3_controller_type)

    def control(self, state, f_des: np.ndarray):
        f_des = np.asarray(f_des, float)
        assert f_des.shape == (3, state.n)
        assert all(f_des[2, :] > 0.0)
        self._eng.set_state(pack_state(state)[None])
        f, M = self._eng.low_level(f_des[None])
        return f[0], M[0]


class RQPClosedLoop:
    """One scenario's closed loop on the GPU (example/rqp_example.py:120-131): HL control every
    ``hl_rel_freq`` steps from the given desired accelerations, SO(3) PD low level and dynamics
    at every step.  ``step(acc_des)`` advances one high-level period."""

    def __init__(self, controller: _DropIn, state: RQPState, hl_rel_freq: int = 10) -> None:
        self.ctrl = controller
        self.hl = hl_rel_freq
        self.ctrl._eng.set_state(pack_state(state)[None], np.zeros(1, dtype=np.int32))

    def step(self, acc_des=None):
        eng = self.ctrl._eng
        acc = None
        if acc_des is not None:
            acc = np.concatenate([np.asarray(acc_des[0], float), np.asarray(acc_des[1], float)])[None]
        r = eng.control(None, acc)
        eng.rollout(self.hl)
        return r

    @property
    def state(self) -> RQPState:
        st, _ = self.ctrl._eng.get_state()
        return RQPState.unpack(st[0], self.ctrl.n)


__all__ = ["BatchedController", "StepResult", "SolverStatistics", "RQPCentralizedController", "RQPCADMMController",
           "RQPDDController", "RQPClosedLoop", "RQPCADMMPrimalSolver", "RQPDDPrimalSolver", "RQPLowLevelController"]
