"""GPU parity: the HIP path (libdat.so through the C-ABI) against the CPU oracle and the golden
fixtures produced by the reference's own code.  Run with ``-m gpu`` on an MI355X.

Tolerances (north_star): per-step controls within 1e-5 relative (relative to the largest force
component of the step), closed-loop states within 1e-4.
"""

import numpy as np
import pytest

from oracle import controllers as oc
from oracle import forest as of
from oracle import model as om
from oracle import scenarios as osc
from tests._golden import load, state_from, unpack_flat

pytestmark = pytest.mark.gpu

REL = 1e-5
# Residual sequences (err_seq) are consensus errors F_i - sum_j f_j: differences of forces of order
# m_T g (17-30 N) that shrink to ~1e-2, so they inherit the agent-QP solution error amplified by that
# cancellation.  tools/dd_sensitivity.py runs the ORACLE against itself on the DD step test's
# scenarios: IPM tolerance 1e-10 vs 1e-11 moves err_seq by up to 9.6e-5 relative (1.3e-6 N
# absolute at err ~ 1e-2), 1e-12 vs 1e-11 by 1.6e-5, while an explicit H^-1 instead of cho_solve
# moves it by 2e-11.  The comparison is therefore rtol 1e-4 OR 2e-6 N absolute (1e-7 of m_T g).
ERR_RTOL, ERR_ATOL = 1e-4, 2e-6
# DD err_seq by team size where the oracle's own sensitivity is larger (tools/dd_sensitivity.py n: IPM
# tolerance 1e-11 -> 1e-10 moves the oracle's err_seq by 1.05e-2 relative at n = 4, 7.7e-4 at n = 11
# and 5.7e-3 at n = 16 -- those teams' agent QPs are strongly convex only through the 1e-6
# regularisation in some directions, so the solution moves ~tol / 1e-6 -- against 4.3e-5 at n = 3,
# 9.6e-5 at n = 6 and 2.7e-5 at n = 8): 3x the measured change.
DD_ERR_RTOL = {4: 3e-2, 11: 2.5e-3, 16: 1.8e-2}


def _eng(mode, n, B, **kw):
    from distributed_aerial_transportation_amd import BatchedController, scenarios

    return BatchedController(mode, n, B, scenarios.params_block(n), **kw)


def _ostate(x, n):
    from distributed_aerial_transportation_amd.system import RQPState

    s = RQPState.unpack(x, n)
    return om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def test_gpu_env_rows_match_oracle():
    from distributed_aerial_transportation_amd import system as S

    d = load("ref_env_rows.npz")
    K = d["lhs_d"].shape[0]
    states = np.stack([S.pack_state(state_from(d, "s_", k)) for k in range(K)])
    eng = _eng("cadmm", 3, K)
    f = of.Forest.__new__(of.Forest)
    f.tree_pos = d["tree_pos"]
    f.num_trees = f.tree_pos.shape[0]
    f.mountain_center, f.mountain_radius = of.MOUNTAIN_CENTER, of.MOUNTAIN_RADIUS
    f.mountain_sphere_radius, f.mountain_center_depth = 87.0, 83.3
    eng.set_forests([f])
    eng.set_state(states)
    lhs, rhs, nr, col, md = eng.env_rows()
    for k in range(K):
        for i in range(3):
            L, R = d["lhs_d"][k, i], d["rhs_d"][k, i]
            keep = np.any(np.abs(L) > 1e-12, axis=1) | (R > 0)
            exp = sorted(map(tuple, np.column_stack([L[keep], R[keep]])))
            gl, gr = lhs[k, i, : nr[k, i]], rhs[k, i, : nr[k, i]]
            keep2 = np.any(np.abs(gl) > 1e-12, axis=1) | (gr > 0)
            got = sorted(map(tuple, np.column_stack([gl[keep2], gr[keep2]])))
            assert len(got) == len(exp)
            if got:
                np.testing.assert_allclose(np.array(got), np.array(exp), atol=1e-9)
            assert bool(col[k, i]) == bool(d["col_d"][k, i])
            assert md[k, i] == pytest.approx(float(d["md_d"][k, i]), abs=1e-8)


@pytest.mark.parametrize("n", [3, 6, 16])
def test_gpu_cadmm_step_matches_oracle(n):
    from distributed_aerial_transportation_amd import scenarios

    B = 6 if n < 16 else 2  # n = 16: config C5 geometry (ring of 16), a few oracle seconds per step
    rng = np.random.default_rng(n)
    states = scenarios.perturbed_states(n, B, rng)
    acc = np.concatenate([rng.uniform(-3, 3, (B, 3)), rng.uniform(-3, 3, (B, 3))], axis=1)
    eng = _eng("cadmm", n, B, record_err=True)
    # two consecutive steps exercise the warm start (f, f_mean, lambda persist)
    r1 = eng.control(states, acc)
    r2 = eng.control(states, acc[::-1].copy())
    for b in range(B):
        ctl = oc.CADMM(osc.params(n), osc.col_radius(n))
        s = _ostate(states[b], n)
        f1, st1 = ctl.control(s, (acc[b, :3], acc[b, 3:]))
        f2, st2 = ctl.control(s, (acc[B - 1 - b, :3], acc[B - 1 - b, 3:]))
        assert r1.iters[b] == st1.iter and r2.iters[b] == st2.iter
        assert _rel(r1.f_des[b], f1) < REL and _rel(r2.f_des[b], f2) < REL
        np.testing.assert_allclose(r1.err_seq[b, : st1.iter - 1], st1.err_seq, rtol=1e-4, atol=1e-6)
        assert np.all(r1.qp_status[b] == 0)
    assert eng.work()["inband_beyond_clarabel_tol"] == 0


def test_gpu_cadmm_convergence_recipe_golden():
    """_plot_convergence_rate (test/control/test_rqpcontrollers.py:101-124): tol 0, 25 iterations,
    aggregate residual -- against the reference's own loop (ref_cadmm.npz)."""
    from distributed_aerial_transportation_amd import scenarios, system

    d = load("ref_cadmm.npz")
    eng = _eng("cadmm", 3, 1, record_err=True)
    eng.set_force_err_tolerance(0.0, False)
    eng.set_max_iter(25)
    x = system.pack_state(scenarios.rest_state(3))[None]
    for k in range(d["fixed_err"].shape[0]):
        a = d["acc"][k][None]
        r = eng.control(x, a)
        assert r.iters[0] == 26
        np.testing.assert_allclose(r.err_seq[0, :25], d["fixed_err"][k], rtol=1e-4, atol=1e-7)
        assert _rel(r.f_des[0], d["fixed_f"][k]) < REL


def test_gpu_cadmm_default_tolerance_golden():
    from distributed_aerial_transportation_amd import scenarios, system

    d = load("ref_cadmm.npz")
    eng = _eng("cadmm", 3, 1)
    x = system.pack_state(scenarios.rest_state(3))[None]
    for k in range(d["tol_iters"].shape[0]):
        r = eng.control(x, d["acc"][k][None])
        assert r.iters[0] == d["tol_iters"][k]
        assert _rel(r.f_des[0], d["tol_f"][k]) < REL


def _ambiguous(seq, tol=1e-2, band=1e-7):
    """The reference stops when err < tol; a residual within `band` (relative) of tol can flip the count
    (such scenarios are excluded from exact-count checks, and tests assert they are rare)."""
    return any(abs(e - tol) < band * tol for e in seq)


@pytest.mark.parametrize("n", [3, 4, 6, 8, 11, 16])
def test_gpu_dd_step_matches_oracle(n):
    """DD control step (control/rqp_dd.py:695-752) incl. the warm multipliers of a second step:
    iteration counts exact, f_des within 1e-5, residual sequences within 1e-4 relative.  n <= 8 runs
    k_dd_setup<n> (H columns in registers), n = 11 and 16 the LDS path (k_dd_setup<0>, > 64 KB LDS)."""
    from distributed_aerial_transportation_amd import scenarios

    B = 6
    rng = np.random.default_rng(10 + n)
    states = scenarios.perturbed_states(n, B, rng)
    acc = np.concatenate([rng.uniform(-3, 3, (B, 3)), rng.uniform(-3, 3, (B, 3))], axis=1)
    eng = _eng("dd", n, B, record_err=True)
    r1 = eng.control(states, acc)
    r2 = eng.control(states, acc[::-1].copy())
    skipped = 0
    for b in range(B):
        ctl = oc.DD(osc.params(n), osc.col_radius(n))
        s = _ostate(states[b], n)
        f1, st1 = ctl.control(s, (acc[b, :3], acc[b, 3:]))
        f2, st2 = ctl.control(s, (acc[B - 1 - b, :3], acc[B - 1 - b, 3:]))
        # a residual within the team size's own err_seq sensitivity of the stopping tolerance can stop
        # one iteration earlier or later (the oracle against itself does at n = 16)
        rtol = DD_ERR_RTOL.get(n, ERR_RTOL)
        band = rtol / 3 if n in DD_ERR_RTOL else 1e-7  # the measured sensitivity itself
        if _ambiguous(st1.err_seq, band=band) or _ambiguous(st2.err_seq, band=band):
            skipped += 1
            continue
        assert r1.iters[b] == st1.iter and r2.iters[b] == st2.iter, (b, r1.iters[b], st1.iter, r2.iters[b], st2.iter)
        assert _rel(r1.f_des[b], f1) < REL and _rel(r2.f_des[b], f2) < REL, (_rel(r1.f_des[b], f1), _rel(r2.f_des[b], f2))
        np.testing.assert_allclose(r1.err_seq[b, : st1.iter - 1], st1.err_seq, rtol=rtol, atol=ERR_ATOL)
        np.testing.assert_allclose(r2.err_seq[b, : st2.iter - 1], st2.err_seq, rtol=rtol, atol=ERR_ATOL)
        assert np.all(r1.qp_status[b] == 0) and np.all(r2.qp_status[b] == 0)
    assert skipped <= (2 if n in DD_ERR_RTOL else 1)
    assert eng.work()["inband_beyond_clarabel_tol"] == 0


def _random_mass_params(n, B, rng):
    """Config C3: per-scenario payload mass ml ~ U(0.15, 0.30), inertia Jl * U(0.8, 1.2)^3 --
    packed blocks for the GPU and the matching oracle Params."""
    from distributed_aerial_transportation_amd import scenarios, system

    m, J, _, Jl0, r = osc.geometry(n)
    col = scenarios.collision(n)
    blocks, ops = [], []
    for _ in range(B):
        ml, Jl = rng.uniform(0.15, 0.30), Jl0 * np.diag(rng.uniform(0.8, 1.2, 3))
        blocks.append(system.pack_params(system.RQPParameters(m, J, ml, Jl, r), col))
        ops.append(om.Params(m, J, ml, Jl, r))
    return np.stack(blocks), ops


@pytest.mark.parametrize("mode", ["cadmm", "dd"])
def test_gpu_per_scenario_params_match_oracle(mode):
    """Randomised payload mass / inertia per scenario (config C3) through dat_set_params(per_scenario=1)."""
    from distributed_aerial_transportation_amd import BatchedController, scenarios

    n, B = 6, 3
    rng = np.random.default_rng(77)
    blocks, ops = _random_mass_params(n, B, rng)
    states = scenarios.perturbed_states(n, B, rng)
    acc = rng.uniform(-0.5, 0.5, (B, 6)) * 10.0
    eng = BatchedController(mode, n, B, blocks, per_scenario_params=True)
    r = eng.control(states, acc)
    for b in range(B):
        ctl = (oc.CADMM if mode == "cadmm" else oc.DD)(ops[b], osc.col_radius(n))
        f, st = ctl.control(_ostate(states[b], n), (acc[b, :3], acc[b, 3:]))
        if _ambiguous(st.err_seq):
            continue
        assert r.iters[b] == st.iter, (b, r.iters[b], st.iter)
        assert _rel(r.f_des[b], f) < REL, (b, _rel(r.f_des[b], f))


def test_gpu_dd_golden():
    from distributed_aerial_transportation_amd import scenarios, system

    d = load("ref_dd.npz")
    x = system.pack_state(scenarios.rest_state(3))[None]
    eng = _eng("dd", 3, 1, record_err=True)
    eng.set_force_err_tolerance(0.0)
    eng.set_max_iter(25)
    for k in range(d["fixed_err"].shape[0]):
        r = eng.control(x, d["acc"][k][None])
        # converged tails sit at the 1e-14 rounding floor: absolute tolerance 1e-9 there
        np.testing.assert_allclose(r.err_seq[0, :25], d["fixed_err"][k], rtol=1e-4, atol=1e-9)
        assert _rel(r.f_des[0], d["fixed_f"][k]) < REL
    eng = _eng("dd", 3, 1, record_err=True)
    for k in range(d["tol_iters"].shape[0]):
        r = eng.control(x, d["acc"][k][None])
        assert r.iters[0] == d["tol_iters"][k]
        assert _rel(r.f_des[0], d["tol_f"][k]) < REL
        it = int(d["tol_iters"][k])
        np.testing.assert_allclose(r.err_seq[0, : it - 1], d["tol_err"][k][: it - 1], rtol=ERR_RTOL, atol=ERR_ATOL)


@pytest.mark.parametrize("n", [3, 4, 5, 6, 8, 11, 16])
def test_gpu_centralized_step_matches_oracle(n):
    """Centralized control step (control/rqp_centralized.py:27-455, generic in n) for team sizes on
    every lane-group width of k_cent<W> (dat_cent.hip: W = 4 for n <= 4, 8 for n <= 8, 16 up to 16;
    lanes n .. W-1 of a group are phantoms, B = 5 leaves most groups of the wavefront empty): two steps
    (the held previous solution persists), f_des within 1e-5 of the oracle's dense IPM, statuses OPTIMAL."""
    from distributed_aerial_transportation_amd import scenarios

    B = 5
    rng = np.random.default_rng(40 + n)
    states = scenarios.perturbed_states(n, B, rng)
    acc = np.concatenate([rng.uniform(-3, 3, (B, 3)), rng.uniform(-3, 3, (B, 3))], axis=1)
    eng = _eng("centralized", n, B)
    r1 = eng.control(states, acc)
    r2 = eng.control(states, acc[::-1].copy())
    assert eng.work()["inband_beyond_clarabel_tol"] == 0
    for b in range(B):
        ctl = oc.Centralized(osc.params(n), osc.col_radius(n))
        s = _ostate(states[b], n)
        f1, _ = ctl.control(s, (acc[b, :3], acc[b, 3:]))
        f2, _ = ctl.control(s, (acc[B - 1 - b, :3], acc[B - 1 - b, 3:]))
        assert _rel(r1.f_des[b], f1) < REL and _rel(r2.f_des[b], f2) < REL, (b, _rel(r1.f_des[b], f1), _rel(r2.f_des[b], f2))
        assert np.all(r1.qp_status[b] == 0) and np.all(r2.qp_status[b] == 0)


@pytest.mark.parametrize("n", [3, 6, 16])
def test_gpu_centralized_forest_rows_match_oracle(n):
    """Centralized QPs with binding forest CBF rows (control/rqp_centralized.py:280-337: the capsule
    distance to every tree in range, no vision cone, alpha_env = 2): payloads 1.6-2.8 m in front of a
    tree and moving towards it; f_des within 1e-5 of the oracle with its forest, collision flags and
    minimum distances equal."""
    from distributed_aerial_transportation_amd import Forest
    from tests.test_gpu_c4 import _oforest, near_tree_states

    B = 12
    rng = np.random.default_rng(70 + n)
    forests = [Forest.seeded(s) for s in range(4)]
    sf = np.arange(B, dtype=np.int32) % 4
    states = near_tree_states(n, forests, sf, rng)
    acc = np.concatenate([rng.uniform(-1, 1, (B, 3)), np.zeros((B, 3))], axis=1)
    eng = _eng("centralized", n, B)
    eng.set_forests(forests, sf)
    r = eng.control(states, acc)
    assert eng.work()["inband_beyond_clarabel_tol"] == 0
    for b in range(B):
        ctl = oc.Centralized(osc.params(n), osc.col_radius(n), _oforest(forests[sf[b]]))
        f, st = ctl.control(_ostate(states[b], n), (acc[b, :3], acc[b, 3:]))
        assert _rel(r.f_des[b], f) < REL, (b, _rel(r.f_des[b], f))
        assert bool(r.collision[b]) == bool(st.collision)
        assert abs(r.min_env_dist[b] - st.min_env_dist) < 1e-6


def test_gpu_centralized_golden():
    from distributed_aerial_transportation_amd import scenarios, system

    d = load("ref_central.npz")
    eng = _eng("centralized", 3, d["f"].shape[0])
    x = np.repeat(system.pack_state(scenarios.rest_state(3))[None], d["f"].shape[0], axis=0)
    r = eng.control(x, d["acc"])
    for k in range(d["f"].shape[0]):
        assert _rel(r.f_des[k], d["f"][k]) < REL
    assert np.all(r.iters == -1)


@pytest.mark.parametrize("n,B", [(3, 5), (4, 17), (6, 11), (16, 5)])
def test_gpu_rollout_matches_oracle(n, B):
    """k_rollout_agents (one lane per agent, floor(64/n) scenarios per block, partial last block)
    over 45 steps (two polar projections) vs the oracle's dynamics and integration."""
    from distributed_aerial_transportation_amd import scenarios

    rng = np.random.default_rng(3)
    states = scenarios.perturbed_states(n, B, rng)
    eng = _eng("cadmm", n, B)
    eng.set_state(states, np.zeros(B, dtype=np.int32))
    fdes = np.stack([np.vstack([rng.uniform(-1, 1, (2, n)), rng.uniform(4, 7, (1, n))]) for _ in range(B)])
    eng.rollout(45, fdes)
    got, cnt = eng.get_state()
    p = osc.params(n)
    for b in range(B):
        s = _ostate(states[b], n)
        for _ in range(45):
            f, M = om.low_level_control(p, s, fdes[b])
            s.integrate(*om.forward_dynamics(p, s, f, M), 1e-3)
        g = _ostate(got[b], n)
        for a in ("R", "w", "xl", "vl", "Rl", "wl"):
            np.testing.assert_allclose(getattr(g, a), getattr(s, a), atol=1e-12)
        assert cnt[b] == s.counter


@pytest.mark.parametrize("tag,mode", [("cons", "cadmm"), ("dual", "dd"), ("cent", "centralized")])
def test_gpu_closed_loop_golden(tag, mode):
    """400 ms of rqp_example's loop (forest seed 0, HL every 10 steps) vs the reference's loop."""
    from distributed_aerial_transportation_amd import Forest, scenarios, system

    d = load("ref_closed_loop.npz")
    eng = _eng(mode, 3, 1)
    eng.set_forests([Forest.seeded(0)])
    eng.set_state(system.pack_state(scenarios.rest_state(3))[None], np.zeros(1, dtype=np.int32))
    steps = d[f"{tag}_states"].shape[0] // 10
    for k in range(steps):
        r = eng.control(None, None)  # forest desired-acceleration law on device
        assert _rel(r.f_des[0], d[f"{tag}_f_des"][k]) < REL, k
        if mode != "centralized":
            assert r.iters[0] == d[f"{tag}_iters"][k]
        eng.rollout(10)
        st, _ = eng.get_state()
        ref = d[f"{tag}_states"][10 * k + 9]
        assert np.max(np.abs(st[0] - _reorder(ref))) < 1e-4, k


def _reorder(x, n=3):
    """fixture states are (R (3,3,n) C-order, w (3,n), xl, vl, Rl, wl) -> dat_layout state block"""
    from distributed_aerial_transportation_amd import system

    return system.pack_state(unpack_flat(x, n))


@pytest.mark.parametrize("mode", ["cadmm", "dd", "centralized"])
def test_gpu_failure_branches(mode):
    """Per-QP status handling, against the oracle running the same two steps:
      * scenario 1, payload upside down (Rl = diag(1, -1, -1), wl = 0): the tilt CBF row becomes
        0 . dwl + (Rl[2,2] - cos 15 deg) >= 0 with a negative constant, so every agent QP is
        infeasible -> hold the previous solution (control/rqp_cadmm.py:496-499,
        control/rqp_dd.py:491-496, control/rqp_centralized.py:441-444);
      * scenario 2, NaN payload velocity: every agent QP fails (the solver-exception branch)
        -> f_eq (control/rqp_cadmm.py:491-494; DD control/rqp_dd.py:484-489 incl. quirk a15);
        centralized has no exception branch (rqp_centralized.py:439) and holds its previous f;
      * scenarios 0 and 3 are ordinary and must be unaffected by their neighbours."""
    from distributed_aerial_transportation_amd import _lib as L, scenarios

    n, B = 3, 4
    rng = np.random.default_rng(55)
    x0 = scenarios.perturbed_states(n, B, rng)
    a0 = rng.uniform(-0.5, 0.5, (B, 6)) * 4.0
    x1, a1 = x0.copy(), rng.uniform(-0.5, 0.5, (B, 6)) * 4.0
    x1[1, 12 * n + 6:12 * n + 15] = np.diag([1.0, -1.0, -1.0]).reshape(-1)  # Rl
    x1[1, 12 * n + 15:12 * n + 18] = 0.0                                     # wl
    x1[2, 12 * n + 3:12 * n + 6] = np.nan                                    # vl
    eng = _eng(mode, n, B, record_err=mode != "centralized")
    r0 = eng.control(x0, a0)
    r1 = eng.control(x1, a1)
    assert np.all(r0.qp_status == L.QP_OPTIMAL)
    assert np.all(r1.qp_status[1] == L.QP_INFEASIBLE), r1.qp_status
    assert np.all(r1.qp_status[2] == L.QP_FAILED), r1.qp_status
    assert np.all(r1.qp_status[[0, 3]] == L.QP_OPTIMAL)
    cls = {"cadmm": oc.CADMM, "dd": oc.DD, "centralized": oc.Centralized}[mode]
    for b in range(B):
        ctl = cls(osc.params(n), osc.col_radius(n))
        ctl.control(_ostate(x0[b], n), (a0[b, :3], a0[b, 3:]))
        f1, st1 = ctl.control(_ostate(x1[b], n), (a1[b, :3], a1[b, 3:]))
        assert _rel(r1.f_des[b], f1) < REL, (b, r1.f_des[b], f1)
        assert r1.iters[b] == st1.iter, (b, r1.iters[b], st1.iter)
        if mode != "centralized":  # DD scenario 2: err_seq[0] carries quirk a15's sum of current forces
            np.testing.assert_allclose(r1.err_seq[b, : st1.iter - 1], st1.err_seq, rtol=ERR_RTOL, atol=ERR_ATOL)
    # infeasible: the previous step's forces are held
    assert _rel(r1.f_des[1], r0.f_des[1]) < 1e-12
    if mode == "cadmm":
        feq = om.equilibrium_forces(osc.params(n))
        assert _rel(r1.f_des[2], feq) < 1e-12


def test_gpu_dd_persistent_drain():
    """k_dd drains a sorted scenario queue with slot refill: B = 48 scenarios (n = 6, G = 10 slots per
    workgroup) on a grid capped at 2 workgroups, two consecutive steps (warm multipliers), must give
    exactly the results of the uncapped grid (a scenario's arithmetic does not depend on its slot),
    every agent QP OPTIMAL, and a sample must match the oracle (iterations exact, f_des within 1e-5)."""
    from distributed_aerial_transportation_amd import scenarios

    n, B = 6, 48
    rng = np.random.default_rng(606)
    states = scenarios.perturbed_states(n, B, rng)
    a1 = rng.uniform(-0.5, 0.5, (B, 6)) * 6.0
    a2 = rng.uniform(-0.5, 0.5, (B, 6)) * 6.0
    runs = []
    for blocks in (2, 0):
        eng = _eng("dd", n, B, record_err=True)
        eng.set_persistent_blocks(blocks)
        runs.append((eng.control(states, a1), eng.control(states, a2)))
        assert eng.work()["inband_beyond_clarabel_tol"] == 0
    for r_cap, r_full in zip(*runs):
        np.testing.assert_array_equal(r_cap.f_des, r_full.f_des)
        np.testing.assert_array_equal(r_cap.iters, r_full.iters)
        assert np.all(r_cap.qp_status == 0)
    r1, r2 = runs[0]
    for b in range(0, B, 8):
        ctl = oc.DD(osc.params(n), osc.col_radius(n))
        s = _ostate(states[b], n)
        f1, st1 = ctl.control(s, (a1[b, :3], a1[b, 3:]))
        f2, st2 = ctl.control(s, (a2[b, :3], a2[b, 3:]))
        if _ambiguous(st1.err_seq) or _ambiguous(st2.err_seq):
            continue
        assert r1.iters[b] == st1.iter and r2.iters[b] == st2.iter, (b, r1.iters[b], st1.iter, r2.iters[b], st2.iter)
        assert _rel(r1.f_des[b], f1) < REL and _rel(r2.f_des[b], f2) < REL
