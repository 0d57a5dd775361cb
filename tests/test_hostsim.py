"""CPU checks of the per-lane device code (csrc/dat_core.hpp) via its TEST-ONLY host build
(tests/hostsim): reduced agent-QP solves vs the oracle's uncondensed formulation, env rows vs
the reference-generated fixture, rollout vs the oracle dynamics.  No GPU needed."""

import numpy as np
import pytest

from oracle import model as om
from oracle import scenarios as osc
from oracle.ipm import OPTIMAL, solve_qp
from tests import hostsim as hs
from tests.hostsim import TAIL_PASS, TAIL_PREV
from tests._golden import load, state_from


def _rand_state(rng, n):
    R = np.stack([om.exp3(rng.uniform(-0.3, 0.3, 3)) for _ in range(n)], 2)
    return om.State(R, rng.uniform(-0.5, 0.5, (3, n)), rng.uniform(-1, 1, 3), rng.uniform(-0.5, 0.5, 3),
                    om.exp3(rng.uniform(-0.1, 0.1, 3)), rng.uniform(-0.2, 0.2, 3))


def _prm(n):
    from distributed_aerial_transportation_amd import scenarios

    return scenarios.params_block(n)


def _env_case(d, k, agent):
    L, R = d["lhs_d"][k, agent], d["rhs_d"][k, agent]
    keep = np.any(np.abs(L) > 1e-12, axis=1) | (R > 0)
    return L, R, L[keep], R[keep]


@pytest.mark.parametrize("n", [3, 6, 16])
def test_reduced_cadmm_qp_matches_oracle(n):
    from distributed_aerial_transportation_amd.system import pack_state

    rng = np.random.default_rng(100 + n)
    p = osc.params(n)
    feq = om.equilibrium_forces(p)
    c = om.Consts.make(p, osc.col_radius(n), distributed=True)
    d = load("ref_env_rows.npz")
    for t in range(12):
        s = _rand_state(rng, n)
        acc = (rng.uniform(-5, 5, 3), rng.uniform(-5, 5, 3))
        i = t % n
        lam = rng.normal(0, 0.5, (3, n))
        fm = feq + rng.normal(0, 1, (3, n))
        env = om.EnvRows.empty(c)
        lhs = np.zeros((0, 3))
        rhs = np.zeros(0)
        if n == 3 and t % 2 == 0:
            L, R, lhs, rhs = _env_case(d, t, 0)
            env = om.EnvRows(L, R, False, 1.0)
        P, q, G, h, dims, A, b = om.build_qp("cadmm", p, c, s, acc, env, i=i, f_eq=feq, lam=lam, rho=1.0, f_mean=fm)
        ro = solve_qp(P, q, G, h, dims, A, b)
        f, status, it = hs.qp_cadmm(_prm(n), n, pack_state(s), np.concatenate(acc), lhs, rhs, i, lam.T.reshape(-1),
                                    fm.T.reshape(-1))
        if ro.status != OPTIMAL:
            continue
        assert status == 0 and it <= 30
        ref = ro.x[9:].reshape(3, n, order="F").T.reshape(-1)
        assert np.max(np.abs(f - ref)) / max(1.0, np.max(np.abs(ref))) < 1e-5


@pytest.mark.parametrize("n", [3, 6])
def test_reduced_dd_qp_matches_oracle(n):
    from distributed_aerial_transportation_amd.system import pack_state

    rng = np.random.default_rng(200 + n)
    p = osc.params(n)
    feq = om.equilibrium_forces(p)
    c = om.Consts.make(p, osc.col_radius(n), distributed=True)
    for t in range(12):
        s = _rand_state(rng, n)
        acc = (rng.uniform(-5, 5, 3), rng.uniform(-5, 5, 3))
        i = t % n
        cv = rng.normal(0, 1, 9)
        P, q, G, h, dims, A, b = om.build_qp("dd", p, c, s, acc, om.EnvRows.empty(c), i=i, f_eq=feq, c_fi=cv[:3],
                                             c_Fi=cv[3:6], c_Mi=cv[6:])
        ro = solve_qp(P, q, G, h, dims, A, b)
        x, status, it = hs.qp_dd(_prm(n), n, pack_state(s), np.concatenate(acc), np.zeros((0, 3)), np.zeros(0), i, cv)
        assert status == 0
        assert np.max(np.abs(x - ro.x[9:])) / max(1.0, np.max(np.abs(ro.x[9:]))) < 1e-5


@pytest.mark.parametrize("n", [3, 6])
def test_reduced_centralized_qp_matches_oracle(n):
    from distributed_aerial_transportation_amd.system import pack_state

    rng = np.random.default_rng(300 + n)
    p = osc.params(n)
    feq = om.equilibrium_forces(p)
    c = om.Consts.make(p, osc.col_radius(n), distributed=False)
    for _ in range(8):
        s = _rand_state(rng, n)
        acc = (rng.uniform(-5, 5, 3), rng.uniform(-5, 5, 3))
        P, q, G, h, dims, A, b = om.build_qp("centralized", p, c, s, acc, om.EnvRows.empty(c), f_eq=feq)
        ro = solve_qp(P, q, G, h, dims, A, b)
        f, status, it = hs.qp_cent(_prm(n), n, pack_state(s), np.concatenate(acc), np.zeros((0, 3)), np.zeros(0))
        assert status == 0
        ref = ro.x[9:].reshape(3, n, order="F").T.reshape(-1)
        assert np.max(np.abs(f - ref)) / max(1.0, np.max(np.abs(ref))) < 1e-5


def test_env_rows_match_reference_fixture():
    from distributed_aerial_transportation_amd.system import pack_state

    d = load("ref_env_rows.npz")
    prm = _prm(3)
    for k in range(d["lhs_d"].shape[0]):
        st = pack_state(state_from(d, "s_", k))
        for agent, alpha in [(0, 1.5), (1, 1.5), (2, 1.5), (-1, 2.0)]:
            lhs, rhs, col, md = hs.env_rows(prm, 3, st, d["tree_pos"], agent, alpha)
            L = d["lhs_c"][k] if agent < 0 else d["lhs_d"][k, agent]
            R = d["rhs_c"][k] if agent < 0 else d["rhs_d"][k, agent]
            keep = np.any(np.abs(L) > 1e-12, axis=1) | (R > 0)
            keep2 = np.any(np.abs(lhs) > 1e-12, axis=1) | (rhs > 0)
            exp = np.array(sorted(map(tuple, np.column_stack([L[keep], R[keep]])))).reshape(-1, 4)
            got = np.array(sorted(map(tuple, np.column_stack([lhs[keep2], rhs[keep2]])))).reshape(-1, 4)
            assert got.shape == exp.shape
            np.testing.assert_allclose(got, exp, atol=1e-9)
            assert col == bool(d["col_c"][k] if agent < 0 else d["col_d"][k, agent])
            assert md == pytest.approx(float(d["md_c"][k] if agent < 0 else d["md_d"][k, agent]), abs=1e-8)


def test_rollout_matches_oracle_dynamics():
    from distributed_aerial_transportation_amd.system import RQPState, pack_state

    rng = np.random.default_rng(7)
    for n in (3, 6):
        p = osc.params(n)
        prm = _prm(n)
        s = _rand_state(rng, n)
        so = s.copy()
        x, cnt = pack_state(s), 0
        for _ in range(45):
            fdes = np.vstack([rng.uniform(-1, 1, (2, n)), rng.uniform(2, 6, (1, n))])
            f, M = om.low_level_control(p, so, fdes)
            so.integrate(*om.forward_dynamics(p, so, f, M), 5e-3)
            x, cnt = hs.sim_step(prm, n, x, cnt, fdes.T.reshape(-1), 5e-3)
        s1 = RQPState.unpack(x, n)
        for a in ("R", "w", "xl", "vl", "Rl", "wl"):
            np.testing.assert_allclose(getattr(s1, a), getattr(so, a), atol=1e-12)
        assert cnt == so.counter


@pytest.mark.parametrize("kind,name", [(0, "ref_lowlevel.npz"), (1, "ref_lowlevel_sm.npz")])
def test_low_level_law_matches_reference_fixture(kind, name):
    """ll_control_agent ("pd" / "sm", incl. the swapped T(e_R, r) of utils/so3_tracking_controllers.py:92)
    against RQPLowLevelController.control of the reference (control/rqp_centralized.py:518-535)."""
    d = load(name)
    p = osc.params(3)
    for k in range(d["f"].shape[0]):
        for i in range(3):
            R = d["s_R"][k][:, :, i]
            f, M = hs.ll_control(R.reshape(-1), d["s_w"][k][:, i], p.J[:, :, i].reshape(-1), d["f_des"][k][:, i], kind)
            assert f == pytest.approx(d["f"][k][i], rel=1e-13, abs=1e-13)
            np.testing.assert_allclose(M, d["M"][k][:, i], rtol=1e-11, atol=1e-13)


def test_sm_closed_loop_matches_reference():
    """400 ms of the reference loop with the "sm" law (centralized HL from the fixture's f_des):
    the host build of sim_step tracks the reference's states within 1e-9."""
    from distributed_aerial_transportation_amd.system import pack_state

    from tests._golden import unpack_flat

    d = load("ref_closed_loop_sm.npz")
    prm = _prm(3)
    p, _, s0 = __import__("distributed_aerial_transportation_amd").scenarios.rqp_setup(3)
    x, cnt = pack_state(s0), 0
    for i in range(d["states"].shape[0]):
        fd = d["f_des"][i // 10]
        x, cnt = hs.sim_step(prm, 3, x, cnt, fd.T.reshape(-1), 1e-3, kind=1)
        if i % 50 == 49:
            ref = pack_state(unpack_flat(d["states"][i], 3))
            assert np.max(np.abs(x - ref)) < 1e-9, i


def test_c4_stall_stretch_matches_oracle():
    """The C4 stall stretches of ref_c4_hard.npz (tests/golden/make_c4_hard.py, n = 6 in seeded forests,
    101-pass ADMM stalls from the second step on) with every agent QP answered by the host build of the
    device solver as the GPU's C-ADMM step runs it (IPM_FAST_REDO: the fast solver, redone robustly when
    not clean; rows certified infeasible held; the tail rule's warm start and stall exit from the second
    pass of every wedged step): ADMM iteration counts exact and f_des within max(1e-5, 5 x the oracle's own
    sensitivity) at every step (or the reference's own spread at Clarabel's 1e-8, f_des_1e8), no accept
    beyond Clarabel's 1e-8.  The first 12 steps of both stretches (the GPU test runs all 20)."""
    from distributed_aerial_transportation_amd import scenarios
    from distributed_aerial_transportation_amd.system import RQPState, pack_state
    from oracle import controllers as oc
    from oracle import forest as of

    d = load("ref_c4_hard.npz")
    n, K = 6, 12
    p = osc.params(n)
    prm = scenarios.params_block(n)
    for j in range(d["x0"].shape[0]):
        np.random.seed(int(d["forest_seed"][j]))
        forest = of.Forest()
        s0 = RQPState.unpack(d["x0"][j], n)
        st = om.State(s0.R, s0.w, s0.xl, s0.vl, s0.Rl, s0.wl, project=False)
        ctl = oc.CADMM(p, osc.col_radius(n), forest)
        tally = {"pass": 0, "tuned": 1, "loose": 0, "prev": 0, "tail": False, "unclean": False}
        wrec = np.zeros((n, hs.WREC_SIZE))

        def solve(self, i, s_, acc, env, rho):
            lam = self.lam[:, :, i].T.reshape(-1).copy()
            fbar = self.f_mean.T.reshape(-1).copy()
            ps = tally["pass"]
            tuned = tally["tuned"] if ps == 0 else 0
            # the tail rule (dat_qp.hpp TAIL_PREV / TAIL_PASS): warm start + stall exit in the passes it names;
            # the passes the tail kernel runs keep the warm-start records
            wson = ps >= 1 and (tally["prev"] > TAIL_PREV or ps >= TAIL_PASS)
            tally["tail"] = tally["tail"] or ps >= TAIL_PASS
            rec = np.ascontiguousarray(wrec[i]) if tally["tail"] else np.zeros(hs.WREC_SIZE)
            f, status, _, inb = hs.qp_cadmm_warm(prm, n, pack_state(s_), np.concatenate(acc), env.lhs, env.rhs, i, lam,
                                                 fbar, rho, rec, wson=wson, tuned=tuned)
            if tally["tail"]:
                wrec[i] = rec
            tally["loose"] += bool(inb) and hs.last_diag()[0] > 1e-8
            tally["unclean"] = tally["unclean"] or bool(hs.last_stiff())
            if status == 0:
                self.prev_f[i] = f.reshape(n, 3).T.copy()
            if i == n - 1:
                tally["pass"] += 1
                tally["tail"] = tally["tail"] or tally["unclean"]
            return self.prev_f[i], None

        ctl.solve_agent = solve.__get__(ctl)
        prev = 0
        for k in range(K):
            tally["pass"], tally["tuned"], tally["prev"] = 0, 1 if prev <= 3 else 0, prev
            tally["tail"], tally["unclean"] = prev > TAIL_PREV, False
            wrec[:] = 0.0
            acc, _, _ = oc.desired_acceleration_forest(st, forest)
            f, stat = ctl.control(st, acc)
            prev = stat.iter
            assert stat.iter == d["iters"][j, k], (j, k)
            ref = d["f_des"][j, k]
            scale = max(1.0, np.max(np.abs(ref)))
            sens = np.max(np.abs(d["f_des_1e10"][j, k] - ref)) / scale
            sens8 = np.max(np.abs(d["f_des_1e8"][j, k] - ref)) / scale  # the reference at Clarabel's 1e-8
            assert np.max(np.abs(f - ref)) / scale < max(1e-5, 5.0 * sens, sens8), (j, k)
            for _ in range(10):
                fl, M = om.low_level_control(p, st, f)
                st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
        assert tally["loose"] == 0, j


def _loose_bound(d, k, x):
    """f within max(1e-5, 5 x the oracle's own 1e-8-vs-1e-11 spread) of the oracle's 1e-11 answer, relative"""
    ref = d["x"][k]
    sc = max(1.0, np.max(np.abs(ref)))
    spread = np.max(np.abs(d["x_1e8"][k] - ref)) / sc
    return np.max(np.abs(x - ref)) / sc, max(1e-5, 5.0 * spread)


def test_loose_caps_solved_within_clarabel_tol():
    """The 20 agent QPs the GPU's 10 s C4 loop accepted in band beyond Clarabel's 1e-8 before the robust solver's
    cone recovery (ref_loose_caps.npz, tests/golden/make_loose_caps.py): the host build of the agent QP
    (IPM_FAST_REDO) ends each one converged or in band within 1e-8, at the oracle's answer up to the oracle's own
    spread between tolerances 1e-8 and 1e-11."""
    from distributed_aerial_transportation_amd import Forest, scenarios
    from distributed_aerial_transportation_amd.system import RQPState
    from oracle import forest as of
    from tests.test_gpu_c4 import _oforest

    d = load("ref_loose_caps.npz")
    n = 6
    p = osc.params(n)
    c = om.Consts.make(p, osc.col_radius(n), distributed=True)
    prm = scenarios.params_block(n)
    for k in range(len(d["agent"])):
        i = int(d["agent"][k])
        s0 = RQPState.unpack(d["state"][k], n)
        s = om.State(s0.R, s0.w, s0.xl, s0.vl, s0.Rl, s0.wl, project=False)
        env = of.env_rows(_oforest(Forest.seeded(int(d["forest"][k]))), c, s, osc.col_radius(n), p.r[:, i])
        f, status, _, inb = hs.qp_cadmm_ex(prm, n, d["state"][k], d["acc"][k], env.lhs, env.rhs, i, d["lam"][k],
                                           d["fbar"][k], float(d["rho"][k]))
        assert status == 0, k
        assert not inb or hs.last_diag()[0] <= 1e-8, (k, hs.last_diag())
        rel, bound = _loose_bound(d, k, f.reshape(n, 3).T)
        assert rel < bound, (k, rel, bound)
