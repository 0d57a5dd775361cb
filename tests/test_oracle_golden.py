"""Pin the oracle against golden vectors produced by the reference's own code (make_golden.py).

CPU-only; no GPU and no reference checkout are needed (fixtures are committed data).
"""

import numpy as np
import pytest

from oracle import controllers as oc
from oracle import forest as of
from oracle import model as om
from oracle import scenarios as osc
from oracle.ipm import ConeDims, OPTIMAL, solve_qp

from tests._golden import load, state_from, unpack_flat


def test_params_golden():
    d = load("ref_params.npz")
    p = osc.params(3)
    np.testing.assert_allclose(p.mT, d["mT"], rtol=0, atol=1e-15)
    np.testing.assert_allclose(p.x_com, d["x_com"], atol=1e-15)
    np.testing.assert_allclose(p.r_com, d["r_com"], atol=1e-15)
    np.testing.assert_allclose(p.JT, d["JT"], atol=1e-15)
    np.testing.assert_allclose(p.JT_inv, d["JT_inv"], rtol=1e-14)
    np.testing.assert_allclose(om.equilibrium_forces(p), d["f_eq"], rtol=1e-13, atol=1e-13)
    assert osc.col_radius(3) == pytest.approx(float(d["col_radius"]), abs=1e-15)
    c = om.Consts.make(p, osc.col_radius(3), distributed=True)
    assert c.min_fz == pytest.approx(float(d["min_fz"]), rel=1e-15)
    assert c.max_f == pytest.approx(float(d["max_f"]), rel=1e-15)
    assert c.vision_radius == pytest.approx(float(d["vision_radius"]), rel=1e-15)
    # SURVEY Appendix B golden numbers
    np.testing.assert_allclose(om.equilibrium_forces(p)[2], [5.644205448171, 5.642411548780, 5.629854253049], atol=1e-11)


@pytest.mark.parametrize("tag,n", [("n3", 3), ("n4", 4)])
def test_forward_dynamics_golden(tag, n):
    d = load("ref_dynamics.npz")
    p = om.Params(d[f"{tag}_m"], d[f"{tag}_J"], float(d[f"{tag}_ml"]), d[f"{tag}_Jl"], d[f"{tag}_r"])
    for k in range(d[f"{tag}_fd_f"].shape[0]):
        s = state_from(d, f"{tag}_fd_", k)
        dw, dvl, dwl = om.forward_dynamics(p, s, d[f"{tag}_fd_f"][k], d[f"{tag}_fd_M"][k])
        np.testing.assert_allclose(dw, d[f"{tag}_fd_dw"][k], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(dvl, d[f"{tag}_fd_dvl"][k], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(dwl, d[f"{tag}_fd_dwl"][k], rtol=1e-12, atol=1e-12)
        err = om.inverse_dynamics_error(s, p, d[f"{tag}_fd_f"][k], d[f"{tag}_fd_M"][k], dw, dvl, dwl)
        assert err < 1e-12 and d[f"{tag}_fd_err"][k] < 1e-12


@pytest.mark.parametrize("tag,n", [("n3", 3), ("n4", 4)])
def test_integrate_golden(tag, n):
    d = load("ref_dynamics.npz")
    p = om.Params(d[f"{tag}_m"], d[f"{tag}_J"], float(d[f"{tag}_ml"]), d[f"{tag}_Jl"], d[f"{tag}_r"])
    s = unpack_flat(d[f"{tag}_int_s0"], n)
    for f, M in zip(d[f"{tag}_int_f"], d[f"{tag}_int_M"]):
        s.integrate(*om.forward_dynamics(p, s, f, M), 5e-3)
    s1 = unpack_flat(d[f"{tag}_int_s1"], n)
    for a in ("R", "w", "xl", "vl", "Rl", "wl"):
        np.testing.assert_allclose(getattr(s, a), getattr(s1, a), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("kind,name", [("pd", "ref_lowlevel.npz"), ("sm", "ref_lowlevel_sm.npz")])
def test_lowlevel_golden(kind, name):
    """RQPLowLevelController("pd" / "sm").control (control/rqp_centralized.py:518-535); "sm" includes the
    swapped T(e_R, r) call of utils/so3_tracking_controllers.py:92."""
    d = load(name)
    p = osc.params(3)
    for k in range(d["f"].shape[0]):
        s = state_from(d, "s_", k)
        f, M = om.low_level_control(p, s, d["f_des"][k], kind)
        np.testing.assert_allclose(f, d["f"][k], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(M, d["M"][k], rtol=1e-12, atol=1e-13)


def test_forest_golden():
    d = load("ref_forest.npz")
    for seed in range(4):
        np.random.seed(seed)
        f = of.Forest()
        np.testing.assert_array_equal(f.tree_pos, d[f"tree_pos_{seed}"])
    assert d["tree_pos_0"].shape[0] == 128  # seed 0 gives 128 trees


def test_env_rows_golden():
    """Selection logic, row formulas and padding of the env CBF rows (geometry: oracle on both sides)."""
    d = load("ref_env_rows.npz")
    p = osc.params(3)
    forest = of.Forest.__new__(of.Forest)
    forest.tree_pos = d["tree_pos"]
    forest.num_trees = forest.tree_pos.shape[0]
    cd = om.Consts.make(p, osc.col_radius(3), distributed=True)
    cc = om.Consts.make(p, osc.col_radius(3), distributed=False)
    nonzero = 0
    for k in range(d["lhs_d"].shape[0]):
        s = state_from(d, "s_", k)
        for i in range(3):
            r = of.env_rows(forest, cd, s, osc.col_radius(3), p.r[:, i])
            # row order inside the 10 slots may differ (argpartition vs sort): compare as sets
            got = sorted(map(tuple, np.column_stack([r.lhs, r.rhs]).round(10)))
            exp = sorted(map(tuple, np.column_stack([d["lhs_d"][k, i], d["rhs_d"][k, i]]).round(10)))
            np.testing.assert_allclose(got, exp, atol=1e-9)
            assert r.collision == bool(d["col_d"][k, i])
            assert r.min_env_dist == pytest.approx(float(d["md_d"][k, i]), abs=1e-12)
            nonzero += int(np.any(r.lhs != 0))
        r = of.env_rows(forest, cc, s, osc.col_radius(3), None)
        got = sorted(map(tuple, np.column_stack([r.lhs, r.rhs]).round(10)))
        exp = sorted(map(tuple, np.column_stack([d["lhs_c"][k], d["rhs_c"][k]]).round(10)))
        np.testing.assert_allclose(got, exp, atol=1e-9)
        assert r.collision == bool(d["col_c"][k])
    assert nonzero > 10  # the fixture exercises real obstacle rows


def _drop_zero_rows(G, h, l):
    keep = np.ones(G.shape[0], bool)
    keep[:l] = np.any(G[:l] != 0, axis=1) | (h[:l] != 0)
    return G[keep], h[keep], int(keep[:l].sum())


@pytest.mark.parametrize("case", range(6))
@pytest.mark.parametrize("kind", ["cadmm", "dd", "cen"])
def test_qp_formulation_golden(kind, case):
    """The oracle's uncondensed QP equals the problem the reference's cvxpy model produces."""
    d = load("ref_qp.npz")
    pre = f"{kind}{case}_"
    p = osc.params(3)
    s = state_from(d, pre + "s_")
    acc = (d[pre + "acc"][:3], d[pre + "acc"][3:])
    feq = om.equilibrium_forces(p)
    if kind == "cen":
        c = om.Consts.make(p, osc.col_radius(3), distributed=False)
        P, q, G, h, dims, A, b = om.build_qp("centralized", p, c, s, acc, om.EnvRows.empty(c), f_eq=feq)
    elif kind == "cadmm":
        c = om.Consts.make(p, osc.col_radius(3), distributed=True)
        P, q, G, h, dims, A, b = om.build_qp("cadmm", p, c, s, acc, om.EnvRows.empty(c), i=int(d[pre + "i"]),
                                             f_eq=feq, lam=d[pre + "lam"], rho=1.0, f_mean=d[pre + "fm"])
    else:
        c = om.Consts.make(p, osc.col_radius(3), distributed=True)
        cc = d[pre + "c"]
        P, q, G, h, dims, A, b = om.build_qp("dd", p, c, s, acc, om.EnvRows.empty(c), i=int(d[pre + "i"]),
                                             f_eq=feq, c_fi=cc[:3], c_Fi=cc[3:6], c_Mi=cc[6:])
    np.testing.assert_allclose(P, d[pre + "P"], atol=1e-12)
    np.testing.assert_allclose(q, d[pre + "q"], atol=1e-12)
    Gr, hr, lr = _drop_zero_rows(d[pre + "G"], d[pre + "h"], int(d[pre + "l"]))
    dims_r = ConeDims(l=lr, q=list(d[pre + "q_dims"]))
    # identical feasible sets => identical (unique) minimisers
    r1 = solve_qp(P, q, G, h, dims, A, b)
    r2 = solve_qp(d[pre + "P"], d[pre + "q"], Gr, hr, dims_r, d[pre + "A"], d[pre + "b"])
    assert r1.status == OPTIMAL and r2.status == OPTIMAL
    np.testing.assert_allclose(r1.x, r2.x, atol=1e-8)
    np.testing.assert_allclose(r1.x, d[pre + "x"], atol=1e-8)
    # and the SOC blocks are the same cones (rows compared as sets)
    assert sorted(dims.q) == sorted(dims_r.q)


@pytest.mark.parametrize("name", ["cadmm", "dd"])
def test_outer_loop_fixed_iterations_golden(name):
    """_plot_convergence_rate recipe: tol 0, max_iter 25 (test/control/test_rqpcontrollers.py:101-124)."""
    d = load(f"ref_{name}.npz")
    p = osc.params(3)
    s = osc.rest_state(3)
    ctl = oc.CADMM(p, osc.col_radius(3)) if name == "cadmm" else oc.DD(p, osc.col_radius(3))
    if name == "cadmm":
        ctl.set_force_err_tolerance(0.0, False)
    else:
        ctl.set_force_err_tolerance(0.0)
    ctl.set_max_iter(25)
    for k in range(d["fixed_err"].shape[0]):
        a = d["acc"][k]
        f, st = ctl.control(s, (a[:3], a[3:]))
        np.testing.assert_allclose(st.err_seq, d["fixed_err"][k], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(f, d["fixed_f"][k], rtol=1e-7, atol=1e-8)


@pytest.mark.parametrize("name", ["cadmm", "dd"])
def test_outer_loop_default_tolerance_golden(name):
    d = load(f"ref_{name}.npz")
    p = osc.params(3)
    s = osc.rest_state(3)
    ctl = oc.CADMM(p, osc.col_radius(3)) if name == "cadmm" else oc.DD(p, osc.col_radius(3))
    for k in range(d["tol_iters"].shape[0]):
        a = d["acc"][k]
        f, st = ctl.control(s, (a[:3], a[3:]))
        assert st.iter == d["tol_iters"][k]
        np.testing.assert_allclose(f, d["tol_f"][k], rtol=1e-7, atol=1e-8)


def test_centralized_golden():
    d = load("ref_central.npz")
    p = osc.params(3)
    ctl = oc.Centralized(p, osc.col_radius(3))
    for k in range(d["f"].shape[0]):
        a = d["acc"][k]
        f, _ = ctl.control(osc.rest_state(3), (a[:3], a[3:]))
        np.testing.assert_allclose(f, d["f"][k], rtol=1e-8, atol=1e-9)


def test_c4_closed_loop_golden():
    """The oracle's C-ADMM + forest + dynamics reproduce the reference's n = 6 C4 closed loop
    (ref_c4_loop.npz: control/rqp_cadmm.py:631-675 in example/rqp_example.py:120-131, seeded forests,
    near-tree starts) over its first HL steps: f_des, ADMM iteration counts, min env distance, states."""
    d = load("ref_c4_loop.npz")
    n = 6
    p = osc.params(n)
    for s, steps in ((0, 6), (2, 4)):
        np.random.seed(int(d["seeds"][s]))
        forest = of.Forest()
        ctl = oc.CADMM(p, osc.col_radius(n), forest)
        st = unpack_flat(d[f"s{s}_states"][0], n)
        for k in range(steps):
            np.testing.assert_allclose(np.concatenate([st.R.reshape(-1), st.w.reshape(-1), st.xl, st.vl,
                                                       st.Rl.reshape(-1), st.wl]), d[f"s{s}_states"][k], atol=1e-9)
            acc, _, _ = oc.desired_acceleration_forest(st, forest)
            f, stat = ctl.control(st, acc)
            assert stat.iter == d[f"s{s}_iters"][k], (s, k)
            np.testing.assert_allclose(f, d[f"s{s}_f_des"][k], rtol=1e-7, atol=1e-7)
            assert stat.min_env_dist == pytest.approx(float(d[f"s{s}_min_dist"][k]), abs=1e-8)
            for _ in range(10):
                fl, M = om.low_level_control(p, st, f)
                st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
