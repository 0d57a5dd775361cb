"""Generate golden fixtures from the reference's OWN Python code (run in the dev container only).

    python -O tests/golden/make_golden.py   # -O = PYTHONOPTIMIZE, required by the reference (README.md:28)

The reference is imported from /root/reference behind the stubs in ``refstubs.py`` (cvxpy
tracing layer answered by the oracle IPM, closed-form pinocchio, oracle geometry for hppfcl,
inert meshcat/polytope).  Everything written here is *data*: inputs and the reference code's
outputs, as small .npz files next to this script.  Nothing of the reference's source travels.

What each fixture pins (reference file:line):
  ref_params.npz      RQPParameters + f_eq + controller constants   system/rigid_quadrotor_payload.py:48-84,
                                                                    control/rqp_cadmm.py:142-236
  ref_dynamics.npz    forward_dynamics, inverse_dynamics_error, RQPState.integrate/project_R
                                                                    system/rigid_quadrotor_payload.py:121-269
  ref_lowlevel.npz    RQPLowLevelController("pd").control          control/rqp_centralized.py:457-535
  ref_forest.npz      Forest() tree layouts for np.random.seed(0..3) example/env_forest.py:47-85
  ref_env_rows.npz    _set_collision_avoidance_cbf_parameters       control/rqp_cadmm.py:307-373,
                                                                    control/rqp_centralized.py:280-337
  ref_qp.npz          the conic problem data cvxpy would receive    control/rqp_*.py constraint/cost builders
  ref_cadmm.npz       RQPCADMMController.control sequences          control/rqp_cadmm.py:631-675
  ref_dd.npz          RQPDDController.control sequences             control/rqp_dd.py:695-752
  ref_central.npz     RQPCentralizedController.control              control/rqp_centralized.py:436-448
  ref_closed_loop.npz rqp_example-style closed loop (HL every 10)   example/rqp_example.py:120-131
  ref_lowlevel_sm.npz RQPLowLevelController("sm").control          utils/so3_tracking_controllers.py:52-95
  ref_closed_loop_sm.npz  400 ms centralized loop with the "sm" law  control/rqp_centralized.py:474-478
  ref_rp.npz          RPCentralizedController + RPDynamics closed loop control/rp_centralized.py:9-302,
                      (test/control/test_rpcentralized.py:main, 20 s)  system/rigid_payload.py:93-130
  ref_c4_loop.npz     the C4 closed loop: n = 6 C-ADMM in seeded forests, 400 HL steps from near-tree starts
                      (python -O make_golden.py c4)               control/rqp_cadmm.py:631-675,
                                                                  example/rqp_example.py:120-131
  ref_long_<tag>.npz  rqp_example over the reference horizon (100 s): f_des, iters, min_dist per HL
                      step, x_err / v_err per log step, states + LL wrench every 10th log step
                      (python -O make_golden.py long <controller_type>)
"""

from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import refstubs  # noqa: E402

refstubs.install()
sys.path.insert(0, REF)

from control.rqp_cadmm import RQPCADMMController  # noqa: E402
from control.rqp_centralized import RQPCentralizedController, RQPLowLevelController  # noqa: E402
from control.rqp_dd import RQPDDController  # noqa: E402
from example.env_forest import Forest  # noqa: E402
from example.setup import rqp_setup  # noqa: E402
from system.rigid_quadrotor_payload import RQPDynamics, RQPParameters, RQPState  # noqa: E402

from oracle.model import exp3  # noqa: E402

OUT = HERE


def rand_rot(rng, scale):
    return exp3(rng.uniform(-scale, scale, 3))


def rand_state(rng, n, big=False):
    R = np.stack([rand_rot(rng, 0.3 if not big else 1.0) for _ in range(n)], axis=2)
    w = rng.uniform(-0.5, 0.5, (3, n))
    xl = rng.uniform(-1, 1, 3)
    vl = rng.uniform(-0.5, 0.5, 3)
    Rl = rand_rot(rng, 0.1 if not big else 0.5)
    wl = rng.uniform(-0.2, 0.2, 3)
    return RQPState(R, w, xl, vl, Rl, wl)


def pack_state(s):
    return dict(R=s.R.copy(), w=s.w.copy(), xl=s.xl.copy(), vl=s.vl.copy(), Rl=s.Rl.copy(), wl=s.wl.copy())


def stack_states(states):
    return {k: np.stack([st[k] for st in states]) for k in states[0]}


def gen_params():
    p, col, s0 = rqp_setup(3)
    ctrl = RQPCADMMController(p, col, s0, 1e-3)
    ps = ctrl.primal_solvers[0]
    np.savez(os.path.join(OUT, "ref_params.npz"), mT=p.mT, x_com=p.x_com, r_com=p.r_com, JT=p.JT,
             JT_inv=p.JT_inv, f_eq=ps.f_eq, col_radius=col.collision_radius,
             max_deceleration=col.max_deceleration, min_fz=ps.min_fz, max_f=ps.max_f,
             vision_radius=ps.vision_radius, sec_max_f_ang=ps.sec_max_f_ang)


def gen_dynamics():
    rng = np.random.default_rng(7)
    out = {}
    for n, tag in ((3, "n3"), (4, "n4")):
        if n == 3:
            p, _, _ = rqp_setup(3)
        else:
            r = rng.uniform(-1, 1, (3, n))
            J = np.stack([np.diag([2.32, 2.32, 4]) * 1e-3] * n, axis=2)
            p = RQPParameters(np.full(n, 0.5), J, 0.225, np.diag([2.1, 1.87, 3.97]) * 1e-2, r)
        states, wr_f, wr_M, dws, dvls, dwls, errs = [], [], [], [], [], [], []
        for _ in range(16):
            s = rand_state(rng, n, big=True)
            f = rng.random(n) * p.mT * 9.80665 / n
            M = rng.random((3, n)) - 0.5
            dyn = RQPDynamics(p, s, 1e-3)
            dw, dvl, dwl = dyn.forward_dynamics((f, M))
            states.append(pack_state(s))
            wr_f.append(f), wr_M.append(M), dws.append(dw), dvls.append(dvl), dwls.append(dwl)
            errs.append(RQPDynamics.inverse_dynamics_error(s, p, (f, M), (dw, dvl, dwl)))
        st = stack_states(states)
        for k, v in st.items():
            out[f"{tag}_fd_{k}"] = v
        out[f"{tag}_fd_f"], out[f"{tag}_fd_M"] = np.array(wr_f), np.array(wr_M)
        out[f"{tag}_fd_dw"], out[f"{tag}_fd_dvl"], out[f"{tag}_fd_dwl"] = np.array(dws), np.array(dvls), np.array(dwls)
        out[f"{tag}_fd_err"] = np.array(errs)
        out[f"{tag}_r"], out[f"{tag}_m"], out[f"{tag}_J"] = p.r, p.m, p.J
        out[f"{tag}_ml"], out[f"{tag}_Jl"] = p.ml, p.Jl
        # integration: 45 steps of dt = 5e-3 with random wrenches (crosses two projections)
        s = rand_state(rng, n, big=True)
        out[f"{tag}_int_s0"] = np.concatenate([s.R.reshape(-1), s.w.reshape(-1), s.xl, s.vl, s.Rl.reshape(-1), s.wl])
        dyn = RQPDynamics(p, s, 5e-3)
        fs, Ms = [], []
        for _ in range(45):
            f = rng.random(n) * p.mT * 9.80665 / n
            M = (rng.random((3, n)) - 0.5) * 0.01
            fs.append(f), Ms.append(M)
            dyn.integrate((f, M))
        out[f"{tag}_int_f"], out[f"{tag}_int_M"] = np.array(fs), np.array(Ms)
        s = dyn.state
        out[f"{tag}_int_s1"] = np.concatenate([s.R.reshape(-1), s.w.reshape(-1), s.xl, s.vl, s.Rl.reshape(-1), s.wl])
    np.savez(os.path.join(OUT, "ref_dynamics.npz"), **out)


def gen_lowlevel(kind="pd", name="ref_lowlevel.npz"):
    rng = np.random.default_rng(11)
    p, _, _ = rqp_setup(3)
    ll = RQPLowLevelController(kind, p, np.pi / 6)
    states, fdes, fs, Ms = [], [], [], []
    for _ in range(16):
        s = rand_state(rng, 3, big=True)
        fd = np.vstack([rng.uniform(-2, 2, (2, 3)), rng.uniform(3, 8, (1, 3))])
        f, M = ll.control(s, fd)
        states.append(pack_state(s)), fdes.append(fd), fs.append(f), Ms.append(M)
    np.savez(os.path.join(OUT, name), **{f"s_{k}": v for k, v in stack_states(states).items()},
             f_des=np.array(fdes), f=np.array(fs), M=np.array(Ms))


def gen_lowlevel_sm():
    """RQPLowLevelController("sm") (control/rqp_centralized.py:474-478, utils/so3_tracking_controllers.py:52-95)
    on the same states, plus a 400 ms rqp_example loop (centralized HL, forest seed 0) with the "sm" law."""
    gen_lowlevel("sm", "ref_lowlevel_sm.npz")
    np.random.seed(0)
    env = Forest()
    p, col, s0 = rqp_setup(3)
    dyn = RQPDynamics(p, s0, 1e-3)
    hl = RQPCentralizedController(p, col, s0, 1e-3, env)
    ll = RQPLowLevelController("sm", p, hl.get_force_cone_angle_bound())
    from example.rqp_example import _desired_acceleration_forest  # noqa: E402
    fdes, xs = [], []
    for i in range(400):
        if i % 10 == 0:
            acc, _, _ = _desired_acceleration_forest(dyn.state, i * 1e-3, env)
            f_des, _ = hl.control(dyn.state, acc)
            fdes.append(f_des.copy())
        dyn.integrate(ll.control(dyn.state, f_des))
        s = dyn.state
        xs.append(np.concatenate([s.R.reshape(-1), s.w.reshape(-1), s.xl, s.vl, s.Rl.reshape(-1), s.wl]))
    np.savez(os.path.join(OUT, "ref_closed_loop_sm.npz"), f_des=np.array(fdes), states=np.array(xs))


def gen_forest():
    out = {}
    for seed in range(4):
        np.random.seed(seed)
        env = Forest()
        out[f"tree_pos_{seed}"] = env.tree_pos
    out["mountain_sphere_radius"] = env.mountain_sphere_radius
    out["mountain_center_depth"] = env.mountain_center_depth
    np.savez(os.path.join(OUT, "ref_forest.npz"), **out)


def forest_state(rng, env, n):
    # payload heading through the forest: pick a tree and start 2-5 m in front of it
    k = rng.integers(env.num_trees)
    tp = env.tree_pos[k]
    ang = rng.uniform(-0.4, 0.4)
    dist = rng.uniform(1.6, 4.0)
    xl = np.array([tp[0] - dist * np.cos(ang), tp[1] - dist * np.sin(ang), tp[2] + rng.uniform(-1.5, 2.5)])
    vl = np.array([rng.uniform(0.2, 0.9), rng.uniform(-0.3, 0.3), rng.uniform(-0.1, 0.1)])
    R = np.stack([rand_rot(rng, 0.2) for _ in range(n)], axis=2)
    return RQPState(R, rng.uniform(-0.3, 0.3, (3, n)), xl, vl, rand_rot(rng, 0.1), rng.uniform(-0.1, 0.1, 3))


def gen_env_rows():
    np.random.seed(0)
    env = Forest()
    rng = np.random.default_rng(5)
    p, col, s0 = rqp_setup(3)
    cad = RQPCADMMController(p, col, s0, 1e-3, env)
    cen = RQPCentralizedController(p, col, s0, 1e-3, env)
    states, lhs_d, rhs_d, col_d, md_d, lhs_c, rhs_c, col_c, md_c = [], [], [], [], [], [], [], [], []
    for _ in range(24):
        s = forest_state(rng, env, 3)
        states.append(pack_state(s))
        L, Rr, C, Md = [], [], [], []
        for i in range(3):
            ps = cad.primal_solvers[i]
            ps._set_collision_avoidance_cbf_parameters(s)
            L.append(ps.env_cbf_lhs.value.copy()), Rr.append(ps.env_cbf_rhs.value.copy())
            C.append(ps.collision), Md.append(ps.min_env_dist)
        lhs_d.append(L), rhs_d.append(Rr), col_d.append(C), md_d.append(Md)
        cen._set_collision_avoidance_cbf_parameters(s)
        lhs_c.append(cen.env_cbf_lhs.value.copy()), rhs_c.append(cen.env_cbf_rhs.value.copy())
        col_c.append(cen.collision), md_c.append(cen.min_env_dist)
    np.savez(os.path.join(OUT, "ref_env_rows.npz"), **{f"s_{k}": v for k, v in stack_states(states).items()},
             tree_pos=env.tree_pos, lhs_d=np.array(lhs_d), rhs_d=np.array(rhs_d), col_d=np.array(col_d),
             md_d=np.array(md_d), lhs_c=np.array(lhs_c), rhs_c=np.array(rhs_c), col_c=np.array(col_c),
             md_c=np.array(md_c))


def gen_qp():
    """Trace the exact problems the reference builds (no env; env rows are pinned separately)."""
    rng = np.random.default_rng(3)
    p, col, s0 = rqp_setup(3)
    out = {}
    cad = RQPCADMMController(p, col, s0, 1e-3)
    dd = RQPDDController(p, col, s0, 1e-3)
    cen = RQPCentralizedController(p, col, s0, 1e-3)
    for case in range(6):
        s = rand_state(rng, 3)
        acc = (rng.uniform(-2, 2, 3), rng.uniform(-2, 2, 3))
        i = case % 3
        lam = rng.normal(0, 0.5, (3, 3))
        fm = rng.normal(0, 2, (3, 3)) + cad.primal_solvers[0].f_eq
        refstubs.TRACE.clear()
        cad.primal_solvers[i].solve(s, acc, lam, 1.0, fm)
        t = refstubs.TRACE[-1]
        pre = f"cadmm{case}_"
        for k in ("P", "q", "A", "b", "G", "h", "l", "q_dims", "x"):
            out[pre + k] = t[k]
        out[pre + "i"], out[pre + "lam"], out[pre + "fm"] = i, lam, fm
        out[pre + "acc"] = np.concatenate(acc)
        for k, v in pack_state(s).items():
            out[pre + "s_" + k] = v
        cf, cF, cM = rng.normal(0, 1, 3), rng.normal(0, 1, 3), rng.normal(0, 0.3, 3)
        refstubs.TRACE.clear()
        dd.primal_solvers[i].solve(s, acc, cf, cF, cM)
        t = refstubs.TRACE[-1]
        pre = f"dd{case}_"
        for k in ("P", "q", "A", "b", "G", "h", "l", "q_dims", "x"):
            out[pre + k] = t[k]
        out[pre + "i"], out[pre + "c"] = i, np.concatenate([cf, cF, cM])
        out[pre + "acc"] = np.concatenate(acc)
        for k, v in pack_state(s).items():
            out[pre + "s_" + k] = v
        refstubs.TRACE.clear()
        cen.control(s, acc)
        t = refstubs.TRACE[-1]
        pre = f"cen{case}_"
        for k in ("P", "q", "A", "b", "G", "h", "l", "q_dims", "x"):
            out[pre + k] = t[k]
        out[pre + "acc"] = np.concatenate(acc)
        for k, v in pack_state(s).items():
            out[pre + "s_" + k] = v
    np.savez(os.path.join(OUT, "ref_qp.npz"), **out)


def gen_outer_loops():
    """_plot_convergence_rate recipe (test/control/test_rqpcontrollers.py:101-124) + default tolerance."""
    p, col, s0 = rqp_setup(3)
    np.random.seed(0)
    accs = [((np.random.random(3) - 0.5) * 10.0, (np.random.random(3) - 0.5) * 10.0) for _ in range(6)]
    for name, cls in (("cadmm", RQPCADMMController), ("dd", RQPDDController)):
        out = {"acc": np.array([np.concatenate(a) for a in accs])}
        c = cls(p, col, s0, 1e-3)
        if name == "cadmm":
            c.set_force_err_tolerance(0.0, False)
        else:
            c.set_force_err_tolerance(0.0)
        c.set_max_iter(25)
        errs, fs = [], []
        for a in accs[:3]:
            f, st = c.control(s0, a)
            errs.append(st.err_seq), fs.append(f.copy())
        out["fixed_err"], out["fixed_f"] = np.array(errs), np.array(fs)
        c = cls(p, col, s0, 1e-3)
        its, fs, errs = [], [], []
        for a in accs:
            f, st = c.control(s0, a)
            its.append(st.iter), fs.append(f.copy()), errs.append(np.pad(np.array(st.err_seq, float), (0, 101 - len(st.err_seq)), constant_values=np.nan))
        out["tol_iters"], out["tol_f"], out["tol_err"] = np.array(its), np.array(fs), np.array(errs)
        np.savez(os.path.join(OUT, f"ref_{name}.npz"), **out)
    c = RQPCentralizedController(p, col, s0, 1e-3)
    fs = [c.control(s0, a)[0].copy() for a in accs]
    np.savez(os.path.join(OUT, "ref_central.npz"), acc=np.array([np.concatenate(a) for a in accs]), f=np.array(fs))


def gen_closed_loop(steps=400):
    """rqp_example main loop (example/rqp_example.py:120-131): forest seed 0, HL every 10 steps."""
    out = {}
    for name in ("consensus-admm", "dual-decomposition", "centralized"):
        np.random.seed(0)
        env = Forest()
        p, col, s0 = rqp_setup(3)
        dyn = RQPDynamics(p, s0, 1e-3)
        cls = {"consensus-admm": RQPCADMMController, "dual-decomposition": RQPDDController,
               "centralized": RQPCentralizedController}[name]
        hl = cls(p, col, s0, 1e-3, env)
        ll = RQPLowLevelController("pd", p, hl.get_force_cone_angle_bound())
        from example.rqp_example import _desired_acceleration_forest  # noqa: E402 (matplotlib import)
        fdes, its, xs, mds = [], [], [], []
        for i in range(steps):
            if i % 10 == 0:
                acc, _, _ = _desired_acceleration_forest(dyn.state, i * 1e-3, env)
                f_des, st = hl.control(dyn.state, acc)
                fdes.append(f_des.copy()), its.append(st.iter), mds.append(st.min_env_dist)
            w = ll.control(dyn.state, f_des)
            dyn.integrate(w)
            s = dyn.state
            xs.append(np.concatenate([s.R.reshape(-1), s.w.reshape(-1), s.xl, s.vl, s.Rl.reshape(-1), s.wl]))
        tag = name.split("-")[0][:4]
        out[f"{tag}_f_des"], out[f"{tag}_iters"] = np.array(fdes), np.array(its)
        out[f"{tag}_states"], out[f"{tag}_min_dist"] = np.array(xs), np.array(mds)
    np.savez(os.path.join(OUT, "ref_closed_loop.npz"), **out)


def gen_rp():
    """RPCentralizedController (control/rp_centralized.py:9-302) and RPDynamics (system/rigid_payload.py:
    93-130): the closed loop of test/control/test_rpcentralized.py:main (n = 3, dt = 10e-3, circle tracking
    law :14-37) for 20 s -- f per step and the state after each step -- plus forward-dynamics cases at
    random states / forces."""
    sys.path.insert(0, os.path.join(REF, "test", "control"))
    from control.rp_centralized import RPCentralizedController
    from example.setup import rp_setup
    from system.rigid_payload import RPDynamics, RPState
    from test_rpcentralized import _desired_acceleration

    params, col, s0 = rp_setup(3)
    dt = 10e-3
    ctl = RPCentralizedController(params, col, s0, dt)
    dyn = RPDynamics(params, s0, dt)
    t_seq = np.arange(0, 20, dt)
    fs, xs, accs = [], [], []
    for i in range(len(t_seq)):
        acc_des, _, _ = _desired_acceleration(dyn.state, t_seq[i])
        f = ctl.control(dyn.state, acc_des)
        dyn.integrate(f)
        s = dyn.state
        fs.append(np.array(f).copy()), accs.append(np.concatenate(acc_des))
        xs.append(np.concatenate([s.xl, s.vl, s.Rl.reshape(-1), s.wl]))
    rng = np.random.default_rng(17)
    fd_s, fd_f, fd_acc = [], [], []
    for _ in range(16):
        s = RPState(rng.uniform(-1, 1, 3), rng.uniform(-1, 1, 3), rand_rot(rng, 0.5), rng.uniform(-1, 1, 3))
        f = np.vstack([rng.uniform(-1, 1, (2, 3)), rng.uniform(0, 2, (1, 3))])
        d = RPDynamics(params, s, dt)
        fd_s.append(np.concatenate([s.xl, s.vl, s.Rl.reshape(-1), s.wl])), fd_f.append(f)
        fd_acc.append(np.concatenate(d.forward_dynamics(f)))
    np.savez(os.path.join(OUT, "ref_rp.npz"), ml=params.ml, Jl=params.Jl, r=params.r, f_eq=ctl.f_eq, dt=dt,
             f=np.array(fs), states=np.array(xs), acc=np.array(accs), min_fz=ctl.min_fz, max_f=ctl.max_f,
             fd_s=np.array(fd_s), fd_f=np.array(fd_f), fd_acc=np.array(fd_acc))


LONG_T = {"centralized": 100.0, "consensus-admm": 100.0, "dual-decomposition": 100.0}


def gen_long_closed_loop(name, T=None, state_every=10):
    """rqp_example's main loop (example/rqp_example.py:85-131) over the reference horizon T = 100 s
    (example/rqp_example.py:92, every controller type): forest seed 0,
    n = 3, HL every 10 steps, LL "pd".  Recorded per HL step: f_des, iter, min_env_dist; per log step
    (i % log_freq == 0, after that step's integrate, :114-120): x_err, v_err; and every
    ``state_every``-th log step the state and the LL wrench w = (f (n), M (3, n)).  Written to
    ref_long_<tag>.npz (compressed)."""
    T = LONG_T[name] if T is None else T
    np.random.seed(0)
    env = Forest()
    p, col, s0 = rqp_setup(3)
    dt, hl = 1e-3, 10
    dyn = RQPDynamics(p, s0, dt)
    cls = {"consensus-admm": RQPCADMMController, "dual-decomposition": RQPDDController,
           "centralized": RQPCentralizedController}[name]
    ctl = cls(p, col, s0, dt, env)
    ll = RQPLowLevelController("pd", p, ctl.get_force_cone_angle_bound())
    from example.rqp_example import _desired_acceleration_forest  # noqa: E402 (matplotlib import)
    steps = int(round(T / dt))
    fdes, its, mds, xe, ve, xs, ws = [], [], [], [], [], [], []
    for i in range(steps):
        if i % hl == 0:
            acc, x_ref, v_ref = _desired_acceleration_forest(dyn.state, i * dt, env)
            f_des, st = ctl.control(dyn.state, acc)
            fdes.append(f_des.copy()), its.append(st.iter), mds.append(st.min_env_dist)
        w = ll.control(dyn.state, f_des)
        dyn.integrate(w)
        if i % hl == 0:
            s = dyn.state
            xe.append(np.linalg.norm(x_ref - s.xl)), ve.append(np.linalg.norm(v_ref - s.vl))
            if (i // hl) % state_every == 0:
                xs.append(np.concatenate([s.R.reshape(-1), s.w.reshape(-1), s.xl, s.vl, s.Rl.reshape(-1), s.wl]))
                ws.append(np.concatenate([np.asarray(w[0]).reshape(-1), np.asarray(w[1]).reshape(-1)]))
        if i % 10000 == 0:
            print(f"{name}: t = {i * dt:.0f} s", flush=True)
    tag = name.split("-")[0][:4]
    np.savez_compressed(os.path.join(OUT, f"ref_long_{tag}.npz"), T=T, dt=dt, hl_rel_freq=hl, state_every=state_every,
                        f_des=np.array(fdes), iters=np.array(its, dtype=np.int16), min_dist=np.array(mds),
                        x_err=np.array(xe), v_err=np.array(ve), states=np.array(xs), w=np.array(ws))


C4_SEEDS = (0, 1, 2, 3)   # forest seeds of the four C4 closed loops
C4_T = 4.0                # seconds (400 HL steps)


def _terrain_z(env, xy):
    """z of the desired-acceleration law's reference height (example/rqp_example.py:38-46) at xy."""
    nrm = np.linalg.norm(np.asarray(xy) - env.mountain_center)
    if nrm >= env.mountain_radius:
        return 1.5
    return np.sqrt(env.mountain_sphere_radius ** 2 - nrm ** 2) - env.mountain_center_depth + 1.5


def c4_start_state(env, n, rng):
    """Config C4 near-tree start: payload 1.6-2.8 m (xy) from the axis of a tree near the forest's
    y = 0 line (where the desired law steers), heading at it within +-0.3 rad at 0.5-1.0 m/s, at the
    reference height, rest attitude; positions closer than 1.5 m to any tree axis are redrawn."""
    inner = np.nonzero((env.tree_pos[:, 0] > 8.0) & (env.tree_pos[:, 0] < 50.0) & (np.abs(env.tree_pos[:, 1]) < 4.0))[0]
    while True:
        k = rng.choice(inner)
        th = rng.uniform(-0.3, 0.3)
        head = np.array([np.cos(th), np.sin(th)])
        xy = env.tree_pos[k, :2] - rng.uniform(1.6, 2.8) * head
        if np.min(np.linalg.norm(env.tree_pos[:, :2] - xy, axis=1)) >= 1.5:
            break
    sp = rng.uniform(0.5, 1.0)
    return RQPState(np.stack([np.eye(3)] * n, axis=2), np.zeros((3, n)), np.array([xy[0], xy[1], _terrain_z(env, xy)]),
                    np.array([sp * head[0], sp * head[1], 0.0]), np.eye(3), np.zeros(3))


def gen_c4_loop(T=C4_T, out_dir=None):
    """The headline configuration's closed loop over many HL steps: n = 6
    C-ADMM (hexagon team, oracle/scenarios.py geometry, reference RQPParameters / RQPCollision) in the
    seeded forests C4_SEEDS, rqp_example's loop (example/rqp_example.py:120-131: forest desired
    acceleration, RQPCADMMController.control control/rqp_cadmm.py:631-675, LL "pd", integrate; HL
    every 10 steps) from near-tree starts for T seconds.  Recorded per HL step: f_des, iter,
    min_env_dist, err_seq; the state at every HL instant (before its control call)."""
    from example.rqp_example import _desired_acceleration_forest  # noqa: E402 (matplotlib import)
    from oracle import scenarios as osc

    n, dt, hl = 6, 1e-3, 10
    m, J, ml, Jl, r = osc.geometry(n)
    p = RQPParameters(m, J, ml, Jl, r)
    R0 = np.linalg.norm(r, axis=0).max()
    from system.rigid_quadrotor_payload import RQPCollision

    # the build's n = 6 collision data (scenarios.collision: radius from the max mesh-vertex norm R0 +
    # 0.1, system/rigid_quadrotor_payload.py:302-306); the reference builds a hull of the mesh, so the
    # flat ring gets an inner, lower copy (norms < R0 + 0.1: the radius is unchanged)
    mesh = r.T * (R0 + 0.1) / R0
    col = RQPCollision(np.vstack([r.T, r.T - [0, 0, 0.1]]), np.vstack([mesh, 0.5 * mesh - [0, 0, 0.1]]))
    rng = np.random.default_rng(606)
    out = {"seeds": np.array(C4_SEEDS), "T": T, "dt": dt, "hl_rel_freq": hl}
    steps = int(round(T / dt))
    for k, seed in enumerate(C4_SEEDS):
        np.random.seed(seed)
        env = Forest()
        s0 = c4_start_state(env, n, rng)
        dyn = RQPDynamics(p, s0, dt)
        ctl = RQPCADMMController(p, col, s0, dt, env)
        ll = RQPLowLevelController("pd", p, ctl.get_force_cone_angle_bound())
        fdes, its, mds, xs, errs = [], [], [], [], []
        for i in range(steps):
            if i % hl == 0:
                s = dyn.state
                xs.append(np.concatenate([s.R.reshape(-1), s.w.reshape(-1), s.xl, s.vl, s.Rl.reshape(-1), s.wl]))
                acc, _, _ = _desired_acceleration_forest(dyn.state, i * dt, env)
                f_des, st = ctl.control(dyn.state, acc)
                fdes.append(f_des.copy()), its.append(st.iter), mds.append(st.min_env_dist)
                errs.append(np.pad(np.array(st.err_seq, float), (0, 101 - len(st.err_seq)), constant_values=np.nan))
            dyn.integrate(ll.control(dyn.state, f_des))
            refstubs.TRACE.clear()
        out[f"s{k}_f_des"], out[f"s{k}_iters"] = np.array(fdes), np.array(its, dtype=np.int16)
        out[f"s{k}_min_dist"], out[f"s{k}_states"] = np.array(mds), np.array(xs)
        out[f"s{k}_err"] = np.array(errs)[:, :8]  # the first 8 residuals of each step (C4 steps take 1-5)
        print(f"c4 loop {k}: min dist {min(mds):.3f}, iters {np.bincount(its)}", flush=True)
    np.savez_compressed(os.path.join(out_dir or OUT, "ref_c4_loop.npz"), **out)


if __name__ == "__main__":
    import time

    if len(sys.argv) > 1 and sys.argv[1] == "c4":
        t = time.time()
        gen_c4_loop()
        print(f"gen_c4_loop: {time.time() - t:.1f}s", flush=True)
        sys.exit(0)

    if len(sys.argv) > 1 and sys.argv[1] == "rp":
        gen_rp()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sm":
        gen_lowlevel_sm()
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[1] == "long":
        t = time.time()
        gen_long_closed_loop(sys.argv[2])
        print(f"gen_long_closed_loop({sys.argv[2]}): {time.time() - t:.1f}s", flush=True)
        sys.exit(0)
    for fn in (gen_params, gen_dynamics, gen_lowlevel, gen_forest, gen_env_rows, gen_qp, gen_outer_loops,
               gen_closed_loop, gen_lowlevel_sm, gen_rp):
        t = time.time()
        fn()
        print(f"{fn.__name__}: {time.time() - t:.1f}s", flush=True)
