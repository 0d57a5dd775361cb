"""Rigid-payload centralized QP (control/rp_centralized.py:9-306) and dynamics (system/rigid_payload.py:
93-130), SURVEY.md 8(f) row 3: the host build of the device code (tests/hostsim) against the reference's
own closed loop of test/control/test_rpcentralized.py:main (ref_rp.npz, 20 s at dt = 10 ms), and
the GPU path (RPCentralizedController + RPDynamics) over the same loop (-m gpu)."""

import numpy as np
import pytest

from tests import hostsim as hs
from tests._golden import load


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _xs(d, k, n=3):
    """fixture state k (xl, vl, Rl, wl) as a dat state block"""
    from distributed_aerial_transportation_amd import rigid_payload as rp

    x = d["states"][k]
    return rp.pack_rp_state(rp.RPState(x[:3], x[3:6], x[6:15].reshape(3, 3), x[15:18], project=False), n)


def test_rp_params_and_f_eq():
    from distributed_aerial_transportation_amd import rigid_payload as rp

    d = load("ref_rp.npz")
    p, _, _ = rp.rp_setup(3)
    np.testing.assert_allclose(rp.rp_equilibrium_forces(p), d["f_eq"], rtol=1e-13, atol=1e-13)
    b = rp.pack_rp_params(p)
    from distributed_aerial_transportation_amd import layout as L

    assert b[L.P["MINFZ"]] == pytest.approx(float(d["min_fz"]), rel=1e-14)
    assert b[L.P["MAXF"]] == pytest.approx(float(d["max_f"]), rel=1e-14)


def test_rp_qp_matches_reference_loop():
    """Every 20th step of the reference loop: the reduced centralized QP with the rigid-payload block
    (host build of k_cent's lane code) at the reference's state and acc_des gives its f within 1e-5."""
    from distributed_aerial_transportation_amd import rigid_payload as rp

    d = load("ref_rp.npz")
    p, _, s0 = rp.rp_setup(3)
    prm = rp.pack_rp_params(p)
    for k in range(0, d["f"].shape[0], 20):
        x = rp.pack_rp_state(s0, 3) if k == 0 else _xs(d, k - 1)
        f, status, it = hs.qp_cent(prm, 3, x, d["acc"][k], np.zeros((0, 3)), np.zeros(0))
        assert status == 0 and it <= 30
        assert _rel(f.reshape(3, 3).T, d["f"][k]) < 1e-5, k


def test_rp_dynamics_matches_reference():
    """rp_step replaying the reference's forces reproduces its states (incl. the projections)."""
    from distributed_aerial_transportation_amd import rigid_payload as rp

    d = load("ref_rp.npz")
    p, _, s0 = rp.rp_setup(3)
    prm = rp.pack_rp_params(p)
    x, cnt = rp.pack_rp_state(s0, 3), 0
    for k in range(d["f"].shape[0]):
        x, cnt = hs.rp_step(prm, 3, x, cnt, d["f"][k].T.reshape(-1), float(d["dt"]))
        if k % 100 == 99:
            assert np.max(np.abs(x - _xs(d, k))) < 1e-10, k


@pytest.mark.gpu
def test_gpu_rp_closed_loop():
    """RPCentralizedController + RPDynamics (GPU) over the reference's 20 s loop."""
    from distributed_aerial_transportation_amd import rigid_payload as rp

    d = load("ref_rp.npz")
    p, col, s0 = rp.rp_setup(3)
    ctl = rp.RPCentralizedController(p, col, s0, float(d["dt"]))
    dyn = rp.RPDynamics(p, s0, float(d["dt"]))
    rad, hgt, fr = 1.0, 1.0, 0.5
    worst_f = worst_x = 0.0
    for k in range(d["f"].shape[0]):
        t = k * float(d["dt"])
        s = dyn.state
        # test/control/test_rpcentralized.py:14-37
        x_ref = np.array([rad * np.cos(fr * t), rad * np.sin(fr * t), hgt])
        v_ref = np.array([-rad * fr * np.sin(fr * t), rad * fr * np.cos(fr * t), 0.0])
        a_ref = np.array([-rad * fr ** 2 * np.cos(fr * t), -rad * fr ** 2 * np.sin(fr * t), 0.0])
        acc = (a_ref - (s.vl - v_ref) - (s.xl - x_ref), np.array([np.sin(t), np.cos(t), np.pi / 12]))
        np.testing.assert_allclose(np.concatenate(acc), d["acc"][k], rtol=0, atol=1e-6)
        f = ctl.control(s, acc)
        worst_f = max(worst_f, _rel(f, d["f"][k]))
        assert _rel(f, d["f"][k]) < 1e-5, k
        dyn.integrate(f)
        xs = dyn.state
        worst_x = max(worst_x, float(np.max(np.abs(np.concatenate([xs.xl, xs.vl, xs.Rl.reshape(-1), xs.wl])
                                                   - d["states"][k]))))
        assert worst_x < 1e-4, k
    print(f"rigid payload 20 s: max f rel diff {worst_f:.2e}, max state diff {worst_x:.2e}")
